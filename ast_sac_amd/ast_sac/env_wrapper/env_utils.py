"""ast_sac/env_wrapper/env_utils.py"""
from ...spaces import get_dim  # noqa: F401
