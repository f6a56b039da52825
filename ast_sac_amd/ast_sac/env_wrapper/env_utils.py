"""Space and env helpers of ast_sac/env_wrapper/env_utils.py (get_dim :13-23, mode :26-30): the replay buffer sizes
its rows with get_dim (env_replay_buffer.py:4,24-27), the algorithm loops switch env modes with mode."""
from ...spaces import Discrete


def get_dim(space):
    """Flat size of a space: a Box's element count (gymnasium's Box or the stand-in of ast_sac_amd.spaces, both carry
    `shape`), a Discrete's n, a Tuple's sum over its spaces, else a `flat_dim` attribute (env_utils.py:13-23)."""
    if hasattr(space, "low") and hasattr(space, "shape"):
        size = 1
        for d in space.shape:
            size *= int(d)
        return size
    if isinstance(space, Discrete) or (hasattr(space, "n") and not hasattr(space, "spaces")):
        return space.n
    if hasattr(space, "spaces"):
        return sum(get_dim(s) for s in space.spaces)
    if hasattr(space, "flat_dim"):
        return space.flat_dim
    raise TypeError("Unknown space: {}".format(space))


def mode(env, mode_type):
    """Call env.<mode_type>() when the env has it (env_utils.py:26-30)."""
    try:
        getattr(env, mode_type)()
    except AttributeError:
        pass
