"""run/env_setup.py:prepare_multiship_rl_env drop-in: the scenario of record on the device env."""
from ..rl_env.ship_in_transit.env import MultiShipRLEnv, BatchedMultiShipRLEnv, config_from_args


def prepare_multiship_rl_env(args, device=None, machinery="detailed", n_envs=None):
    """Returns (env, assets) like the reference; `assets` is the shipsim config (both ships).
    With n_envs the batched device env is returned instead of the single-env view."""
    cfg = config_from_args(args, machinery)
    if n_envs is None:
        env = MultiShipRLEnv(args, device=device, machinery=machinery, cfg=cfg)
    else:
        env = BatchedMultiShipRLEnv(args, n_envs, device=device, machinery=machinery, cfg=cfg)
    return env, cfg
