"""run/env_setup.py:prepare_multiship_rl_env drop-in: the scenario of record on the device env."""
from .. import shipsim_abi as abi
from ..rl_env.ship_in_transit.env import MultiShipRLEnv, BatchedMultiShipRLEnv, config_from_args


def prepare_multiship_rl_env(args, device=None, machinery="detailed", n_envs=None, machinery_mode="PTI",
                             record_trajectory=False):
    """Returns (env, assets) like the reference; `assets` is the shipsim config (both ships).
    With n_envs the batched device env is returned instead of the single-env view.
    machinery_mode selects the MachineryModes([...]) entry of env_setup.py:62-84 (the runner: PTI);
    record_trajectory keeps the reference's simulation_results / RewardTracker surface (N = 1 view)."""
    cfg = config_from_args(args, machinery)
    abi.set_machinery_mode(cfg, machinery_mode)
    if n_envs is None:
        env = MultiShipRLEnv(args, device=device, machinery=machinery, cfg=cfg, record_trajectory=record_trajectory)
    else:
        env = BatchedMultiShipRLEnv(args, n_envs, device=device, machinery=machinery, cfg=cfg)
    return env, cfg
