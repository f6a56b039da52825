"""Trained-policy replay (run/ast-sac_run_trained_policy.py:24-65), SURVEY.md §8(f) f3.

Loads a snapshot written by this package's logger (`logger.save_itr_params`, params.pkl / itr_*.pkl:
torch.save of the snapshot dict), takes 'evaluation/policy' (MakeDeterministic(TanhGaussianPolicy) in
the runner's snapshot), and replays one episode with ast_sac_rollout on the device env with
trajectory recording on, exposing the same attributes the reference's plotting/animation code reads:
ts_results_df / os_results_df (simulation_results DataFrames), waypoint_sampling_times, test / obs
(ShipAssetView), env.wrapped_env.reward_tracker.

    python -m ast_sac_amd.run.ast_sac_run_trained_policy <params.pkl> [--collav_mode sbmpc]
Plotting and animation (the reference's do_plot / animate, matplotlib) are not part of this build.
"""
import argparse

import numpy as np
import torch

from ..ast_sac.env_wrapper.normalized_box_env import NormalizedBoxEnv
from ..ast_sac.samplers.data_collector.rollout_functions import ast_sac_rollout
from ..ast_sac.torch.utils import pytorch_util as ptu
from ..rl_env.ship_in_transit.env import default_args
from .env_setup import prepare_multiship_rl_env


def load_snapshot(filename, device=None):
    """Snapshots are produced by this package's own logger (not third-party files): they hold the
    policy modules themselves, as the reference's params.pkl does (logging.py:314-335)."""
    return torch.load(filename, map_location=device, weights_only=False)


class SimulatePolicyEnvSetup:
    def __init__(self, filename, max_path_length=np.inf, gpu_mode=True, env_args=None, policy=None):
        if gpu_mode:
            ptu.set_gpu_mode(True)
        self.data = load_snapshot(filename, ptu.device) if policy is None else {"evaluation/policy": policy}
        self.max_path_length = max_path_length
        self.policy = self.data["evaluation/policy"]
        self.env_args = env_args if env_args is not None else default_args()
        env, _ = prepare_multiship_rl_env(self.env_args, record_trajectory=True)
        self.env = NormalizedBoxEnv(env)
        self.test = env.test
        self.obs = env.obs

    def simulate_policy(self):
        import pandas as pd
        path = ast_sac_rollout(self.env, self.policy, max_path_length=self.max_path_length)
        w = self.env.wrapped_env
        self.ts_results_df = pd.DataFrame().from_dict(w.test.ship_model.simulation_results)
        self.os_results_df = pd.DataFrame().from_dict(w.obs.ship_model.simulation_results)
        self.waypoint_sampling_times = w.waypoint_sampling_times
        return path


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("snapshot")
    p.add_argument("--collav_mode", default="sbmpc")
    p.add_argument("--cpu", action="store_true", help="policy on the CPU (the env always runs on the GPU)")
    a = p.parse_args(argv)
    setup = SimulatePolicyEnvSetup(a.snapshot, np.inf, not a.cpu, default_args(collav_mode=a.collav_mode))
    path = setup.simulate_policy()
    for i in range(len(path["actions"])):
        print("STEP", i + 1)
        print("Observation      :", path["observations"][i])
        print("Action           :", path["actions"][i])
        print("Scoping Angle    :", np.rad2deg(setup.env.wrapped_env.do_denormalize_action(path["actions"][i])))
        print("Next observation :", path["next_observations"][i])
        print("Rewards          :", path["rewards"][i])
        print("Terminal         :", path["terminals"][i])
        print("Done             :", path["dones"][i])
        print("------------------")
    print("Sum Reward       :", np.sum(path["rewards"]))
    print(setup.ts_results_df.tail(3).to_string())
    return setup, path


if __name__ == "__main__":
    main()
