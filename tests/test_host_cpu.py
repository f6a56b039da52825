"""Host-side pieces that need no GPU: action normalisation, runner defaults, logger, replay buffer."""
import csv
import os

import numpy as np
import torch

from ast_sac_amd import shipsim_abi as abi


def test_batched_action_mapping_is_bitwise_the_reference_float32_rule():
    """BatchedNormalizedBoxEnv's torch mapping == NormalizedBoxEnv's numpy float32 rule, bit for bit."""
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import denormalize_action
    lb = np.array([-np.deg2rad(30)], np.float32)
    ub = np.array([np.deg2rad(30)], np.float32)
    a = np.random.default_rng(0).uniform(-1.3, 1.3, (100000, 1)).astype(np.float32)
    a[:4, 0] = [-1, 1, 0, np.float32(0.999999)]
    ref = np.clip(lb + (a + 1.0) * 0.5 * (ub - lb), lb, ub)
    got = denormalize_action(torch.from_numpy(a), float(lb[0]), float(ub[0])).numpy()
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(abi.normalized_to_scoping(a[:, 0]), ref[:, 0])


def test_runner_defaults_are_the_reference_defaults():
    from ast_sac_amd.run.ast_sac_runner import parse_cli_args, make_variant
    a = parse_cli_args([])
    v = make_variant(a)
    assert (a.max_sampling_frequency, a.time_step, a.radius_of_acceptance, a.lookahead_distance, a.collav_mode) == \
        (9, 4, 300, 1000, "sbmpc")
    assert v["layer_size"] == 256 and v["replay_buffer_size"] == 300000
    assert v["algorithm_kwargs"] == dict(num_epochs=500, num_eval_steps_per_epoch=180, num_trains_per_train_loop=240,
                                         num_expl_steps_per_train_loop=256, min_num_steps_before_training=8192,
                                         max_path_length=9, batch_size=256)
    assert v["trainer_kwargs"] == dict(discount=0.965, soft_target_tau=1e-3, target_update_period=1, policy_lr=8e-5,
                                       qf_lr=8e-5, reward_scale=0.75, use_automatic_entropy_tuning=True,
                                       action_reg_coeff=0.01, clip_val=100)


def test_logger_progress_csv_keeps_first_dump_columns(tmp_path):
    from ast_sac_amd.ast_sac.core.logging import Logger
    lg = Logger()
    lg.quiet = True
    lg.add_tabular_output(str(tmp_path / "progress.csv"))
    lg.record_dict({"b": 1, "a": 2})
    lg.dump_tabular(with_prefix=False, with_timestamp=False)
    lg.record_dict({"a": 3, "b": 4, "c": 5})
    lg.dump_tabular(with_prefix=False, with_timestamp=False)
    rows = list(csv.reader(open(tmp_path / "progress.csv")))
    assert rows == [["a", "b"], ["2", "1"], ["3", "4"]]
    lg.set_snapshot_dir(str(tmp_path))
    lg.set_snapshot_mode("last")
    lg.save_itr_params(0, {"x": torch.zeros(2)})
    assert os.path.exists(tmp_path / "params.pkl")


def test_reference_algorithm_loop_on_a_cpu_stub_env():
    """TorchBatchRLAlgorithm + MdpPathCollector + EnvReplayBuffer + SACTrainer wired like the runner,
    on a tiny stand-in env with the reference env API (the loop logic, not the ship physics)."""
    from ast_sac_amd.spaces import Box
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import NormalizedBoxEnv
    from ast_sac_amd.ast_sac.data_management.replay_buffer import EnvReplayBuffer
    from ast_sac_amd.ast_sac.samplers.data_collector.path_collector import MdpPathCollector
    from ast_sac_amd.ast_sac.samplers.data_collector.rollout_functions import ast_sac_rollout
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac_amd.ast_sac.torch.sac.policies.base import MakeDeterministic
    from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac_amd.ast_sac.torch.sac.sac import SACTrainer
    from ast_sac_amd.ast_sac.torch.core.torch_rl_algorithm import TorchBatchRLAlgorithm
    from ast_sac_amd.ast_sac.core.logging import logger

    class Stub:
        observation_space = Box(low=np.zeros(8, np.float32), high=np.ones(8, np.float32), dtype=np.float32)
        action_space = Box(low=np.array([-0.5], np.float32), high=np.array([0.5], np.float32), dtype=np.float32)

        def reset(self):
            self.t = 0
            return np.zeros(8, np.float32)

        def step(self, a):
            self.t += 1
            assert -0.5 <= float(a[0]) <= 0.5
            done = self.t >= 4
            return (np.full(8, self.t, np.float32), float(a[0]), done,
                    {"events": "", "terminal": done, "test_ship_stop": False, "obs_ship_stop": False})

    torch.manual_seed(0)
    env = NormalizedBoxEnv(Stub(), reward_scale=0.75)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[16, 16])
    qs = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[16, 16]) for _ in range(4)]
    tr = SACTrainer(env=env, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2], target_qf2=qs[3])
    rb = EnvReplayBuffer(100, env)
    algo = TorchBatchRLAlgorithm(trainer=tr, exploration_env=env, evaluation_env=env,
                                 exploration_data_collector=MdpPathCollector(env, pol, rollout_fn=ast_sac_rollout),
                                 evaluation_data_collector=MdpPathCollector(env, MakeDeterministic(pol),
                                                                            rollout_fn=ast_sac_rollout),
                                 replay_buffer=rb, batch_size=8, max_path_length=9, num_epochs=2,
                                 num_eval_steps_per_epoch=6, num_expl_steps_per_train_loop=5,
                                 num_trains_per_train_loop=3, min_num_steps_before_training=10)
    logger.quiet = True
    algo.train()
    logger.quiet = False
    # 10 initial (3 whole episodes of 4 = 12 decisions, last one cut to the remaining budget) + 2 × 5
    assert rb.num_steps_can_sample() == 10 + 2 * 5
    assert tr._n_train_steps_total == 6
    assert rb._terminals[:4, 0].tolist() == [0, 0, 0, 1]
