"""Reference-API surface on the device env (needs an MI355X).

* the reference rollout stack (MultiShipRLEnv N=1 view → NormalizedBoxEnv → ast_sac_rollout) replays
  the golden reference episodes: same observations, rewards, dones, terminals and events strings;
* the batched collector + DeviceReplayBuffer + FusedSACTrainer (HIP graph) loop runs and its
  transitions equal the single-env reference rollout under a deterministic policy.
"""
import numpy as np
import pytest
import torch

from ast_sac_amd import shipsim_abi as abi
from parity import rel_err

pytestmark = pytest.mark.gpu


def _bits_from_string(s):
    return sum(1 << i for i, e in enumerate(abi.EVENT_STRINGS) if e in s)


class _TableAgent:
    def __init__(self, actions):
        self.actions = list(actions)
        self.i = 0

    def reset(self):
        self.i = 0

    def get_action(self, o):
        a = np.array([self.actions[self.i]], dtype=np.float32)
        self.i += 1
        return a, {}


@pytest.mark.parametrize("collav", ["none", "sbmpc", "simple"])
def test_reference_rollout_stack_replays_golden(golden, collav):
    from ast_sac_amd.run.env_setup import prepare_multiship_rl_env
    from ast_sac_amd.rl_env.ship_in_transit.env import default_args
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import NormalizedBoxEnv
    from ast_sac_amd.ast_sac.samplers.data_collector.rollout_functions import ast_sac_rollout
    g = golden("rl_env_detailed")
    env, _ = prepare_multiship_rl_env(default_args(collav_mode=collav))
    nenv = NormalizedBoxEnv(env, reward_scale=1.0)
    for ep in range(int(g[f"{collav}_n_episodes"])):
        p = f"{collav}_ep{ep}"
        path = ast_sac_rollout(nenv, _TableAgent(g[p + "_a_norm"]), max_path_length=9)
        n = len(g[p + "_reward"])
        assert len(path["actions"]) == n, p
        np.testing.assert_array_equal(path["observations"][0], g[p + "_o0"])
        assert float(rel_err(path["next_observations"], g[p + "_obs"]).max()) <= 1e-5, p
        np.testing.assert_allclose(path["rewards"][:, 0], g[p + "_reward"], rtol=1e-5, atol=1e-8)
        np.testing.assert_array_equal(path["dones"][:, 0], g[p + "_done"].astype(bool))
        np.testing.assert_array_equal(path["terminals"][:, 0], g[p + "_terminal"].astype(bool))
        got_bits = [_bits_from_string(i["events"]) for i in path["env_infos"]]
        np.testing.assert_array_equal(got_bits, g[p + "_bits"], err_msg=p)
        assert env.sampling_count == n or path["dones"][-1, 0]
    env.close()


def test_batched_collector_matches_single_env_rollout():
    """Deterministic policy: every device env runs the same episode as the N=1 reference rollout."""
    from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, MultiShipRLEnv, default_args
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import NormalizedBoxEnv, BatchedNormalizedBoxEnv
    from ast_sac_amd.ast_sac.samplers.data_collector.rollout_functions import ast_sac_rollout
    from ast_sac_amd.ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac_amd.ast_sac.torch.sac.policies.base import MakeDeterministic
    from ast_sac_amd.ast_sac.torch.utils import pytorch_util as ptu
    ptu.set_gpu_mode(True)  # as run/ast-sac_runner.py does: numpy observations go to the HIP device
    try:
        _collector_vs_single(BatchedMultiShipRLEnv, MultiShipRLEnv, default_args, NormalizedBoxEnv,
                             BatchedNormalizedBoxEnv, ast_sac_rollout, BatchedPathCollector, DeviceReplayBuffer,
                             TanhGaussianPolicy, MakeDeterministic)
    finally:
        ptu.set_gpu_mode(False)


def _collector_vs_single(BatchedMultiShipRLEnv, MultiShipRLEnv, default_args, NormalizedBoxEnv,
                         BatchedNormalizedBoxEnv, ast_sac_rollout, BatchedPathCollector, DeviceReplayBuffer,
                         TanhGaussianPolicy, MakeDeterministic):
    torch.manual_seed(3)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[64, 64], init_w=0.5).cuda()
    det = MakeDeterministic(pol)
    args = default_args(collav_mode="none")
    single = NormalizedBoxEnv(MultiShipRLEnv(args), reward_scale=0.75)
    ref = ast_sac_rollout(single, det, max_path_length=9)
    n_dec = len(ref["actions"])

    N = 64
    benv = BatchedNormalizedBoxEnv(BatchedMultiShipRLEnv(args, N), reward_scale=0.75)
    coll = BatchedPathCollector(benv, det, max_path_length=9, max_ticks=48, deterministic=True)
    rb = DeviceReplayBuffer(N * n_dec, 8, 1, "cuda")
    got = 0
    while got < N * n_dec:
        _, k = coll.step(rb)
        got += int(k)
    assert got == N * n_dec  # every env finished the same n_dec decisions in the same pass
    obs = rb._observations.cpu().numpy().reshape(n_dec, N, 8)
    act = rb._actions.cpu().numpy().reshape(n_dec, N)
    rew = rb._rewards.cpu().numpy().reshape(n_dec, N)
    nob = rb._next_obs.cpu().numpy().reshape(n_dec, N, 8)
    term = rb._terminals.cpu().numpy().reshape(n_dec, N)
    for d in range(n_dec):
        assert float(rel_err(obs[d], np.repeat(ref["observations"][d][None], N, 0)).max()) <= 1e-5
        assert float(rel_err(nob[d], np.repeat(ref["next_observations"][d][None], N, 0)).max()) <= 1e-5
        np.testing.assert_allclose(act[d], ref["actions"][d, 0], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(rew[d], ref["rewards"][d, 0], rtol=1e-5, atol=1e-6)
        np.testing.assert_array_equal(term[d], float(ref["terminals"][d, 0]))
    # collect(record_paths): the ended episodes are the reference path, env by env
    coll2 = BatchedPathCollector(BatchedNormalizedBoxEnv(BatchedMultiShipRLEnv(args, N), reward_scale=0.75), det,
                                 max_path_length=9, max_ticks=48, deterministic=True)
    coll2.collect(N * n_dec, None, record_paths=True)
    paths = list(coll2.get_epoch_paths())
    assert len(paths) == N
    for p in paths:
        np.testing.assert_allclose(p["rewards"], ref["rewards"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(p["actions"], ref["actions"], rtol=1e-5, atol=1e-6)
        assert [i["terminal"] for i in p["env_infos"]] == [bool(i["terminal"]) for i in ref["env_infos"]]


def test_device_training_loop_runs():
    """Collector → DeviceReplayBuffer → graph-captured FusedSACTrainer, a few hundred grad steps."""
    from ast_sac_amd.run.ast_sac_runner import parse_cli_args, make_variant, experiment_device
    args = parse_cli_args(["--n_envs", "512", "--eval_envs", "64", "--num_epochs", "2",
                           "--min_num_steps_before_training", "1024", "--num_expl_steps_per_train_loop", "256",
                           "--num_trains_per_train_loop", "120", "--num_eval_steps_per_epoch", "64",
                           "--collav_mode", "none", "--do_logging", "false"])
    algo = experiment_device(make_variant(args), args, torch.device("cuda", 0))
    algo.train()  # logs to a throwaway dir (do_logging false): exercises _log_stats with epoch paths
    d = algo.trainer.get_diagnostics()
    assert np.isfinite(d["QF1 Loss"]) and np.isfinite(d["Policy Loss"])
    assert algo.replay_buffer.num_steps_can_sample() >= 1024 + 2 * 256
    # num_trains / num_expl grad steps per collected exploration decision (the reference's ratio)
    n_expl = algo.num_loop_expl_steps_total
    assert algo.num_train_steps_total == algo.trainer._n_train_steps_total
    assert abs(algo.num_train_steps_total - n_expl * 120 / 256) < 1 + 1e-9  # --num_trains_per_train_loop 120
    assert n_expl >= 2 * 256


def test_shared_eval_env_carries_sbmpc_memory():
    """Q10 + Q7 on the device runner's default shape: evaluation and exploration wrap ONE batched env
    (run/ast-sac_runner.py:113-114). The evaluation collector's episodes advance those envs; when the
    exploration collector takes them back it resets every env (each reference path starts with reset())
    and the reset leaves the SBMPC memory P_ca_last / Chi_ca_last as the evaluation episodes left it
    (sbmpc.py:143-145 is never reset, env.py:238-295): the same envs, the same carried state."""
    from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, default_args
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import BatchedNormalizedBoxEnv
    from ast_sac_amd.ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector
    from ast_sac_amd.ast_sac.torch.sac.policies.base import MakeDeterministic
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    N = 64
    env = BatchedMultiShipRLEnv(default_args(collav_mode="sbmpc"), N)
    expl_env, eval_env = BatchedNormalizedBoxEnv(env, 0.75), BatchedNormalizedBoxEnv(env, 0.75)
    torch.manual_seed(0)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[32, 32]).cuda()
    expl = BatchedPathCollector(expl_env, pol, max_path_length=9, max_ticks=128)
    ev = BatchedPathCollector(eval_env, MakeDeterministic(pol), max_path_length=9, max_ticks=128, deterministic=True)
    expl.collect(32, None)
    ev.collect(1000, None, record_paths=True)  # > 12 passes of 128 ticks: episodes (~1,400 ticks) end
    assert len(ev.get_epoch_paths()) > 0
    # distinctive SBMPC memory in the shared envs, as an evaluation episode in an encounter leaves it
    p = torch.linspace(0.4, 1.0, N, dtype=torch.float64, device="cuda")
    c = torch.linspace(-0.5, 0.5, N, dtype=torch.float64, device="cuda")
    env.sim.set(abi.E_SBMPC_P_LAST, p)
    env.sim.set(abi.E_SBMPC_CHI_LAST, c)
    expl._take_over()  # what expl.collect does first: reset every env, restart every episode
    torch.cuda.synchronize()
    assert int(expl._path_len.max()) == 0 and bool(expl._awaiting.all())
    assert torch.equal(env.sim.get(abi.E_SBMPC_P_LAST), p) and torch.equal(env.sim.get(abi.E_SBMPC_CHI_LAST), c)
    assert int(env.sim.get(abi.E_SAMPLING_COUNT).max()) == 0  # everything else restarted
    got = expl.collect(32, None)
    assert got >= 32
