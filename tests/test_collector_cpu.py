"""BatchedPathCollector host logic on a scripted CPU env (no GPU): the policy runs only on the envs
that wait for a decision, every decision's transition reaches the buffer with the action chosen at its
start, and the episodes that end become reference-shaped epoch paths (MdpPathCollector.get_epoch_paths,
path_collector.py:77-78) from which eval_util.get_generic_path_information builds the progress.csv
columns (eval_util.py:10-60)."""
from collections import OrderedDict

import numpy as np
import torch

from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.ast_sac.core import eval_util
from ast_sac_amd.ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector


class _ScriptedEnv:
    """Env i takes 1 + i % 3 passes per decision and ends (done) after 2 + i % 4 decisions; reward of a
    decision = 10·i + decision index; observation = (i, decision index, episode, 0...)."""

    def __init__(self, n):
        self.n_envs, self.device, self._reward_scale = n, torch.device("cpu"), 0.5
        self.dur = 1 + torch.arange(n) % 3
        self.eplen = 2 + torch.arange(n) % 4
        self.left = self.dur.clone()
        self.dec = torch.zeros(n, dtype=torch.int64)
        self.ep = torch.zeros(n, dtype=torch.int64)
        self.actions_seen = [[] for _ in range(n)]
        self.ready_counts = []

    def _obs(self):
        o = torch.zeros((self.n_envs, 8))
        o[:, 0] = torch.arange(self.n_envs)
        o[:, 1] = self.dec.float()
        o[:, 2] = self.ep.float()
        return o

    def reset(self, mask=None, obs_out=None):
        m = torch.ones(self.n_envs, dtype=torch.bool) if mask is None else mask.bool()
        self.dec[m] = 0
        self.ep[m] += 0 if mask is None else 1
        self.left[m] = self.dur[m]
        o = self._obs()
        if obs_out is not None:
            obs_out.copy_(o)
        return o

    def step_async(self, act, max_ticks=64, out=None):
        self.left -= 1
        ready = self.left == 0
        self.ready_counts.append(int(ready.sum()))
        for i in torch.nonzero(ready).flatten().tolist():
            self.actions_seen[i].append(float(act[i, 0]))
        rew = (10 * torch.arange(self.n_envs) + self.dec).double()
        self.dec += ready.long()
        done = ready & (self.dec >= self.eplen)
        self.left = torch.where(ready, self.dur, self.left)
        ev = torch.where(done, torch.full_like(self.dec, abi.EV_TERMINAL | abi.EV_TEST_STOP), torch.zeros_like(self.dec))
        out.update(obs=self._obs(), reward=rew, done=done.to(torch.uint8), events=ev.to(torch.int32),
                   ticks=torch.full((self.n_envs,), 5, dtype=torch.int32), ready=ready.to(torch.uint8))
        return out


class _Dist:
    def __init__(self, a):
        self.a = a

    def mle_estimate(self):
        return self.a


class _Policy:
    def __init__(self):
        self.batch_sizes = []

    def __call__(self, obs):
        self.batch_sizes.append(obs.shape[0])
        return _Dist(torch.tanh(0.01 * obs[:, :1] + 0.1 * obs[:, 1:2] - 0.05 * obs[:, 2:3]))


class _Buffer:
    def __init__(self):
        self.rows = []

    def add_batch(self, obs, act, rew, nobs, term, mask):
        for i in torch.nonzero(mask).flatten().tolist():
            self.rows.append((obs[i].clone(), float(act[i, 0]), float(rew[i, 0]), float(term[i, 0])))


def test_policy_only_on_awaiting_envs_and_paths():
    N = 24
    env, pol, rb = _ScriptedEnv(N), _Policy(), _Buffer()
    coll = BatchedPathCollector(env, pol, max_path_length=9, deterministic=True)
    got = coll.collect(200, rb, record_paths=True)
    assert got >= 200 and got == len(rb.rows)
    # first pass: all N wait; afterwards exactly the envs that completed a decision in the pass before
    assert pol.batch_sizes[0] == N
    assert pol.batch_sizes[1:] == env.ready_counts[:-1]
    assert sum(pol.batch_sizes) < N * len(pol.batch_sizes) * 3 // 4
    # every transition: the action is the policy's at the decision's observation
    for obs, a, r, t in rb.rows:
        i, d, ep = (int(x) for x in obs[:3])
        assert abs(a - float(torch.tanh(torch.tensor(0.01 * i + 0.1 * d - 0.05 * ep)))) < 1e-6
        assert r == 0.5 * (10 * i + d)
        assert t == float(d + 1 == int(env.eplen[i]))
    # executed actions == buffered actions, env by env
    per_env = [[a for (o, a, _, _) in rb.rows if int(o[0]) == i] for i in range(N)]
    assert per_env == env.actions_seen
    paths = list(coll.get_epoch_paths())
    assert paths and all(p["rewards"].shape == p["actions"].shape == (len(p["env_infos"]), 1) for p in paths)
    for p in paths:
        i = int(round((p["rewards"][0, 0] / 0.5) / 10))
        L = int(env.eplen[i])
        np.testing.assert_array_equal(p["rewards"][:, 0], 0.5 * (10 * i + np.arange(L)))
        assert p["env_infos"][-1]["terminal"] and p["env_infos"][-1]["test_ship_stop"]
        assert not any(x["terminal"] for x in p["env_infos"][:-1])
    st = eval_util.get_generic_path_information(paths)
    for k in ("Rewards Mean", "Returns Mean", "Actions Mean", "Num Paths", "Average Returns"):
        assert k in st
    assert st["Num Paths"] == len(paths)
    d = coll.get_diagnostics()
    assert isinstance(d, OrderedDict) and d["num steps total"] == got and "path length Mean" in d
    coll.end_epoch(0)
    assert len(coll.get_epoch_paths()) == 0


def test_max_num_epoch_paths_saved():
    env, pol = _ScriptedEnv(8), _Policy()
    coll = BatchedPathCollector(env, pol, max_path_length=9, deterministic=True, max_num_epoch_paths_saved=3)
    coll.collect(100, None, record_paths=True)
    assert len(coll.get_epoch_paths()) == 3


def test_path_cut_at_max_path_length():
    env, pol = _ScriptedEnv(8), _Policy()
    coll = BatchedPathCollector(env, pol, max_path_length=2, deterministic=True)
    coll.collect(60, None, record_paths=True)
    assert {len(p["actions"]) for p in coll.get_epoch_paths()} == {2}


class _Trainer:
    networks = []

    def __init__(self):
        self.n = 0

    def train_from_buffer(self, rb, k):
        self.n += k

    def get_diagnostics(self):
        return OrderedDict([("QF1 Loss", 1.0), ("num train calls", self.n)])

    def end_epoch(self, epoch):
        pass

    def get_snapshot(self):
        return {}


class _RB(_Buffer):
    def get_diagnostics(self):
        return OrderedDict(size=len(self.rows))

    def end_epoch(self, epoch):
        pass

    def get_snapshot(self):
        return {}


def test_device_algorithm_progress_header_equals_reference(tmp_path):
    """f2: the progress.csv DeviceBatchRLAlgorithm writes has exactly the header the reference's own
    TorchBatchRLAlgorithm writes (tests/golden/progress_header.json, generated by running it:
    gen_golden.py progress): the same column names in the same (sorted, logging.py:285-305) order,
    including the time/<stamp> (s) columns of every gtimer stamp (sac training included), the
    replay-buffer / trainer / expl / eval statistics and no build-only columns. Here with the real
    trainer (FusedSACTrainer, torch backend) and DeviceReplayBuffer on the CPU, scripted envs."""
    import csv
    import json
    import os
    from ast_sac_amd.ast_sac.core.device_rl_algorithm import DeviceBatchRLAlgorithm
    from ast_sac_amd.ast_sac.core.logging import logger
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    ref = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "progress_header.json")))

    class _E:
        class action_space:
            shape = (1,)

    torch.manual_seed(0)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[16, 16])
    qs = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[16, 16]) for _ in range(4)]
    tr = FusedSACTrainer(env=_E, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2], target_qf2=qs[3],
                         discount=0.965, reward_scale=0.75, policy_lr=8e-5, qf_lr=8e-5, soft_target_tau=1e-3,
                         action_reg_coeff=0.01, clip_val=100.0, batch_size=8, use_graph=False, backend="torch")
    env_x, env_e = _ScriptedEnv(16), _ScriptedEnv(8)
    cx = BatchedPathCollector(env_x, _Policy(), max_path_length=9, deterministic=True)
    ce = BatchedPathCollector(env_e, _Policy(), max_path_length=9, deterministic=True)
    algo = DeviceBatchRLAlgorithm(tr, env_x, env_e, cx, ce, DeviceReplayBuffer(1000, 8, 1, "cpu"), batch_size=8,
                                  max_path_length=9, num_epochs=2, num_eval_steps_per_epoch=20,
                                  num_expl_steps_per_train_loop=30, num_trains_per_train_loop=5,
                                  min_num_steps_before_training=40)
    f = str(tmp_path / "progress.csv")
    logger.add_tabular_output(f)
    try:
        algo.train()
    finally:
        logger.remove_tabular_output(f)
    with open(f) as fh:
        rows = list(csv.reader(fh))
    assert len(rows) - 1 == ref["n_rows"] == 2
    header = rows[0]
    missing, extra = sorted(set(ref["columns"]) - set(header)), sorted(set(header) - set(ref["columns"]))
    assert not missing and not extra, (missing, extra)
    assert header == ref["columns"]
    assert rows[2][header.index("Epoch")] == "1"


def test_update_ratio_follows_collected_decisions():
    """match_update_ratio: grad steps = collected x num_trains / num_expl (fraction carried); off: as set."""
    from ast_sac_amd.ast_sac.core.device_rl_algorithm import DeviceBatchRLAlgorithm
    for match in (True, False):
        env_x, env_e = _ScriptedEnv(40), _ScriptedEnv(8)
        tr = _Trainer()
        algo = DeviceBatchRLAlgorithm(tr, env_x, env_e, BatchedPathCollector(env_x, _Policy(), deterministic=True),
                                      BatchedPathCollector(env_e, _Policy(), deterministic=True), _RB(),
                                      batch_size=32, max_path_length=9, num_epochs=3, num_eval_steps_per_epoch=0,
                                      num_expl_steps_per_train_loop=7, num_trains_per_train_loop=5,
                                      num_train_loops_per_epoch=2, min_num_steps_before_training=0,
                                      match_update_ratio=match)
        algo.log_stats = False
        algo.train()
        n = algo.num_loop_expl_steps_total
        assert n > 6 * 7  # the 40-env passes overshoot 7 decisions per loop
        if match:
            assert tr.n == algo.num_train_steps_total == int(n * 5 / 7 + 1e-9)
        else:
            assert tr.n == 6 * 5


def test_trace_records_each_decision():
    """trace(): every decision of the traced envs in order, ticks summed over the slices it took,
    episode / decision counters following the collector's episode ends."""
    env, pol = _ScriptedEnv(12), _Policy()
    coll = BatchedPathCollector(env, pol, max_path_length=9, deterministic=True)
    idx = [0, 5, 7, 11]
    coll.trace(idx)
    coll.collect(150, None)
    for j, i in enumerate(idx):
        log = coll.trace_log()[j]
        assert [d["action"] for d in log] == [np.float32(a) for a in env.actions_seen[i]]
        assert all(d["ticks"] == 5 * int(env.dur[i]) for d in log)  # 5 ticks per pass, dur passes
        L = int(env.eplen[i])
        for k, d in enumerate(log):
            assert (d["episode"], d["decision"]) == (k // L, k % L)
            assert d["done"] == (k % L == L - 1) and d["reward"] == 10 * i + k % L
            assert bool(d["events"] & abi.EV_TERMINAL) == d["done"]


def test_shared_env_eval_then_expl_resets_and_restarts_episodes():
    """Q10 (run/ast-sac_runner.py:113-114): an evaluation collector over the exploration collector's env
    takes it over — every env is reset and every episode starts afresh (the reference begins each path
    with env.reset()) — and the exploration collector takes it back the same way; a collector that
    already drives the env does not reset it again."""
    env = _ScriptedEnv(12)
    calls = []
    real_reset = env.reset

    def reset(mask=None, obs_out=None):
        calls.append(None if mask is None else int(mask.sum()))
        return real_reset(mask, obs_out)

    env.reset = reset
    expl = BatchedPathCollector(env, _Policy(), max_path_length=9, deterministic=True)
    ev = BatchedPathCollector(env, _Policy(), max_path_length=9, deterministic=True)
    calls.clear()
    ev.collect(10, None, record_paths=True)        # the env was last set up by ev's constructor: no takeover
    assert None not in calls
    expl.collect(10, _Buffer())                     # takes over: one full reset, then only masked resets
    assert calls.count(None) == 1
    n_full = calls.count(None)
    assert int(expl._path_len.max()) <= 9
    expl.collect(10, _Buffer())                     # still the owner: no full reset
    assert calls.count(None) == n_full
    ev.collect(10, None, record_paths=True)
    assert calls.count(None) == n_full + 1
    # after the takeover the eval collector's episodes all restarted at decision 0
    paths = ev.get_epoch_paths()
    assert all(len(p["actions"]) >= 1 for p in paths)


class _PolicySim:
    """Stands in for ShipSim.run_policy (shipsim_run_policy's contract, include/shipsim.h): env i
    completes (i + call) % 4 decisions per call (at most the room left in its log), decision d of an
    episode returns obs (i, d + 1, ep, ...), the episode ends by done after 2 + i % 5 decisions or by the
    n_dec cut, env 3's second decision ends non-finite (EV_NONFINITE, done)."""
    n_ships = 2

    def __init__(self, n):
        self.n, self.calls = n, 0
        self.obs = torch.zeros((n, 8), dtype=torch.float64)
        self.obs[:, 0] = torch.arange(n)
        self.cfg = abi.Config()
        self.cfg.normalize_action = 0
        self.cfg.action_low, self.cfg.action_high = float(np.float32(-np.deg2rad(30))), float(np.float32(np.deg2rad(30)))

    def synchronize(self):
        pass

    def run_policy(self, weights, max_ticks, n_dec, ep, dec, deterministic=False, seed=0, counter=None, out=None,
                   log=None, log_len=None):
        cap = log.shape[1]
        for i in range(self.n):
            k = min((i + self.calls) % 4, cap - int(log_len[i]))
            for _ in range(k):
                d, e = int(dec[i]), int(ep[i])
                nonfinite = i == 3 and d == 1
                done = nonfinite or d + 1 >= 2 + i % 5
                rec = log[i, int(log_len[i])]
                rec.zero_()
                rec[abi.DL_OBS0:abi.DL_OBS0 + 8] = self.obs[i]
                rec[abi.DL_ACTION] = float(np.float32(np.tanh(0.01 * i + 0.1 * d - 0.05 * e)))
                rec[abi.DL_REWARD] = 10.0 * i + d
                ev = (abi.EV_TERMINAL | abi.EV_TEST_STOP) if done else 0
                rec[abi.DL_EVENTS] = ev | (abi.EV_NONFINITE | abi.EV_TERMINAL if nonfinite else 0)
                rec[abi.DL_DONE] = float(done)
                rec[abi.DL_EPISODE], rec[abi.DL_DECISION], rec[abi.DL_TICKS] = e, d, 37
                nxt = torch.tensor([i, d + 1, e, 0, 0, 0, 0, 0], dtype=torch.float64)
                rec[abi.DL_OBS:abi.DL_OBS + 8] = nxt
                log_len[i] += 1
                if done or d + 1 >= n_dec:
                    ep[i] += 1
                    dec[i] = 0
                    self.obs[i] = torch.tensor([i, 0, e + 1, 0, 0, 0, 0, 0], dtype=torch.float64)
                else:
                    dec[i] += 1
                    self.obs[i] = nxt
            out["ticks"][i] = 37 * k
            out["decisions"][i] = k
        self.calls += 1
        return out


class _PolicyEnv(_ScriptedEnv):
    def __init__(self, n):
        super().__init__(n)
        self.sim = _PolicySim(n)
        self._lb, self._ub = self.sim.cfg.action_low, self.sim.cfg.action_high


class _DevicePolicy:
    deterministic, seed = True, 5

    def __init__(self):
        self.counter = torch.zeros(1, dtype=torch.int64)

    def reserve(self, n):
        pass

    def weights(self):
        return (0, 0, 8, 64)


def test_fused_pass_rows_and_paths_follow_the_decision_log():
    """Fused collection (the policy inside the env launch, shipsim_run_policy): the decision log becomes
    replay rows (good records, env by env) and reference-shaped epoch paths (records in each env's order;
    a non-finite record ends its episode without a transition), with the counters the sliced pass keeps."""
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    N, T = 12, 4
    env = _PolicyEnv(N)
    coll = BatchedPathCollector(env, _Policy(), max_path_length=T, max_ticks=64, deterministic=True,
                                device_policy=_DevicePolicy(), use_graph=False, stream_tail=0)
    assert coll.fused and coll._log_cap() == 4
    rb = DeviceReplayBuffer(1000, 8, 1, "cpu")
    got = coll.collect(60, rb, record_paths=True)
    # expected, from the same log by hand: re-run the scripted sim for the same number of calls
    ref, calls = _PolicySim(N), env.sim.calls
    ep = torch.zeros(N, dtype=torch.int32)
    dec = torch.zeros(N, dtype=torch.int32)
    cap = 4
    log = torch.zeros((N, cap, abi.DECLOG_COLS), dtype=torch.float64)
    ln = torch.zeros(N, dtype=torch.int32)
    rows, paths, cur = [], [], [[] for _ in range(N)]
    for _ in range(calls):
        ln.zero_()
        ref.run_policy(None, 64, T, ep, dec, log=log, log_len=ln,
                       out=dict(ticks=torch.zeros(N, dtype=torch.int32), decisions=torch.zeros(N, dtype=torch.int32)))
        for i in range(N):
            for r in log[i, :int(ln[i])]:
                if not int(r[abi.DL_EVENTS]) & abi.EV_NONFINITE:
                    rows.append((r[abi.DL_OBS0:abi.DL_OBS0 + 8].float(), float(np.float32(r[abi.DL_ACTION])),
                                 float(np.float32(r[abi.DL_REWARD] * 0.5)), float(bool(int(r[abi.DL_EVENTS]) & abi.EV_TERMINAL))))
        for j in range(cap):
            for i in range(N):
                if j >= int(ln[i]):
                    continue
                r = log[i, j]
                nf = int(r[abi.DL_EVENTS]) & abi.EV_NONFINITE
                if not nf:
                    cur[i].append(float(r[abi.DL_REWARD]) * 0.5)
                if r[abi.DL_DONE] or nf or r[abi.DL_DECISION] + 1 >= T:
                    if cur[i]:
                        paths.append(cur[i])
                    cur[i] = []
    n = rb.num_steps_can_sample()
    assert got == n == len(rows) >= 60
    st = rb._store
    for k, (o, a, r, t) in enumerate(rows):
        assert torch.equal(st["observations"][k], o)
        assert float(st["actions"][k, 0]) == a and float(st["rewards"][k, 0]) == r and float(st["terminals"][k, 0]) == t
    got_paths = list(coll.get_epoch_paths())
    assert len(got_paths) == len(paths) > N
    for g, p in zip(got_paths, paths):
        np.testing.assert_array_equal(g["rewards"][:, 0], np.array(p))
    assert any(len(p) == T for p in paths) and any(len(p) < T for p in paths)
    d = coll.device_diagnostics()
    assert d["num nonfinite decisions dropped"] >= 1 and d["num env ticks total"] > 0
    assert coll.get_diagnostics()["num steps total"] == got
