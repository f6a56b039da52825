"""The collector's policy on the matrix cores (libsacfused sacf_policy_act, FusedSACTrainer.device_policy)
against the same TanhGaussianPolicy in PyTorch fp32 ops (gaussian_policy.py:105-118, distributions.py:
394-425; MakeDeterministic policies/base.py:54-64), and the graph-replayed collector pass against the
eager one. Needs an MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Env:
    class action_space:
        shape = (1,)


def _trainer(H=256, seed=3):
    from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    torch.manual_seed(seed)
    dev = torch.device("cuda", 0)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[H, H]).to(dev)
    with torch.no_grad():  # raw AST observations are O(1e4): scale the first layer so tanh is not saturated
        pol.fcs[0].weight.mul_(1e-3)
        pol.last_fc_log_std.bias.fill_(-0.5)
    qs = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[H, H]).to(dev) for _ in range(4)]
    tr = FusedSACTrainer(env=_Env, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2], target_qf2=qs[3],
                         discount=0.965, reward_scale=0.75, policy_lr=8e-5, qf_lr=8e-5, soft_target_tau=1e-3,
                         action_reg_coeff=0.01, clip_val=100.0, batch_size=256, backend="hip")
    return tr, pol


def _obs(n, seed=1):
    g = torch.Generator().manual_seed(seed)
    o = torch.rand(n, 8, generator=g) * torch.tensor([10000, 20000, 3000, 10000, 20000, 6, 5, 500]) - \
        torch.tensor([0, 0, 1500, 0, 0, 3, 0, 250])
    return o.cuda()


@pytest.mark.parametrize("H,n", [(256, 8192), (256, 1000), (64, 77)])
def test_device_policy_matches_torch_policy(H, n):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    tr, pol = _trainer(H)
    obs = _obs(n)
    with torch.no_grad():
        dist = pol(obs)
        mean, std = dist.normal_mean, dist.normal_std
    # deterministic: tanh(mean)
    dp = tr.device_policy(deterministic=True)
    dp.reserve(n)
    act = torch.full((n, 1), 7.0, device="cuda")
    dp.act(obs, None, act)
    torch.cuda.synchronize()
    ref = torch.tanh(mean)
    err = (act - ref).abs().max().item()
    assert err < 5e-6, err
    # stochastic: tanh(mean + std * eps) with the kernel's eps, which is N(0, 1)
    sp = tr.device_policy(deterministic=False, seed=123)
    sp.reserve(n)
    eps = torch.zeros(n, device="cuda")
    act2 = torch.zeros((n, 1), device="cuda")
    sp.act(obs, None, act2, eps_out=eps)
    torch.cuda.synchronize()
    ref2 = torch.tanh(mean + std * eps[:, None])
    assert (act2 - ref2).abs().max().item() < 5e-6
    if n >= 4096:
        e = eps.double()
        assert abs(e.mean().item()) < 0.05 and abs(e.std().item() - 1) < 0.05
    # the counter advanced: a second call draws fresh noise; the mask keeps the unmasked rows
    eps_b = torch.zeros(n, device="cuda")
    mask = (torch.arange(n, device="cuda") % 3 == 0).to(torch.uint8)
    act3 = act2.clone()
    sp.act(obs, mask, act3, eps_out=eps_b)
    torch.cuda.synchronize()
    assert not torch.equal(eps, eps_b)
    keep = mask == 0
    assert torch.equal(act3[keep], act2[keep])
    ref3 = torch.tanh(mean + std * eps_b[:, None])
    assert (act3[~keep] - ref3[~keep]).abs().max().item() < 5e-6


@pytest.mark.parametrize("fused", [False, True])
def test_graph_replayed_collector_equals_eager_collector(fused):
    """A deterministic device-policy collector: the HIP-graph pass and the eager pass produce the same
    transitions in the same replay rows and the same epoch paths (sliced passes, and fused ones with the
    policy inside the env launch)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, default_args
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import BatchedNormalizedBoxEnv
    from ast_sac_amd.ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    tr, pol = _trainer(64)
    res = []
    for use_graph in (True, False):
        env = BatchedNormalizedBoxEnv(BatchedMultiShipRLEnv(default_args(collav_mode="sbmpc"), 512), 0.75)
        coll = BatchedPathCollector(env, pol, max_path_length=9, max_ticks=128, deterministic=True,
                                    device_policy=tr.device_policy(True), use_graph=use_graph, fused=fused,
                                    stream_tail=0)  # (fixed launch boundaries: compared pass by pass)
        assert coll.fused == fused
        rb = DeviceReplayBuffer(40000, 8, 1, "cuda")
        got = coll.collect(6500, rb, record_paths=True)  # ~15 passes of 128 ticks: episodes end
        torch.cuda.synchronize()
        n = rb.num_steps_can_sample()
        res.append((got, n, {k: v[:n].cpu() for k, v in rb._store.items()},
                    [(p["rewards"].copy(), p["actions"].copy()) for p in coll.get_epoch_paths()],
                    int(coll._ticks_total.item())))
    (g1, n1, s1, p1, t1), (g2, n2, s2, p2, t2) = res
    assert g1 == g2 and n1 == n2 and t1 == t2 and n1 >= 6500
    for k in s1:
        assert torch.equal(s1[k], s2[k]), k
    assert len(p1) == len(p2) > 0
    for (r1, a1), (r2, a2) in zip(p1, p2):
        np.testing.assert_array_equal(r1, r2)
        np.testing.assert_array_equal(a1, a2)


def test_fused_collector_rows_and_paths_follow_the_decision_log():
    """The fused collector's bookkeeping: its replay rows are the policy stream's decision records (good ones,
    pass by pass, env by env, record by record) with the reward scaled, and its epoch paths are the episodes
    those records form (rollout_functions.py:161-181) — checked against run_policy driven by hand on a second
    env with the same policy, slice and log capacity."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ast_sac_amd import shipsim_abi as abi
    from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, default_args
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import BatchedNormalizedBoxEnv
    from ast_sac_amd.ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    tr, pol = _trainer(128)
    N, T, ticks, P, scale = 256, 9, 160, 12, 0.75
    env = BatchedNormalizedBoxEnv(BatchedMultiShipRLEnv(default_args(collav_mode="sbmpc"), N), scale)
    dp = tr.device_policy(True)
    coll = BatchedPathCollector(env, pol, max_path_length=T, max_ticks=ticks, deterministic=True, device_policy=dp,
                                use_graph=False, stream_tail=0)  # (fixed launch boundaries: compared pass by pass)
    assert coll.fused
    rb = DeviceReplayBuffer(200000, 8, 1, "cuda")
    coll._take_over()
    coll._enter("fused")
    for _ in range(P):
        coll._fused_pass(rb, True)
    coll._drain_ring()
    torch.cuda.synchronize()
    # by hand
    env2 = BatchedMultiShipRLEnv(default_args(collav_mode="sbmpc"), N)
    sim = env2.sim
    sim.reset()
    cap = coll._log_cap()
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    log = torch.zeros((N, cap, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    ln = torch.zeros(N, dtype=torch.int32, device="cuda")
    rows, paths, cur = [], [], [[] for _ in range(N)]
    for _ in range(P):
        ln.zero_()
        sim.run_policy(dp.weights(), ticks, T, ep, dec, deterministic=True, log=log, log_len=ln)
        L, n = log.cpu().numpy(), ln.cpu().numpy()
        assert n.max() <= cap
        for i in range(N):
            for r in L[i, :n[i]]:
                ev = int(r[abi.DL_EVENTS])
                if not ev & abi.EV_NONFINITE:
                    rows.append((r[abi.DL_OBS0:abi.DL_OBS0 + 8].astype(np.float32), np.float32(r[abi.DL_ACTION]),
                                 np.float32(r[abi.DL_REWARD] * scale), r[abi.DL_OBS:abi.DL_OBS + 8].astype(np.float32),
                                 np.float32(bool(ev & abi.EV_TERMINAL))))
        for j in range(cap):
            for i in range(N):
                if j >= n[i]:
                    continue
                r = L[i, j]
                ev = int(r[abi.DL_EVENTS])
                if not ev & abi.EV_NONFINITE:
                    cur[i].append((r[abi.DL_REWARD] * scale, np.float32(r[abi.DL_ACTION])))
                if r[abi.DL_DONE] or ev & abi.EV_NONFINITE or r[abi.DL_DECISION] + 1 >= T:
                    if cur[i]:
                        paths.append(cur[i])
                    cur[i] = []
    n_rows = rb.num_steps_can_sample()
    assert n_rows == len(rows) > 4 * N
    st = {k: v[:n_rows].cpu().numpy() for k, v in rb._store.items()}
    np.testing.assert_array_equal(st["observations"], np.stack([r[0] for r in rows]))
    np.testing.assert_array_equal(st["actions"][:, 0], np.array([r[1] for r in rows]))
    np.testing.assert_array_equal(st["rewards"][:, 0], np.array([r[2] for r in rows]))
    np.testing.assert_array_equal(st["next_observations"], np.stack([r[3] for r in rows]))
    np.testing.assert_array_equal(st["terminals"][:, 0], np.array([r[4] for r in rows]))
    got = list(coll.get_epoch_paths())
    assert len(got) == len(paths) > N // 2
    for g, p in zip(got, paths):
        np.testing.assert_array_equal(g["rewards"][:, 0], np.array([x[0] for x in p]))
        np.testing.assert_array_equal(g["actions"][:, 0], np.array([x[1] for x in p]))
    assert coll.get_diagnostics()["num steps total"] == len(rows)


def test_sliced_then_fused_collect_rows_match_the_policy():
    """A collector switched from sliced passes (step()) to fused ones (collect()) starts its episodes afresh:
    every replay row the fused passes write has a real observation and the deterministic policy's action on
    it (a decision a sliced pass began and left in flight would have no stored observation / action in the
    policy stream's log: ADVICE round 3)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, default_args
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import BatchedNormalizedBoxEnv
    from ast_sac_amd.ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    tr, pol = _trainer(128)
    N = 128
    env = BatchedNormalizedBoxEnv(BatchedMultiShipRLEnv(default_args(collav_mode="sbmpc"), N), 0.75)
    dp = tr.device_policy(True)
    coll = BatchedPathCollector(env, pol, max_path_length=9, max_ticks=40, deterministic=True, device_policy=dp,
                                use_graph=False)
    assert coll.fused
    for _ in range(3):  # sliced passes of 40 ticks: most envs are mid-decision afterwards
        coll.step()
    rb = DeviceReplayBuffer(100000, 8, 1, "cuda")
    coll.max_ticks = 256
    got = coll.collect(400, rb)
    torch.cuda.synchronize()
    n = rb.num_steps_can_sample()
    assert n == got >= 400
    obs0, act = rb._observations[:n], rb._actions[:n]
    assert bool((obs0.abs().sum(1) > 0).all()), "replay row with an all-zero observation"
    with torch.no_grad():
        ref = torch.tanh(pol(obs0).normal_mean)
    err = (act - ref).abs().max().item()
    assert err < 5e-6, err


def test_fused_collect_with_launch_tail_rows_match_the_policy():
    """The fused collector with the env launch's work-conserving tail (stream_tail): its log capacity covers the
    extra ticks, every replay row is a real observation with the deterministic policy's action on it, and the
    passes ran past max_ticks (the tail is in use). Per-env record parity under the tail is pinned in
    test_gpu_run_policy.py::test_policy_stream_launch_tail_keeps_every_record."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, default_args
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import BatchedNormalizedBoxEnv
    from ast_sac_amd.ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    tr, pol = _trainer(128)
    N, ticks, X = 256, 128, 256
    env = BatchedNormalizedBoxEnv(BatchedMultiShipRLEnv(default_args(collav_mode="sbmpc"), N), 0.75)
    dp = tr.device_policy(True)
    coll = BatchedPathCollector(env, pol, max_path_length=9, max_ticks=ticks, deterministic=True, device_policy=dp,
                                stream_tail=X)
    assert coll.fused and coll._log_cap() == (ticks + X) // 32
    rb = DeviceReplayBuffer(200000, 8, 1, "cuda")
    t0 = coll.device_diagnostics()["num env ticks total"]
    got = coll.collect(4 * N, rb)
    torch.cuda.synchronize()
    n = rb.num_steps_can_sample()
    assert n == got >= 4 * N
    obs0, act = rb._observations[:n], rb._actions[:n]
    assert bool((obs0.abs().sum(1) > 0).all()), "replay row with an all-zero observation"
    with torch.no_grad():
        ref = torch.tanh(pol(obs0).normal_mean)
    err = (act - ref).abs().max().item()
    assert err < 5e-6, err
    assert coll._base_env().sim.stream_tail == X
    print(f"\n[collector tail] rows {n}, env ticks {coll.device_diagnostics()['num env ticks total'] - t0}")
