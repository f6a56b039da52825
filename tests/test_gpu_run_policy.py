"""The decision stream with the policy in the loop (shipsim_run_policy): every decision's action is
the TanhGaussianPolicy's (gaussian_policy.py:105-118, distributions.py:394-425; MakeDeterministic
policies/base.py:54-64) on the observation the env returned, denormalized as NormalizedBoxEnv does
(normalized_box_env.py:48-51), inside the env launch. Checked three ways:
  - the env side: replaying the logged actions through the open-loop stream (shipsim_run_table, itself
    pinned bitwise to the host-driven step loop in test_gpu_table.py) gives the same records bit for bit;
  - the rollout bookkeeping: each decision's logged observation is the previous decision's returned one
    (or the reset state after an episode ended), rollout_functions.py:53-91;
  - the policy: logged actions equal the PyTorch fp32 policy on the logged observations (tolerance 5e-6
    deterministic; stochastic with the kernel's Philox4x32-10 / Box-Muller noise restated in numpy, 2e-5).
Needs an MI355X."""
import numpy as np
import pytest
import torch

from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import ShipSim
from test_gpu_policy_act import _trainer

pytestmark = pytest.mark.gpu

_KEEP = [abi.DL_REWARD, abi.DL_EVENTS, abi.DL_DONE, abi.DL_EPISODE, abi.DL_DECISION, abi.DL_TICKS] + \
    list(range(abi.DL_OBS, abi.DL_OBS + 8))


def _run(cfg, N, n_calls, max_ticks, step, cap=160):
    sim = ShipSim(cfg, N)
    init = sim.reset()[0].cpu().numpy().astype(np.float64)  # the reference's float32 initial_states row
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    log = torch.zeros((N, cap, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    spans = []
    for c in range(n_calls):
        before = log_len.clone()
        o = step(sim, c, ep, dec, log, log_len)
        assert int(o["ticks"].max()) <= max_ticks
        assert torch.equal(o["decisions"], log_len - before)
        spans.append((before.cpu().numpy(), log_len.cpu().numpy()))
    ln = log_len.cpu().numpy()
    assert ln.max() <= cap
    L = log.cpu().numpy()
    sim.close()
    return [L[i, :ln[i]] for i in range(N)], spans, init


def _philox(c0, c1, c2, c3, k0, k1):
    c = [np.asarray(x, np.uint64) for x in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(k0), np.uint64(k1)
    m32 = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        n0 = (p1 >> np.uint64(32)) ^ c[1] ^ k0
        n2 = (p0 >> np.uint64(32)) ^ c[3] ^ k1
        c = [n0 & m32, p1 & m32, n2 & m32, p0 & m32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & m32
        k1 = (k1 + np.uint64(0xBB67AE85)) & m32
    return c


def _eps(env, ctr, seq, seed):
    c = _philox(env, np.uint64(ctr) & np.uint64(0xFFFFFFFF), np.uint64(ctr) >> np.uint64(32),
                np.uint64(0x5A100000) ^ np.asarray(seq, np.uint64), seed & 0xFFFFFFFF, seed >> 32)
    u1 = (c[0].astype(np.float32) + np.float32(1)) * np.float32(2.3283064365386963e-10)
    u2 = c[1].astype(np.float32) * np.float32(2.3283064365386963e-10)
    return np.sqrt(np.float32(-2) * np.log(u1)) * np.cos(np.float32(6.283185307179586) * u2)


def _check_rollout(recs, n_dec, init):
    n = 0
    for r in recs:
        for j in range(len(r)):
            if j == 0 or r[j - 1, abi.DL_DONE] or r[j - 1, abi.DL_DECISION] + 1 >= n_dec:
                want = init
            else:
                want = r[j - 1, abi.DL_OBS:abi.DL_OBS + 8]
            np.testing.assert_array_equal(r[j, abi.DL_OBS0:abi.DL_OBS0 + 8], want)
            n += 1
    return n


# 512: two full 256-unit slices of the in-kernel fc1; 320: a full slice and a one-unit-per-lane one
@pytest.mark.parametrize("collav,H", [("sbmpc", 256), ("none", 64), ("simple", 128), ("sbmpc", 512), ("none", 320)])
def test_policy_stream_deterministic(collav, H):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    tr, pol = _trainer(H)
    dp = tr.device_policy(True)
    cfg = abi.ast_config(collav)
    n_dec = int(cfg.max_sampling_frequency)
    N, max_ticks, n_calls = 192, 96, 40
    recs, _, init = _run(cfg, N, n_calls, max_ticks,
                         lambda sim, c, ep, dec, log, ln: sim.run_policy(dp.weights(), max_ticks, n_dec, ep, dec,
                                                                         deterministic=True, log=log, log_len=ln))
    assert _check_rollout(recs, n_dec, init) > 10 * N
    # the policy: tanh(mean(obs0))
    obs0 = torch.from_numpy(np.concatenate([r[:, abi.DL_OBS0:abi.DL_OBS0 + 8] for r in recs]).astype(np.float32))
    a_log = np.concatenate([r[:, abi.DL_ACTION] for r in recs]).astype(np.float32)
    with torch.no_grad():
        ref = torch.tanh(pol(obs0.cuda()).normal_mean).squeeze(1).cpu().numpy()
    assert np.abs(a_log - ref).max() < 5e-6
    # the env: the logged actions replayed through the open-loop stream give the same records
    n_eps = int(max(r[:, abi.DL_EPISODE].max() for r in recs)) + 2
    table = np.zeros((n_eps, n_dec, N), np.float32)
    for i, r in enumerate(recs):
        table[r[:, abi.DL_EPISODE].astype(int), r[:, abi.DL_DECISION].astype(int), i] = \
            abi.normalized_to_scoping(r[:, abi.DL_ACTION].astype(np.float32))
    t = torch.from_numpy(table).cuda()
    rep, _, _ = _run(cfg, N, n_calls, max_ticks,
                  lambda sim, c, ep, dec, log, ln: sim.run_table(t, max_ticks, ep, dec, log=log, log_len=ln))
    for i in range(N):
        k = len(recs[i])
        assert len(rep[i]) >= k
        np.testing.assert_array_equal(rep[i][:k][:, _KEEP], recs[i][:, _KEEP], err_msg=f"{collav} env {i}")


@pytest.mark.parametrize("H", [256, 512])
def test_policy_stream_stochastic_noise(H):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    tr, pol = _trainer(H)
    seed = 0x1234_5678_9ABC
    dp = tr.device_policy(False, seed=seed)
    cfg = abi.ast_config("sbmpc")
    n_dec = int(cfg.max_sampling_frequency)
    N, max_ticks, n_calls = 256, 128, 24
    counter = torch.full((1,), 5, dtype=torch.int64, device="cuda")

    def step(sim, c, ep, dec, log, ln):
        o = sim.run_policy(dp.weights(), max_ticks, n_dec, ep, dec, deterministic=False, seed=seed,
                           counter=counter, log=log, log_len=ln)
        counter.add_(1)
        return o

    recs, spans, init = _run(cfg, N, n_calls, max_ticks, step)
    _check_rollout(recs, n_dec, init)
    obs0 = torch.from_numpy(np.concatenate([r[:, abi.DL_OBS0:abi.DL_OBS0 + 8] for r in recs]).astype(np.float32))
    with torch.no_grad():
        d = pol(obs0.cuda())
        mean = d.normal_mean.squeeze(1).cpu().numpy()
        std = d.normal_std.squeeze(1).cpu().numpy()
    a_log = np.concatenate([r[:, abi.DL_ACTION] for r in recs]).astype(np.float32)
    # candidate (counter, seq) of each record's draw: chosen in the call it completed in, after the
    # previous completion of that call (seq = completions before it), or — the first completion of a
    # call — at the start of that call (seq 0) or after the last completion of an earlier call
    row = 0
    n_ok = 0
    for i, r in enumerate(recs):
        call_of = np.zeros(len(r), int)
        done_in = []
        for c, (b, a) in enumerate(spans):
            call_of[b[i]:a[i]] = c
            done_in.append(a[i] - b[i])
        for j in range(len(r)):
            c = call_of[j]
            first = spans[c][0][i]
            cands = [(5 + c, j - first)]
            if j == first:
                cands = [(5 + c, 0)] + [(5 + cc, done_in[cc]) for cc in range(c) if done_in[cc] > 0]
            ok = False
            for ctr, seq in cands:
                e = _eps(np.uint64(i), ctr, seq, seed)
                want = np.tanh(np.float32(mean[row] + std[row] * e))
                if abs(float(want) - float(a_log[row])) < 2e-5:
                    ok = True
                    break
            assert ok, (i, j, a_log[row])
            n_ok += 1
            row += 1
    assert n_ok > 8 * N
    # the actions are not deterministic ones
    assert np.abs(a_log - np.tanh(mean)).max() > 0.05


def test_policy_stream_launch_tail_keeps_every_record():
    """run_policy with the work-conserving launch tail (shipsim_set_stream_tail): launch boundaries move,
    a deterministic policy's records do not — every env's records equal the fixed-length launches' record for
    record (the common prefix), every launch's decisions are logged, and no env ticks past max_ticks + extra."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    tr, _ = _trainer(256)
    dp = tr.device_policy(True)
    cfg = abi.ast_config("sbmpc")
    n_dec = int(cfg.max_sampling_frequency)
    N, max_ticks, n_calls, X = 256, 96, 20, 160

    def step(sim, c, ep, dec, log, ln):
        return sim.run_policy(dp.weights(), max_ticks, n_dec, ep, dec, deterministic=True, log=log, log_len=ln)

    ref, _, init = _run(cfg, N, n_calls, max_ticks, step, cap=256)
    sim = ShipSim(cfg, N)
    sim.reset()
    sim.set_stream_tail(X)
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    log = torch.zeros((N, 256, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    over = 0
    for _ in range(n_calls):
        before = log_len.clone()
        o = step(sim, 0, ep, dec, log, log_len)
        assert int(o["ticks"].max()) <= max_ticks + X
        assert torch.equal(o["decisions"], log_len - before)
        over += int((o["ticks"] > max_ticks).sum())
    ln = log_len.cpu().numpy()
    assert ln.max() <= 256
    L = log.cpu().numpy()
    sim.close()
    got = [L[i, :ln[i]] for i in range(N)]
    _check_rollout(got, n_dec, init)
    keep = _KEEP + [abi.DL_ACTION]
    for i in range(N):
        n = min(len(got[i]), len(ref[i]))
        assert len(got[i]) >= len(ref[i]) and n > 0
        np.testing.assert_array_equal(got[i][:n][:, keep], ref[i][:n][:, keep], err_msg=f"env {i}")
    assert over > 0  # the tail ran
    print(f"\n[policy launch tail] env-launches past max_ticks: {over} of {N * n_calls}")
