"""Open-loop decision stream (shipsim_run_table, the C3 workload): decisions chained and episodes
reset inside the kernel must give, env by env and decision by decision, bitwise the records of the
host-driven loop (shipsim_step slices + masked shipsim_reset between calls, as bench.py did).
Needs an MI355X."""
import numpy as np
import pytest
import torch

from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import ShipSim

pytestmark = pytest.mark.gpu


def _table(n_eps, n_dec, N, seed=20251015):
    g = np.random.Generator(np.random.PCG64(seed))
    a = g.uniform(-1, 1, (n_eps, n_dec, N)).astype(np.float32)
    return torch.from_numpy(abi.normalized_to_scoping(a)).cuda()


def _host_driven(cfg, N, table, max_ticks, n_calls):
    n_eps, n_dec = table.shape[0], table.shape[1]
    sim = ShipSim(cfg, N)
    sim.reset()
    ep = torch.zeros(N, dtype=torch.long, device="cuda")
    dec = torch.zeros(N, dtype=torch.long, device="cuda")
    ar = torch.arange(N, device="cuda")
    recs = [[] for _ in range(N)]
    for _ in range(n_calls):
        out = sim.step(table[ep % n_eps, dec, ar], max_ticks=max_ticks)
        ready = out["ready"].bool()
        done = out["done"].bool()
        r = torch.cat([out["reward"].unsqueeze(1), out["events"].double().unsqueeze(1), done.double().unsqueeze(1),
                       ep.double().unsqueeze(1), dec.double().unsqueeze(1), out["obs"].double()], 1).cpu().numpy()
        for i in np.nonzero(ready.cpu().numpy())[0]:
            recs[i].append(r[i])
        end = ready & (done | (dec + 1 >= n_dec))
        dec += ready.long()
        dec.masked_fill_(end, 0)
        ep += end.long()
        sim.reset(mask=end.to(torch.uint8))
    sim.close()
    return [np.array(x).reshape(-1, 13) for x in recs]


def _chained(cfg, N, table, max_ticks, n_calls, cap=128):
    sim = ShipSim(cfg, N)
    sim.reset()
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    log = torch.zeros((N, cap, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    ticks = decisions = 0
    for _ in range(n_calls):
        o = sim.run_table(table, max_ticks, ep, dec, log=log, log_len=log_len)
        assert int(o["ticks"].max()) <= max_ticks
        ticks += int(o["ticks"].sum())
        decisions += int(o["decisions"].sum())
    ln = log_len.cpu().numpy()
    assert ln.max() <= cap and decisions == int(ln.sum())
    L = log.cpu().numpy()
    keep = [abi.DL_REWARD, abi.DL_EVENTS, abi.DL_DONE, abi.DL_EPISODE, abi.DL_DECISION] + \
        list(range(abi.DL_OBS, abi.DL_OBS + 8))
    sim.close()
    return [L[i, :ln[i]][:, keep] for i in range(N)], ticks


@pytest.mark.parametrize("collav,mach", [("none", "detailed"), ("sbmpc", "detailed"), ("simple", "detailed"),
                                         ("sbmpc", "simplified")])
def test_chained_decisions_equal_host_driven_loop(collav, mach):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    cfg = abi.ast_config(collav, machinery=abi.MACH_DETAILED if mach == "detailed" else abi.MACH_SIMPLIFIED)
    N = 192
    table = _table(3, cfg.max_sampling_frequency, N)
    host = _host_driven(cfg, N, table, 96, 110)
    chain, ticks = _chained(cfg, N, table, 96, 40)
    assert ticks > 0
    n_cmp = 0
    for i in range(N):
        k = min(len(host[i]), len(chain[i]))
        assert k >= 10, (i, len(host[i]), len(chain[i]))
        np.testing.assert_array_equal(chain[i][:k], host[i][:k], err_msg=f"{collav} {mach} env {i}")
        n_cmp += k
    assert n_cmp > 10 * N
    # episodes ended by done and by the 9-decision cap both occur
    eps = np.concatenate([c[:, 3] for c in chain])
    assert eps.max() >= 2


@pytest.mark.parametrize("collav,lpe", [("sbmpc", 8), ("none", 8), ("sbmpc", 4), ("simple", 4)])
def test_stream_lanes_per_env_bitwise(collav, lpe):
    """The decision stream at 8 / 4 lanes per env (more envs per wave) equals the 16-lane kernel bit
    for bit: same per-lane arithmetic, only the split of the map queries / exps over sub-lanes moves."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    cfg = abi.ast_config(collav)
    N = 160
    table = _table(2, cfg.max_sampling_frequency, N, seed=99)
    ref, t_ref = _chained(cfg, N, table, 200, 6)
    cfg.lanes_per_env = lpe
    got, t_got = _chained(cfg, N, table, 200, 6)
    assert t_got == t_ref
    for i in range(N):
        np.testing.assert_array_equal(got[i], ref[i], err_msg=f"{collav} lpe {lpe} env {i}")


@pytest.mark.parametrize("collav,epw", [("sbmpc", 1), ("sbmpc", 3), ("none", 2)])
def test_stream_envs_per_wave_bitwise(collav, epw):
    """Waves launched with fewer envs than they hold (config envs_per_wave: the idle lanes of each wave take no
    part; the wave-cooperative SBMPC pass serves the envs it has) give bitwise the full-wave records."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    cfg = abi.ast_config(collav)
    N = 96
    table = _table(2, cfg.max_sampling_frequency, N, seed=7)
    ref, t_ref = _chained(cfg, N, table, 200, 6)
    cfg.envs_per_wave = epw
    got, t_got = _chained(cfg, N, table, 200, 6)
    assert t_got == t_ref
    for i in range(N):
        np.testing.assert_array_equal(got[i], ref[i], err_msg=f"{collav} epw {epw} env {i}")


@pytest.mark.parametrize("collav", ["sbmpc", "none"])
def test_stream_launch_tail_keeps_every_record(collav):
    """The work-conserving launch tail (shipsim_set_stream_tail): waves that met max_ticks tick on while the
    launch's slowest wave has not. Launch boundaries move, results do not: every env's decision records equal
    the fixed-length launches' record for record (the common prefix), and no env ticks past max_ticks + extra."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    cfg = abi.ast_config(collav)
    N, T, X, calls = 512, 200, 256, 5
    table = _table(2, cfg.max_sampling_frequency, N, seed=5)
    ref, _ = _chained(cfg, N, table, T, calls, cap=256)
    sim = ShipSim(cfg, N)
    sim.reset()
    sim.set_stream_tail(X)
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    log = torch.zeros((N, 256, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    over = 0
    for _ in range(calls):
        o = sim.run_table(table, T, ep, dec, log=log, log_len=log_len)
        assert int(o["ticks"].max()) <= T + X
        over += int((o["ticks"] > T).sum())
    ln = log_len.cpu().numpy()
    assert ln.max() <= 256
    L = log.cpu().numpy()
    keep = [abi.DL_REWARD, abi.DL_EVENTS, abi.DL_DONE, abi.DL_EPISODE, abi.DL_DECISION] + \
        list(range(abi.DL_OBS, abi.DL_OBS + 8))
    sim.close()
    for i in range(N):
        got = L[i, :ln[i]][:, keep]
        n = min(len(got), len(ref[i]))
        assert len(got) >= len(ref[i]) and n > 0
        np.testing.assert_array_equal(got[:n], ref[i][:n], err_msg=f"{collav} env {i}")
    print(f"\n[launch tail {collav}] env-launches past max_ticks: {over} of {N * calls}")
