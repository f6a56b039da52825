"""Boundary contract of the C ABI, on the device. Needs an MI355X.

* NaN/Inf in a ship state -> the env's decision ends at once, done, SHIPSIM_EV_NONFINITE |
  SHIPSIM_EV_TERMINAL; the other envs are untouched; shipsim_synchronize reports the count.
* The decision stream with a table whose every sampling fails (IW outside the map, env.py:673-693):
  every decision completes without a tick, episodes end at once, and a launch still returns (each env
  completes at most a bounded burst of such decisions per launch and resumes in the next) while its
  wave-mates keep ticking, with their records identical to a run without the failing envs.
"""
import numpy as np
import pytest
import torch

from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import ShipSim, ShipSimNonFiniteError

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("collav", ["none", "sbmpc"])
def test_nonfinite_state_flags_env(collav):
    cfg = abi.ast_config(collav)
    N, bad = 64, 5
    sim = ShipSim(cfg, N)
    sim.reset()
    act = torch.zeros(N, dtype=torch.float32, device="cuda")
    sim.step(act, max_ticks=7)
    sim.synchronize()
    u = sim.get(abi.F_U)
    u[2 * bad + 1] = float("nan")  # the obstacle ship of env `bad`
    sim.set(abi.F_U, u)
    out = sim.step(act, max_ticks=0)
    ready = out["ready"].cpu().numpy().astype(bool)
    done = out["done"].cpu().numpy().astype(bool)
    ev = out["events"].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    ticks = out["ticks"].cpu().numpy()
    assert ready.all()
    assert ev[bad] & abi.EV_NONFINITE and ev[bad] & abi.EV_TERMINAL and done[bad]
    assert ticks[bad] == 1  # flagged at the end of the first tick on the poisoned state
    others = np.arange(N) != bad
    assert not (ev[others] & abi.EV_NONFINITE).any()
    assert np.isfinite(out["obs"].cpu().numpy()[others]).all()
    with pytest.raises(ShipSimNonFiniteError):
        sim.synchronize()
    assert sim.nonfinite_count() == 1
    sim.synchronize()  # reported once
    # the flagged env restarts cleanly after its reset
    mask = torch.zeros(N, dtype=torch.uint8, device="cuda")
    mask[bad] = 1
    sim.reset(mask=mask)
    out = sim.step(act, max_ticks=0)
    assert not (int(out["events"][bad]) & abi.EV_NONFINITE)
    sim.synchronize()
    sim.close()


def test_nonfinite_in_decision_stream():
    cfg = abi.ast_config("none")
    N, bad = 64, 9
    sim = ShipSim(cfg, N)
    sim.reset()
    table = torch.zeros((1, cfg.max_sampling_frequency, N), dtype=torch.float32, device="cuda")
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    log = torch.zeros((N, 64, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    sim.run_table(table, 20, ep, dec, log=log, log_len=log_len)
    y = sim.get(abi.F_YAW)
    y[2 * bad] = float("inf")
    sim.set(abi.F_YAW, y)
    sim.run_table(table, 400, ep, dec, log=log, log_len=log_len)
    L, n = log.cpu().numpy(), log_len.cpu().numpy()
    ev = L[:, :, abi.DL_EVENTS].astype(np.int64)
    flagged = [(i, k) for i in range(N) for k in range(n[i]) if ev[i, k] & abi.EV_NONFINITE]
    assert [i for i, _ in flagged] == [bad]
    i, k = flagged[0]
    assert L[i, k, abi.DL_DONE] == 1 and L[i, k, abi.DL_TICKS] >= 1
    assert np.isfinite(L[i, k + 1:n[i], abi.DL_OBS:]).all() and n[i] > k + 1  # reset in place, then normal
    with pytest.raises(ShipSimNonFiniteError):
        sim.synchronize()
    sim.close()


def _stream(cfg, N, table, slices, launches):
    sim = ShipSim(cfg, N)
    sim.reset()
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    cap = 256
    log = torch.zeros((N, cap, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    ticks = []
    for _ in range(launches):
        o = sim.run_table(table, slices, ep, dec, log=log, log_len=log_len)
        ticks.append(o["ticks"].cpu().numpy())
    sim.synchronize()
    out = log.cpu().numpy(), log_len.cpu().numpy(), np.array(ticks)
    sim.close()
    return out


def test_all_failing_sampling_table_returns():
    """a table whose decision-0 sampling fails for every row must not hang a launch."""
    cfg = abi.ast_config("sbmpc")
    N, n_dec = 64, cfg.max_sampling_frequency
    g = np.random.Generator(np.random.PCG64(7))
    good = abi.normalized_to_scoping(g.uniform(-1, 1, (2, n_dec, N)).astype(np.float32))
    tab = good.copy()
    failing = np.arange(N) % 3 == 1  # mixed into every wave (4 envs per wave)
    tab[:, :, failing] = 1.5        # tan(1.5) * 1414 m: the intermediate waypoint leaves the map
    L, n, ticks = _stream(cfg, N, torch.from_numpy(tab).cuda(), 256, 3)
    Lg, ng, _ = _stream(cfg, N, torch.from_numpy(good).cuda(), 256, 3)
    for i in np.nonzero(failing)[0]:
        rows = L[i, :n[i]]
        assert n[i] == 8 * 3  # a burst of 8 zero-tick decisions per launch, resumed by the next launch
        assert (rows[:, abi.DL_EVENTS].astype(np.int64) & abi.EV_SAMPLING_FAILURE).all()
        assert (rows[:, abi.DL_DONE] == 1).all() and (rows[:, abi.DL_TICKS] == 0).all()
        np.testing.assert_array_equal(rows[:, abi.DL_EPISODE], np.arange(n[i]))
        assert (ticks[:, i] == 0).all()
    for i in np.nonzero(~failing)[0]:  # wave-mates are unaffected
        np.testing.assert_array_equal(L[i, :n[i]], Lg[i, :ng[i]])
        assert (ticks[:, i] == 256).all()
