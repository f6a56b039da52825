"""C5 multi-obstacle envs (K obstacle ships, include/shipsim.h shipsim_create) on the device.

* K = 1 through the new create argument is the reference env, bit for bit.
* K = 2 / 4 with the further ships far away (tests/test_multi_obstacle_cpu.py::_far_traffic) reduce to
  the K = 1 episodes bit for bit on the device too (the 4- and 8-slot kernels against the 2-slot one).
* K = 2 / 3 / 4 with the default traffic (shipsim_abi.TRAFFIC_SHIPS): every decision against the CPU
  oracle's restatement of the same generalisation (parity w.r.t. the reference itself is unpinned
  beyond K = 1), in the step kernels and in the decision stream.
Needs an MI355X."""
import numpy as np
import pytest
import torch

import gpu_harness as H
from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import ShipSim
from parity import assert_close
from test_multi_obstacle_cpu import _far_traffic

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _records(gpu):
    return [[(o0.tobytes(), [(o.tobytes(), r, d, b, t) for (o, r, d, b, t) in decs]) for (o0, decs) in env]
            for env in gpu]


@pytest.mark.parametrize("collav", ["none", "sbmpc"])
def test_one_obstacle_ship_is_the_reference_env(collav):
    tables = H.make_tables(32, 2)
    a, fa, _, _ = H.run_gpu(abi.ast_config(collav), tables)
    cfg = abi.ast_config(collav)
    cfg.n_ships = 7  # overridden by n_obs_ships = 1 at create
    sim = ShipSim(cfg, 4, n_obs_ships=1)
    assert sim.n_ships == 2
    sim.close()
    b, fb, _, _ = H.run_gpu(abi.ast_config(collav, n_obs_ships=1), tables)
    assert _records(a) == _records(b)
    for f in fa:
        np.testing.assert_array_equal(fa[f], fb[f])


@pytest.mark.parametrize("collav", ["none", "sbmpc"])
@pytest.mark.parametrize("k", [2, 4])
def test_far_traffic_reduces_to_one_obstacle_on_device(collav, k):
    tables = H.make_tables(48, 2, seed=77)
    a, fa, ea, _ = H.run_gpu(abi.ast_config(collav), tables)
    b, fb, eb, _ = H.run_gpu(_far_traffic(abi.ast_config(collav), k), tables)
    assert _records(a) == _records(b)
    for f in fa:  # ships 0 and 1 of every env
        np.testing.assert_array_equal(fa[f].reshape(48, 2, *fa[f].shape[1:]),
                                      fb[f].reshape(48, 1 + k, *fb[f].shape[1:])[:, :2])
    for f in ea:
        np.testing.assert_array_equal(ea[f], eb[f])


@pytest.mark.parametrize("collav,k,n_envs", [("none", 2, 96), ("sbmpc", 2, 64), ("none", 3, 64), ("sbmpc", 4, 48),
                                             ("none", 4, 64)])
def test_multi_obstacle_vs_oracle(collav, k, n_envs):
    cfg = abi.ast_config(collav, n_obs_ships=k)
    tables = H.make_tables(n_envs, 2, seed=11, special=False)
    gpu, fields, env_fields, _ = H.run_gpu(cfg, tables)
    orcs = H.run_oracle_variants(cfg, tables)
    worst, msgs, chosen = H.compare(gpu, orcs)
    assert not msgs, "\n".join(msgs[:20])
    assert worst <= 1e-5
    assert (chosen != 0).mean() <= 0.1, (chosen != 0).sum()
    orc = [orcs[v][i] for i, v in enumerate(chosen)]
    ships = np.array([o[1] for o in orc])  # (N, 1 + k, 20)
    for f, col in ((abi.F_NORTH, 0), (abi.F_EAST, 1), (abi.F_YAW, 2), (abi.F_U, 3), (abi.F_TIME, 7)):
        assert_close(fields[f].reshape(n_envs, 1 + k), ships[:, :, col], what=f"K={k} field {f}")
    np.testing.assert_array_equal(fields[abi.F_STOP].reshape(n_envs, 1 + k), ships[:, :, 18])
    np.testing.assert_array_equal(fields[abi.F_NEXT_WPT].reshape(n_envs, 1 + k), ships[:, :, 17])
    envs = np.array([o[2] for o in orc])
    np.testing.assert_array_equal(env_fields[abi.E_SBMPC_P_LAST], envs[:, 6])


@pytest.mark.parametrize("collav,k", [("sbmpc", 2), ("none", 4), ("sbmpc", 4)])
def test_multi_obstacle_decision_stream(collav, k):
    """shipsim_run_table with K obstacle ships: records of every 4th env against the oracle replaying
    the same table (tick counts exact), every env's counters in order."""
    from test_gpu_table_fullsize import _episodes, _match
    cfg = abi.ast_config(collav, n_obs_ships=k)
    N, n_dec, n_eps = 256, cfg.max_sampling_frequency, 3
    a_norm = np.random.Generator(np.random.PCG64(4242)).uniform(-1, 1, (n_eps, n_dec, N)).astype(np.float32)
    sim = ShipSim(cfg, N)
    sim.reset()
    table = torch.from_numpy(abi.normalized_to_scoping(a_norm)).cuda()
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    log = torch.zeros((N, 64, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    for _ in range(3):
        sim.run_table(table, 1024, ep, dec, log=log, log_len=log_len)
    sim.synchronize()
    L, n = log.cpu().numpy(), log_len.cpu().numpy()
    sim.close()
    assert (n >= 4).all() and n.max() <= 64
    idx = np.arange(0, N, 4)
    tables = [[a_norm[e % n_eps, :, i] for e in range(int(L[i, n[i] - 1, abi.DL_EPISODE]) + 1)] for i in idx]
    orc = H.run_oracle(cfg, tables)
    bad = []
    for j, i in enumerate(idx):
        rows = L[i, :n[i]]
        assert np.isfinite(rows).all()
        if not _match(_episodes(rows), orc[j][0]) <= 1e-5:
            bad.append(int(i))
    assert len(bad) <= 0.1 * len(idx), f"envs off the oracle: {bad[:20]}"
