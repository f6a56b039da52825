"""HIP path (through the C ABI) vs the CPU oracle and the reference golden vectors. Needs an MI355X."""
import numpy as np
import pytest

import gpu_harness as H
from ast_sac_amd import shipsim_abi as abi
from parity import assert_close, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def _set_c2_initial(sim, init, torch):
    for f, col in ((abi.F_NORTH, 0), (abi.F_EAST, 1), (abi.F_YAW, 2), (abi.F_U, 3)):
        sim.set(f, torch.from_numpy(np.ascontiguousarray(init[:, col])))


@pytest.mark.parametrize("dt", [30, 4])
def test_c2_single_ship_vs_golden_trace(golden, torch_cuda, dt):
    """4 (dt=30) / 2 (dt=4) reference ships, checked tick by tick against the fixture trace."""
    from ast_sac_amd.shipsim import ShipSim
    torch = torch_cuda
    g = golden("c2_single_ship")
    init = g[f"dt{dt}_init"]
    ref = g[f"dt{dt}_trace"]
    sim = ShipSim(abi.c2_config(dt), len(init))
    _set_c2_initial(sim, init, torch)
    T = ref.shape[1]
    got = np.zeros((len(init), T, 7))
    for k in range(T):
        got[:, k] = np.stack([sim.get(f).cpu().numpy() for f in (abi.F_TIME, abi.F_NORTH, abi.F_EAST, abi.F_YAW,
                                                                  abi.F_U, abi.F_V, abi.F_R)], 1)
        sim.tick(1)
    assert_close(got, ref[..., :7], what=f"c2 dt{dt} per-tick state")
    fin = np.stack([sim.get(f).cpu().numpy() for f in (abi.F_TIME, abi.F_NORTH, abi.F_EAST, abi.F_YAW, abi.F_U,
                                                        abi.F_V, abi.F_R)], 1)
    assert_close(fin, g[f"dt{dt}_final"], what="c2 final")


@pytest.mark.parametrize("dt", [30, 4])
def test_c2_launch_boundaries_do_not_move_the_state(torch_cuda, dt):
    """The C2 kernel (three pipelined waves per 64 ships, shipsim_tick) carries every ship's state exactly across
    launches: 97 ticks as one launch and as launches of 1, 2, 3, 5, 8, 13, 21 and 44 ticks give the same bits in
    every state field, for ship counts that do and do not fill the last 64-ship block."""
    from ast_sac_amd.shipsim import ShipSim
    torch = torch_cuda
    fields = (abi.F_TIME, abi.F_NORTH, abi.F_EAST, abi.F_YAW, abi.F_U, abi.F_V, abi.F_R, abi.F_E_CT, abi.F_E_CT_INT,
              abi.F_HDG_EI, abi.F_HDG_PREV, abi.F_SPD_A, abi.F_SPD_B, abi.F_RUDDER, abi.F_THRUST, abi.F_LOG_ECT,
              abi.F_NEXT_WPT)
    for n in (4096, 1000):
        init = abi.c2_initial_states(n)
        out = []
        for chunks in ([97], [1, 2, 3, 5, 8, 13, 21, 44]):
            sim = ShipSim(abi.c2_config(dt), n)
            _set_c2_initial(sim, init, torch)
            for k in chunks:
                sim.tick(k)
            out.append(np.stack([sim.get(f).cpu().numpy().astype(np.float64) for f in fields], 1))
            sim.close()
        np.testing.assert_array_equal(out[0], out[1], err_msg=f"dt {dt}, {n} ships")


@pytest.mark.parametrize("dt,ticks", [(30, 334), (4, 2500)])
def test_c2_4096_ships_vs_oracle(torch_cuda, dt, ticks):
    """C2 config at full size: 4096 perturbed ships over the 10000 s horizon in one launch.

    At dt=30 the reference loop is ill-conditioned for ~10 % of the ships: a 1e-12 relative
    perturbation of the initial state moves the oracle's own final state by >1e-7 (rudder saturated
    near a waypoint switch). Those ships are identified with the oracle itself and excluded from the
    strict check; every well-conditioned ship (all of them at dt=4) must match to 1e-5."""
    import oracle_ffi as O
    from ast_sac_amd.shipsim import ShipSim
    torch = torch_cuda
    cfg = abi.c2_config(dt)
    init = abi.c2_initial_states(4096)
    sim = ShipSim(cfg, 4096)
    _set_c2_initial(sim, init, torch)
    sim.tick(ticks)
    fin = np.stack([sim.get(f).cpu().numpy() for f in (abi.F_TIME, abi.F_NORTH, abi.F_EAST, abi.F_YAW, abi.F_U,
                                                        abi.F_V, abi.F_R)], 1)
    _, ref = O.c2_run(cfg, init, trace=False, n_threads=8)
    sens = np.zeros(len(init))
    for col in (0, 2):
        for sgn in (1, -1):
            pert = init.copy()
            pert[:, col] *= 1 + sgn * 1e-12
            _, p = O.c2_run(cfg, pert, trace=False, n_threads=8)
            sens = np.maximum(sens, rel_err(p, ref).max(axis=1))
    ill = sens > 1e-7
    assert ill.mean() < (0.15 if dt == 30 else 1e-9), ill.sum()
    err = rel_err(fin, ref).max(axis=1)
    assert err[~ill].max() <= 1e-5, (err[~ill].max(), int(np.argmax(np.where(ill, 0, err))))
    wpt = sim.get(abi.F_NEXT_WPT).cpu().numpy()
    assert (wpt >= 1).all() and (wpt <= 6).all()


@pytest.mark.parametrize("collav,machinery,n_envs,n_eps", [
    ("none", abi.MACH_DETAILED, 256, 3),
    ("simple", abi.MACH_DETAILED, 128, 3),
    ("sbmpc", abi.MACH_DETAILED, 96, 2),
    ("none", abi.MACH_SIMPLIFIED, 128, 2),
    ("sbmpc", abi.MACH_SIMPLIFIED, 64, 2),
])
def test_ast_env_vs_oracle(torch_cuda, collav, machinery, n_envs, n_eps):
    """Batched MultiShipRLEnv.step on device vs the oracle, env by env, several episodes per env
    (reset between episodes; SBMPC memory and the 'simple' self.states persist across resets)."""
    cfg = abi.ast_config(collav, machinery=machinery)
    tables = H.make_tables(n_envs, n_eps)
    gpu, fields, env_fields, _ = H.run_gpu(cfg, tables)
    orcs = H.run_oracle_variants(cfg, tables)
    worst, msgs, chosen = H.compare(gpu, orcs)
    assert not msgs, "\n".join(msgs[:20])
    assert worst <= 1e-5
    # ill-conditioned envs (matched only by a perturbed oracle run) must stay rare
    assert (chosen != 0).mean() <= 0.1, (chosen != 0).sum()
    orc = [orcs[v][i] for i, v in enumerate(chosen)]
    # end-of-run ship state, both ships of every env
    ships = np.array([o[1] for o in orc])  # (N, 2, 20)
    for f, col in ((abi.F_NORTH, 0), (abi.F_EAST, 1), (abi.F_YAW, 2), (abi.F_U, 3), (abi.F_V, 4), (abi.F_R, 5),
                   (abi.F_TIME, 7), (abi.F_E_CT_INT, 9)):
        got = fields[f].reshape(n_envs, 2)
        assert_close(got, ships[:, :, col], what=f"field {f}")
    np.testing.assert_array_equal(fields[abi.F_NEXT_WPT].reshape(n_envs, 2), ships[:, :, 17])
    envs = np.array([o[2] for o in orc])
    np.testing.assert_array_equal(env_fields[abi.E_SAMPLING_COUNT], envs[:, 0])
    np.testing.assert_array_equal(env_fields[abi.E_SBMPC_P_LAST], envs[:, 6])
    np.testing.assert_array_equal(env_fields[abi.E_SBMPC_CHI_LAST], envs[:, 7])


@pytest.mark.parametrize("collav", ["none", "sbmpc"])
def test_sliced_steps_are_bitwise_identical(torch_cuda, collav):
    """Pausing a decision after max_ticks and resuming it in the next call must not change a bit."""
    cfg = abi.ast_config(collav)
    tables = H.make_tables(48, 2)
    full, f_fields, _, calls_full = H.run_gpu(cfg, tables)
    for mt in (1, 7, 64):
        sl, s_fields, _, calls = H.run_gpu(cfg, tables, max_ticks=mt)
        assert calls > calls_full
        for a, b in zip(full, sl):
            assert len(a) == len(b)
            for (a0, ad), (b0, bd) in zip(a, b):
                np.testing.assert_array_equal(a0, b0)
                assert len(ad) == len(bd)
                for x, y in zip(ad, bd):
                    np.testing.assert_array_equal(x[0], y[0])
                    assert x[1:] == y[1:]
        for f in f_fields:
            np.testing.assert_array_equal(f_fields[f], s_fields[f])


@pytest.mark.parametrize("lpe", [2, 4, 16])
def test_lanes_per_env_variants_identical(torch_cuda, lpe):
    """The lanes-per-env layout only changes the work split; results are bitwise identical up to the
    order of the sub-lane min/or reductions (min is exact)."""
    cfg = abi.ast_config("sbmpc")
    tables = H.make_tables(40, 2)
    ref, r_fields, _, _ = H.run_gpu(cfg, tables)
    cfg2 = abi.ast_config("sbmpc")
    cfg2.lanes_per_env = lpe
    got, g_fields, _, _ = H.run_gpu(cfg2, tables)
    for a, b in zip(ref, got):
        for (a0, ad), (b0, bd) in zip(a, b):
            assert len(ad) == len(bd)
            for x, y in zip(ad, bd):
                np.testing.assert_array_equal(x[0], y[0])
                assert x[1:] == y[1:]
    for f in r_fields:
        np.testing.assert_array_equal(r_fields[f], g_fields[f])


@pytest.mark.parametrize("collav,machinery", [("none", abi.MACH_DETAILED), ("simple", abi.MACH_DETAILED),
                                               ("sbmpc", abi.MACH_DETAILED), ("sbmpc", abi.MACH_SIMPLIFIED)])
def test_layout_and_slicing_matrix(torch_cuda, collav, machinery):
    """Every (lanes-per-env, slice) combination reproduces the LPE=2 whole-decision run bit for bit."""
    tables = H.make_tables(192, 2, seed=7)
    cfg = abi.ast_config(collav, machinery=machinery)
    cfg.lanes_per_env = 2
    ref, r_fields, _, _ = H.run_gpu(cfg, tables)
    for lpe, mt in ((8, 0), (8, 3), (8, 32), (16, 5), (4, 11)):
        c = abi.ast_config(collav, machinery=machinery)
        c.lanes_per_env = lpe
        got, g_fields, _, _ = H.run_gpu(c, tables, max_ticks=mt)
        for a, b in zip(ref, got):
            assert len(a) == len(b)
            for (a0, ad), (b0, bd) in zip(a, b):
                assert len(ad) == len(bd), (lpe, mt)
                for x, y in zip(ad, bd):
                    np.testing.assert_array_equal(x[0], y[0])
                    assert x[1:] == y[1:], (lpe, mt)
        for f in r_fields:
            np.testing.assert_array_equal(r_fields[f], g_fields[f], err_msg=f"field {f} lpe {lpe} mt {mt}")


def test_ast_env_vs_golden_episodes(golden, torch_cuda):
    """The golden fixture episodes (reference run) replayed on device, one env per collav mode."""
    import torch
    from ast_sac_amd.shipsim import ShipSim
    g = golden("rl_env_detailed")
    for collav in ("none", "sbmpc", "simple"):
        sim = ShipSim(abi.ast_config(collav), 1)
        for ep in range(int(g[f"{collav}_n_episodes"])):
            p = f"{collav}_ep{ep}"
            o0 = sim.reset().cpu().numpy()[0]
            np.testing.assert_array_equal(o0, g[p + "_o0"])
            for d, a in enumerate(g[p + "_a"]):
                out = sim.step(torch.tensor([a], dtype=torch.float32))
                assert int(out["ticks"][0]) == g[p + "_nticks"][d], (p, d)
                assert (int(out["events"][0]) & abi.EVENT_MASK) == g[p + "_bits"][d], (p, d)
                assert bool(out["done"][0]) == bool(g[p + "_done"][d])
                assert float(rel_err(out["obs"].cpu().numpy(), g[p + "_obs"][d][None]).max()) <= 1e-5
                assert abs(float(out["reward"][0]) - g[p + "_reward"][d]) <= 1e-5 * (abs(g[p + "_reward"][d]) + 1e-3)
        sim.close()


def test_step_inactive_mask_and_errors(torch_cuda):
    import torch
    from ast_sac_amd.shipsim import ShipSim, ShipSimError
    sim = ShipSim(abi.ast_config("none"), 8)
    with pytest.raises(ShipSimError):
        sim.step(torch.zeros(8))  # step before reset
    sim.reset()
    before = sim.get(abi.F_NORTH).cpu().numpy()
    active = torch.tensor([1, 0, 1, 0, 1, 0, 1, 0], dtype=torch.uint8)
    out = sim.step(torch.zeros(8), active=active)
    after = sim.get(abi.F_NORTH).cpu().numpy().reshape(8, 2)
    np.testing.assert_array_equal(after[1::2], before.reshape(8, 2)[1::2])
    assert (out["ticks"].cpu().numpy()[::2] > 0).all()
    with pytest.raises(ShipSimError):
        sim.step(torch.zeros(7))
    sim.close()


@pytest.mark.parametrize("collav", ["none", "sbmpc"])
def test_map_grid_is_exact(torch_cuda, collav):
    """The map grid (cell edge lists + inside/outside classification) changes no result: 2048 C3 envs
    under random actions give bitwise-identical obs/reward/events/state with and without it."""
    import torch
    from ast_sac_amd.shipsim import ShipSim
    n = 2048
    tables = abi.normalized_to_scoping(abi.ast_action_table(n, n_dec=9, seed=99)).T  # (9, n)
    res = []
    for query in (abi.MAP_ALL_EDGES, abi.MAP_GRID):
        cfg = abi.ast_config(collav)
        cfg.map_query = query
        sim = ShipSim(cfg, n)
        sim.reset()
        outs = []
        dec = torch.zeros(n, dtype=torch.long, device="cuda")
        tab = torch.from_numpy(np.ascontiguousarray(tables)).cuda()
        ar = torch.arange(n, device="cuda")
        for _ in range(60):
            o = sim.step(tab[dec.clamp(max=8), ar], max_ticks=40)
            ready = o["ready"].bool()
            obs = torch.where(ready.unsqueeze(1), o["obs"], 0)  # obs rows are only written for ready envs
            outs.append(torch.cat([obs.double().reshape(-1), torch.where(ready, o["reward"], 0).reshape(-1),
                                   torch.where(ready, o["events"], 0).double(), o["ticks"].double()]).cpu())
            end = ready & (o["done"].bool() | (dec >= 8))
            dec = torch.where(ready, dec + 1, dec).masked_fill(end, 0)
            sim.reset(mask=end.to(torch.uint8))
        st = torch.cat([sim.get(f).double().reshape(-1) for f in (abi.F_NORTH, abi.F_EAST, abi.F_YAW, abi.F_U)]).cpu()
        res.append((torch.stack(outs), st))
        sim.close()
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
