"""C1 on the device: MultiShipNonIWEnv._step (run_colav/env.py:613-676) in the run_simplified_model.py:245-249 loop,
two ships on fixed routes, collav none / simple / sbmpc (shipsim_tick on a KIND_NONIW handle). Pinned to the
reference's own run of the scenario (tests/golden/c1_noniw.npz, made by tests/golden/gen_golden.py from
/root/reference): the env_info bits and both stop flags of every tick exactly, each ship's state after every tick
against the reference's next simulation_results row while the ship runs, and the final states, within the
north-star tolerance (tests/parity.py)."""
import numpy as np
import pytest
import torch

from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import ShipSim
from parity import assert_close

pytestmark = pytest.mark.gpu

N_ENVS = 3  # identical envs: every lane pair must give the same bits


@pytest.mark.parametrize("collav", ["none", "simple", "sbmpc"])
def test_c1_noniw_vs_reference(golden, collav):
    g = golden("c1_noniw")
    ref_bits = g[f"{collav}_event_bits"]
    ref_stops = g[f"{collav}_stops"][:, :2]
    logs = (g[f"{collav}_test_log"], g[f"{collav}_obs_log"])
    cfg = abi.c1_config(collav)
    sim = ShipSim(cfg, N_ENVS)
    sim.reset()  # init_step (run_colav/env.py:279-323)
    ev = torch.zeros(N_ENVS, dtype=torch.int32, device=sim.device)
    sim_time = float(cfg.simulation_time) if hasattr(cfg, "simulation_time") else None
    # simulation_results row k holds the state at the start of the k-th stored tick (row 0: init_step), so the state
    # after loop tick t is row t + 2 — while the ship runs (a frozen ship's rows repeat its last one)
    cols = [0, 1, 2, 3, 5, 6, 7]  # time, north, east, yaw [deg], u, v, yaw rate [deg/s] (log_cols)
    fields = (abi.F_TIME, abi.F_NORTH, abi.F_EAST, abi.F_YAW, abi.F_U, abi.F_V, abi.F_R)
    for t in range(len(ref_bits)):
        time_before = sim.get(abi.F_TIME).cpu().numpy().reshape(N_ENVS, 2)[:, 0]
        assert sim_time is None or np.all(time_before < sim_time), f"tick {t}: the loop would have ended"
        sim.tick(1, ev)
        bits = ev.cpu().numpy().astype(np.uint32) & abi.EVENT_MASK
        assert np.all(bits == ref_bits[t]), f"tick {t}: bits {bits} vs reference {ref_bits[t]}"
        stops = sim.get(abi.F_STOP).cpu().numpy().reshape(N_ENVS, 2)
        assert np.all(stops == ref_stops[t]), f"tick {t}: stops {stops} vs reference {ref_stops[t]}"
        state = np.stack([sim.get(f).cpu().numpy().reshape(N_ENVS, 2) for f in fields], axis=-1)  # (N, 2, 7)
        assert np.all(state == state[:1]), f"tick {t}: envs differ"
        for ship in (0, 1):
            if not ref_stops[t][ship] and t + 2 < len(logs[ship]):
                got = state[0, ship].copy()
                got[3] = np.rad2deg(got[3])
                got[6] = np.rad2deg(got[6])
                assert_close(got, logs[ship][t + 2, cols], what=f"c1 {collav} tick {t} ship {ship}")
    if sim_time is not None:
        assert np.all(sim.get(abi.F_TIME).cpu().numpy().reshape(N_ENVS, 2)[:, 0] >= sim_time)
    names = (abi.F_TIME, abi.F_NORTH, abi.F_EAST, abi.F_YAW, abi.F_U, abi.F_V, abi.F_R)
    fin = np.stack([sim.get(f).cpu().numpy().reshape(N_ENVS, 2)[0] for f in names], axis=-1)  # (2, 7)
    assert_close(fin, g[f"{collav}_final"], what=f"c1 {collav} final")
    sim.close()


def test_c1_noniw_rejects_detailed_machinery():
    cfg = abi.c1_config("none")
    cfg.machinery = abi.MACH_DETAILED
    sim = ShipSim(cfg, 2)
    with pytest.raises(Exception):
        sim.tick(1)
    sim.close()


@pytest.mark.parametrize("collav", [None, "sbmpc"])
def test_c1_facade_loop_matches_reference(golden, collav):
    """the facade's run_simplified_model loop (BatchedMultiShipNonIWEnv.run) and the one-env object API"""
    from ast_sac_amd.run_colav.env import BatchedMultiShipNonIWEnv, MultiShipNonIWEnv
    name = "none" if collav is None else collav
    g = golden("c1_noniw")
    env = BatchedMultiShipNonIWEnv(collav=collav, n_envs=2)
    events, stops = env.run()
    ev = events.cpu().numpy().astype(np.uint32) & abi.EVENT_MASK
    assert ev.shape[0] == len(g[f"{name}_event_bits"])
    for j in range(2):
        np.testing.assert_array_equal(ev[:, j], g[f"{name}_event_bits"])
        np.testing.assert_array_equal(stops[:, j].cpu().numpy(), g[f"{name}_stops"][:, :2])
    one = MultiShipNonIWEnv(collav=collav)
    one.init_step()
    k = 0
    while one.time < one.sim_time:
        s, done, info = one._step()
        assert s.dtype == np.float32 and s.shape == (6,)
        assert info["events"] == abi.events_to_string(int(g[f"{name}_event_bits"][k]))
        k += 1
    assert k == len(g[f"{name}_event_bits"])


def _c1_device_run(cfg):
    sim = ShipSim(cfg, 1)
    sim.reset()
    ev = torch.zeros(1, dtype=torch.int32, device=sim.device)
    bits, stops = [], []
    while float(sim.get(abi.F_TIME).cpu()[0]) < float(cfg.simulation_time):
        sim.tick(1, ev)
        bits.append(int(ev.cpu()[0]) & abi.EVENT_MASK)
        stops.append(sim.get(abi.F_STOP).cpu().numpy().reshape(2).copy())
        assert len(bits) < 5000
    names = (abi.F_TIME, abi.F_NORTH, abi.F_EAST, abi.F_YAW, abi.F_U, abi.F_V, abi.F_R)
    fin = np.stack([sim.get(f).cpu().numpy().reshape(2) for f in names], axis=-1)
    sim.close()
    return np.array(bits, np.uint32), np.array(stops, np.int32).reshape(-1, 2), fin


@pytest.mark.parametrize("case", range(6))
def test_c1_noniw_vs_oracle_perturbed(case):
    """C1 scenarios off the record (both ships' start moved / turned, every collav mode) against the CPU oracle
    (oracle/shipsim_oracle.c, itself pinned to the reference's run above): event bits and stop flags of every tick
    exactly, the final states within the north-star tolerance"""
    import oracle_ffi as O
    rng = np.random.default_rng(100 + case)
    cfg = abi.c1_config(("none", "simple", "sbmpc")[case % 3])
    t, o = cfg.ship[0], cfg.ship[1]
    t.initial_north_position_m += float(rng.uniform(-300, 300))
    t.initial_east_position_m += float(rng.uniform(-300, 300))
    t.initial_yaw_angle_rad += float(rng.uniform(-0.2, 0.2))
    o.initial_north_position_m += float(rng.uniform(-500, 500))
    o.initial_east_position_m += float(rng.uniform(-500, 500))
    bits, stops, fin = _c1_device_run(cfg)
    env = O.OracleEnv(cfg, log_cap=0)
    ref_bits, ref_stops = env.run_c1()
    assert len(bits) == len(ref_bits)
    np.testing.assert_array_equal(bits, ref_bits.astype(np.uint32) & abi.EVENT_MASK)
    np.testing.assert_array_equal(stops, ref_stops)
    ref_fin = np.array([env.ship_state(s)[[7, 0, 1, 2, 3, 4, 5]] for s in (0, 1)])
    assert_close(fin, ref_fin, what=f"c1 perturbed case {case} final")
