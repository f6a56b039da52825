"""Pin the CPU oracle (oracle/shipsim_oracle.c) against the golden vectors captured from the
reference (tests/golden/gen_golden.py). CPU only."""
import numpy as np
import pytest

import oracle_ffi as O
from ast_sac_amd import shipsim_abi as abi
from parity import assert_close

# oracle log columns -> fixture log columns
AST_COLS = list(range(13))                          # AST_KEYS incl. shaft rpm, thrust kN, fuel
SR_COLS = [0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11]       # SR_KEYS (SimpleShipModel; no shaft / fuel)


@pytest.mark.parametrize("dt", [30, 4])
def test_c2_single_ship_trace(golden, dt):
    g = golden("c2_single_ship")
    tr, fin = O.c2_run(abi.c2_config(dt), g[f"dt{dt}_init"])
    ref = g[f"dt{dt}_trace"]
    assert tr.shape == ref.shape
    np.testing.assert_array_equal(tr[..., 11], ref[..., 11])  # waypoint index: exact
    assert_close(tr[..., :11], ref[..., :11], what=f"c2 dt{dt} trace")
    assert_close(fin, g[f"dt{dt}_final"], what="c2 final")


def test_c2_initial_states_match_fixture(golden):
    g = golden("c2_single_ship")
    init = abi.c2_initial_states(6)
    np.testing.assert_array_equal(init[:4], g["dt30_init"])
    np.testing.assert_array_equal(init[4:6], g["dt4_init"])


@pytest.mark.parametrize("collav", ["none", "sbmpc", "simple"])
def test_c1_noniw_loop(golden, collav):
    g = golden("c1_noniw")
    env = O.OracleEnv(abi.c1_config(collav), log_cap=2000)
    bits, stops = env.run_c1()
    np.testing.assert_array_equal(bits & abi.EVENT_MASK, g[f"{collav}_event_bits"])
    np.testing.assert_array_equal(stops, g[f"{collav}_stops"][:, :2])
    for s, name in ((0, "test"), (1, "obs")):
        assert_close(env.log(s)[:, SR_COLS], g[f"{collav}_{name}_log"], what=f"c1 {collav} {name}")
    fin = np.array([env.ship_state(s)[[7, 0, 1, 2, 3, 4, 5]] for s in (0, 1)])
    assert_close(fin, g[f"{collav}_final"], what="c1 final")


def test_ast_single_ship_and_machinery_dt_quirk(golden):
    """ShipModelAST + PTI machinery; reset() switches the machinery integrator to dt=0.01 (Q1)."""
    g = golden("ast_single_ship")
    cfg = abi.ast_config("none")
    cfg.kind = abi.KIND_SINGLE
    cfg.n_ships = 1
    env = O.OracleEnv(cfg, log_cap=600)
    assert env.ship_state(0)[19] == float(g["fresh_mach_dt"])
    env.run_single(500)
    assert_close(env.log(0), g["fresh_log"], what="fresh")
    assert_close(env.ship_state(0)[[0, 1, 2, 3, 4, 5, 6]], g["fresh_final"], what="fresh final")
    env.reset()
    assert env.ship_state(0)[19] == float(g["after_reset_mach_dt"]) == 0.01
    env.run_single(500)
    assert_close(env.log(0), g["after_reset_log"], what="after reset")
    assert_close(env.ship_state(0)[[0, 1, 2, 3, 4, 5, 6]], g["after_reset_final"], what="after reset final")


def _run_episodes(golden, fname, collav, machinery, cols, cfg=None, prefix=None):
    g = golden(fname)
    prefix = prefix or collav
    env = O.OracleEnv(cfg if cfg is not None else abi.ast_config(collav, machinery=machinery), log_cap=4000)
    for ep in range(int(g[f"{prefix}_n_episodes"])):
        p = f"{prefix}_ep{ep}"
        np.testing.assert_array_equal(env.reset(), g[p + "_o0"])
        n_dec = len(g[p + "_a"])
        got = {k: [] for k in ("obs", "reward", "done", "bits", "nticks")}
        for a in g[p + "_a"]:
            o, r, d, bits, ticks = env.step(a)
            got["obs"].append(o)
            got["reward"].append(r)
            got["done"].append(d)
            got["bits"].append(bits)
            got["nticks"].append(ticks)
            if d:
                break
        assert len(got["obs"]) == n_dec
        np.testing.assert_array_equal(got["nticks"], g[p + "_nticks"], err_msg=p)
        np.testing.assert_array_equal(np.array(got["bits"]) & abi.EVENT_MASK, g[p + "_bits"], err_msg=p)
        np.testing.assert_array_equal(got["done"], g[p + "_done"].astype(bool), err_msg=p)
        bits = np.array(got["bits"])
        np.testing.assert_array_equal((bits & abi.EV_TERMINAL) != 0, g[p + "_terminal"].astype(bool))
        np.testing.assert_array_equal((bits & abi.EV_TEST_STOP) != 0, g[p + "_test_stop"].astype(bool))
        np.testing.assert_array_equal((bits & abi.EV_OBS_STOP) != 0, g[p + "_obs_stop"].astype(bool))
        assert_close(np.array(got["obs"]), g[p + "_obs"], what=p + " obs")
        assert_close(np.array(got["reward"]), g[p + "_reward"], what=p + " reward")
        assert_close(env.log(0)[:, cols], g[p + "_test_log"], what=p + " test log")
        assert_close(env.log(1)[:, cols], g[p + "_obs_log"], what=p + " obs log")
        r_tick = env.rewards_per_tick()
        ref_r = g[p + "_r_tick"]
        # the reference's reward tracker also holds the sampling-failure total (update_r_total_only)
        if bits[-1] & abi.EV_SAMPLING_FAILURE:
            ref_r = ref_r[:-1]
        assert_close(r_tick, ref_r, what=p + " reward per tick")
        np.testing.assert_allclose(env.route(), g[p + "_obs_route"], rtol=0, atol=1e-3)


@pytest.mark.parametrize("collav", ["none", "sbmpc", "simple"])
def test_rl_env_detailed_episodes(golden, collav):
    _run_episodes(golden, "rl_env_detailed", collav, abi.MACH_DETAILED, AST_COLS)


@pytest.mark.parametrize("collav", ["none", "sbmpc"])
def test_rl_env_simplified_episodes(golden, collav):
    _run_episodes(golden, "rl_env_simplified", collav, abi.MACH_SIMPLIFIED, SR_COLS)


MODE_NAMES = {"pto": "PTO", "pti": "PTI", "mec": "MEC"}


@pytest.mark.parametrize("mode", ["pto", "mec"])
@pytest.mark.parametrize("collav", ["none", "sbmpc"])
def test_rl_env_machinery_modes(golden, mode, collav):
    """C5: MachineryModes([pto_mode]) / ([mec_mode]) of run/env_setup.py:62-81 instead of PTI."""
    cfg = abi.set_machinery_mode(abi.ast_config(collav), MODE_NAMES[mode])
    _run_episodes(golden, "rl_env_modes", collav, abi.MACH_DETAILED, AST_COLS, cfg=cfg, prefix=f"{mode}_{collav}")


TRAJ_CASES = [("pti", "none", 2), ("pti", "sbmpc", 1), ("pti", "simple", 1), ("pto", "none", 1), ("mec", "none", 1)]


@pytest.mark.parametrize("mode,collav,n_eps", TRAJ_CASES)
def test_trajectory_schema_from_oracle_rows(golden, mode, collav, n_eps):
    """f1: raw rows in the device trajectory layout (the oracle's) -> the reference's full
    simulation_results dict (all 27 ShipModelAST keys, reference order), time_list, integrator_term."""
    from ast_sac_amd.rl_env.ship_in_transit.trajectory import simulation_results, AST_RESULT_KEYS
    g = golden("rl_env_traj")
    cfg = abi.set_machinery_mode(abi.ast_config(collav), MODE_NAMES[mode])
    env = O.OracleEnv(cfg, log_cap=4000)
    for ep in range(n_eps):
        p = f"{mode}_{collav}_ep{ep}"
        env.reset()
        for a in g[p + "_a"]:
            if env.step(a)[2]:
                break
        for s, name in ((0, "test"), (1, "obs")):
            keys = [str(k) for k in g[p + f"_{name}_keys"]]
            assert tuple(keys) == AST_RESULT_KEYS
            raw = env.raw_rows(s)
            sr = simulation_results(raw, cfg.ship[s], detailed=True, as_lists=False)
            assert list(sr) == keys
            ref = g[p + f"_{name}_sr"]
            assert len(raw) == len(ref), (p, name)
            got = np.stack([sr[k] for k in keys], 1)
            assert_close(got, ref, what=f"{p} {name} simulation_results")
            assert_close(raw[1:, abi.TS_TIME_LIST], g[p + f"_{name}_time_list"], what=p + " time_list")
            assert_close(raw[1:, abi.TS_E_CT_INT], g[p + f"_{name}_integrator_term"], what=p + " integrator_term")


DRAW_CASES = [("none", 3), ("sbmpc", 2)]


def _draw_snapshots_from(env_factory, g, collav, n_eps, rows_of, now_of, step):
    """Drive consecutive episodes of one env object and collect ShipSnapshots (f4) the way the
    MultiShipRLEnv facade does; compare the drawings and the timer with the reference."""
    from ast_sac_amd.rl_env.ship_in_transit.trajectory import ShipSnapshots
    env = env_factory()
    snap = ShipSnapshots(4.0, 30.0)
    for ep in range(n_eps):
        p = f"{collav}_ep{ep}"
        env.reset()
        snap.reset()
        for a in g[p + "_a"]:
            done, ticks = step(env, a)
            fire = snap.advance(ticks)
            if fire:
                snap.draw(fire, [rows_of(env, s) for s in (0, 1)], [now_of(env, s) for s in (0, 1)])
            if done:
                break
        assert snap.timer == g[p + "_timer"], p
        for s, name in ((0, "test"), (1, "obs")):
            ref = g[p + f"_{name}_draw"]
            got = np.array([np.stack([x, y]) for x, y in zip(*snap.drawings[s])]).reshape(-1, 2, 6)
            assert got.shape == ref.shape, (p, name, got.shape, ref.shape)
            assert_close(got.reshape(len(got), -1), ref.reshape(len(ref), -1), what=f"{p} {name} ship_drawings")


@pytest.mark.parametrize("collav,n_eps", DRAW_CASES)
def test_ship_drawings_from_oracle_rows(golden, collav, n_eps):
    """f4: ShipDraw snapshots (env.py:573-579) rebuilt from trajectory rows in the device layout
    (oracle rows here) + the ships' state now; timer carried across resets, drawings cleared."""
    g = golden("rl_env_draw")

    def step(env, a):
        _, _, d, _, ticks = env.step(a)
        return d, ticks

    _draw_snapshots_from(lambda: O.OracleEnv(abi.ast_config(collav), log_cap=4000), g, collav, n_eps,
                         lambda env, s: env.raw_rows(s), lambda env, s: tuple(env.ship_state(s)[:3]), step)


def test_sbmpc_known_answers(golden):
    g = golden("sbmpc_geometry_reward")
    p_last, chi_last = 1.0, 0.0
    for row, out in zip(g["sbmpc_in"], g["sbmpc_out"]):
        res, p_last, chi_last = O.sbmpc(p_last, chi_last, row[0], row[1], row[2:8], row[8:13])
        np.testing.assert_array_equal(res[:2], out[:2])
        assert res[2] == out[2]
        assert (p_last, chi_last) == (out[3], out[4])
    res, _, _ = O.sbmpc(1.0, 0.0, 4.5, -1.0, [1000, 1000, -1, 4.5, 0, 0], [2000, 1500, 2, 4, 0])
    np.testing.assert_array_equal(res[:2], g["sbmpc_survey_ka"])


@pytest.mark.parametrize("K", [2, 3, 4])
def test_sbmpc_multi_obstacle_known_answers(golden, K):
    """get_optimal_ctrl_offset over a do_list of K obstacles (sbmpc.py:149-178), one persistent controller per K:
    the reference's own answers (tests/golden/gen_golden.py gen_sbmpc_multi), exactly, call after call."""
    g = golden("sbmpc_multi")
    p_last, chi_last = 1.0, 0.0
    for row, out in zip(g[f"k{K}_in"], g[f"k{K}_out"]):
        obs = row[8:8 + 7 * K].reshape(K, 7)
        res, p_last, chi_last = O.sbmpc_multi(p_last, chi_last, row[0], row[1], row[2:8], obs)
        np.testing.assert_array_equal(res[:2], out[:2])
        assert res[2] == out[2]
        assert (p_last, chi_last) == (out[3], out[4])


def test_polygon_map_queries(golden):
    g = golden("sbmpc_geometry_reward")
    inside, dist = O.map_query(abi.ast_config(), g["poly_pts_ne"])
    np.testing.assert_array_equal(inside, g["poly_inside"])
    np.testing.assert_allclose(dist, g["poly_dist"], rtol=1e-12, atol=1e-9)


def test_encounter_and_reward_terms(golden):
    g = golden("sbmpc_geometry_reward")
    enc = g["encounter"]
    out = np.zeros((len(enc), 3))
    O.lib().oracle_encounter(len(enc), np.ascontiguousarray(enc[:, :6]), out)
    np.testing.assert_allclose(out[:, 0], enc[:, 6], rtol=1e-14)
    np.testing.assert_array_equal(out[:, 1], enc[:, 7])
    np.testing.assert_allclose(out[:, 2], enc[:, 8], rtol=1e-13, atol=1e-300)
    rt = g["reward_terms"]
    out = np.zeros((len(rt), 4))
    O.lib().oracle_reward_terms(len(rt), np.ascontiguousarray(rt[:, :3]), out)
    np.testing.assert_allclose(out, rt[:, 3:], rtol=1e-13, atol=1e-300)
    for row in g["terminal_reward"]:
        cond = np.ascontiguousarray(row[2:7].astype(np.int32))
        assert O.lib().oracle_termination_reward(row[0], row[1], cond) == pytest.approx(row[7], rel=1e-14, abs=0)


def test_map_bounds(golden):
    g = golden("sbmpc_geometry_reward")
    np.testing.assert_array_equal(g["map_bounds"], [0, 10000, 0, 20000])


@pytest.mark.parametrize("collav", ["none", "simple", "sbmpc"])
def test_legacy_multiship_env(golden, collav):
    """f4: the legacy per-tick MultiShipEnv (env.py:783-1181): next_states, the 10
    get_termination_status flags (termination_flags.py:5-70) and done, per tick, two episodes."""
    g = golden("rl_env_legacy")
    env = O.OracleEnv(abi.ast_config(collav))
    for ep in range(2):
        p = f"{collav}_ep{ep}"
        env.reset()
        ref_s, ref_c, ref_d = g[p + "_states"], g[p + "_cond"], g[p + "_done"]
        got_s, got_c, got_d = [], [], []
        for _ in range(len(ref_d)):
            s, d, b = env.legacy_step()
            got_s.append(s)
            got_c.append([(b >> i) & 1 for i in range(10)])
            got_d.append(d)
        assert_close(np.array(got_s), ref_s, what=p + " next_states")
        np.testing.assert_array_equal(np.array(got_c, np.int8), ref_c, err_msg=p + " termination flags")
        np.testing.assert_array_equal(np.array(got_d, np.int8), ref_d, err_msg=p + " done")
        assert int(env.ship_state(1)[18]) == int(g[p + "_obs_stop"])


@pytest.mark.parametrize("tag", ["none_a", "sbmpc_a", "sbmpc_b"])
def test_trained_policy_closed_loop(golden, tag):
    """f3 on the oracle: the reference's trained-policy replay (golden `trained_policy.npz`) closes the
    loop through this package's deterministic TanhGaussianPolicy (CPU) and the oracle env, with
    NormalizedBoxEnv's float32 action mapping (normalized_box_env.py:48-51)."""
    import torch
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac_amd.ast_sac.torch.sac.policies.base import MakeDeterministic
    from ast_sac_amd.ast_sac.torch.utils import pytorch_util as ptu
    g = golden("trained_policy")
    ptu.set_gpu_mode(False)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[64, 64], init_w=0.5)
    pol.load_state_dict({k[len(tag) + 7:]: torch.from_numpy(g[k]) for k in g.files if k.startswith(tag + "/param/")})
    agent = MakeDeterministic(pol)
    env = O.OracleEnv(abi.ast_config(str(g[tag + "/collav"])))
    lb, ub = np.float32(-np.deg2rad(30)), np.float32(np.deg2rad(30))
    o = env.reset()
    np.testing.assert_array_equal(o, g[tag + "/path/observations"][0])
    acts, rews, obs, dones = [], [], [], []
    while True:
        a, _ = agent.get_action(o)
        a = np.asarray(a, np.float32).reshape(1)
        acts.append(a)
        scaled = np.clip(lb + (a + np.float32(1.)) * np.float32(0.5) * (ub - lb), lb, ub)
        o, r, d, bits, _ = env.step(scaled[0])
        rews.append(r)
        obs.append(o)
        dones.append(d)
        if d:
            break
    n = len(g[tag + "/path/actions"])
    assert len(acts) == n, tag
    np.testing.assert_allclose(np.array(acts), g[tag + "/path/actions"], rtol=1e-5, atol=1e-7)
    assert_close(np.array(obs), g[tag + "/path/next_observations"], what=tag + " obs")
    assert_close(np.array(rews), g[tag + "/path/rewards"][:, 0], what=tag + " rewards")
    np.testing.assert_array_equal(dones, g[tag + "/path/dones"][:, 0])
