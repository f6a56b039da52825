"""Legacy per-tick MultiShipEnv (rl_env/ship_in_transit/env.py:783-1181) on the
device — shipsim_legacy_step through the N = 1 facade and batched — against the reference fixtures
(tests/golden/rl_env_legacy.npz) and the CPU oracle. Needs an MI355X."""
import numpy as np
import pytest

import oracle_ffi as O
from ast_sac_amd import shipsim_abi as abi
from parity import assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


@pytest.mark.parametrize("collav", ["none", "simple", "sbmpc"])
def test_legacy_env_matches_reference(golden, torch_cuda, collav):
    """next_states, the 10 termination flags and done of every tick, the obstacle ship's stop flag
    and the ShipDraw snapshots, over two episodes of one env object."""
    from ast_sac_amd.rl_env.ship_in_transit.env import MultiShipEnv, default_args
    g = golden("rl_env_legacy")
    env = MultiShipEnv(ship_draw=True, collav=collav, args=default_args(collav_mode=collav))
    for ep in range(2):
        p = f"{collav}_ep{ep}"
        env.reset()
        ref_d = g[p + "_done"]
        got_s, got_c, got_d = [], [], []
        for _ in range(len(ref_d)):
            s, d, c = env.step()
            got_s.append(s)
            got_c.append(c)
            got_d.append(d)
        assert_close(np.array(got_s), g[p + "_states"], what=p + " next_states")
        np.testing.assert_array_equal(np.array(got_c, np.int8), g[p + "_cond"], err_msg=p + " termination flags")
        np.testing.assert_array_equal(np.array(got_d, np.int8), ref_d, err_msg=p + " done")
        assert env.obs.stop_flag == bool(g[p + "_obs_stop"])
        for ship, name in ((env.test, "test"), (env.obs, "obs")):
            dr = ship.ship_model.ship_drawings
            got = np.array([np.stack([x, y]) for x, y in zip(dr[0], dr[1])]).reshape(-1, 2, 6)
            ref = g[p + f"_{name}_draw"]
            assert got.shape == ref.shape, (p, name)
            assert_close(got.reshape(len(got), -1), ref.reshape(len(ref), -1), what=f"{p} {name} ship_drawings")
    env.close()


@pytest.mark.parametrize("collav", ["none", "simple", "sbmpc"])
def test_batched_legacy_steps_match_oracle(torch_cuda, collav):
    """N envs, k ticks per call: every env equals the oracle's per-tick run; an env stops ticking at
    done inside a call; the simplified-machinery variant runs the same kernel path."""
    from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, default_args
    for mach in ("detailed", "simplified"):
        cfg = abi.ast_config(collav, machinery=abi.MACH_DETAILED if mach == "detailed" else abi.MACH_SIMPLIFIED)
        n = 67
        b = BatchedMultiShipRLEnv(default_args(collav_mode=collav), n, cfg=cfg)
        b.reset()
        ora = O.OracleEnv(cfg)
        ora.reset()
        ref = []
        for _ in range(4000):
            s, d, bits = ora.legacy_step()
            ref.append((s, d, bits))
            if d:
                break
        t = 0
        for k in (1, 7, 64, 500, 4000):
            out = b.legacy_step(k)
            t = min(t + k, len(ref))
            s, d, bits = ref[t - 1]
            st = out["states"].cpu().numpy()
            assert_close(st, np.tile(s, (n, 1)), what=f"{collav} {mach} tick {t} states")
            assert (out["done"].cpu().numpy() == int(d)).all(), (collav, mach, t)
            assert (out["status"].cpu().numpy() == bits).all(), (collav, mach, t)
            if t == len(ref):
                break
        assert t == len(ref) and ref[-1][1], "the episode ends within the ticks run"
        b.close()
