"""ctypes binding of the CPU oracle (oracle/liboracle.so). Test infrastructure only."""
import ctypes as C
import os
import subprocess

import numpy as np

from ast_sac_amd import shipsim_abi as abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")

_lib = None
_native = None


def native_lib():
    """The same oracle source compiled for the host it runs on (-O3 -march=native, OpenMP), into a
    private temp dir: the CPU baseline of bench.py (CPU-baseline plan). The shipped
    oracle/liboracle.so stays -O2 generic x86-64 because it is built in one container and run on
    another machine."""
    global _native
    if _native is None:
        import tempfile
        out = os.path.join(tempfile.mkdtemp(prefix="oracle_native_"), "liboracle_native.so")
        subprocess.check_call(["gcc", "-O3", "-march=native", "-fPIC", "-fopenmp", "-ffp-contract=off",
                               "-fno-fast-math", "-shared", "-I" + os.path.join(ROOT, "include"), "-o", out,
                               os.path.join(ROOT, "oracle", "shipsim_oracle.c"), "-lm"])
        _native = _bind(C.CDLL(out))
    return _native


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ROOT, "oracle", "shipsim_oracle.c")
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        _lib = _bind(C.CDLL(LIB))
    return _lib


def _bind(L):
    if True:
        P = C.c_void_p
        dp = np.ctypeslib.ndpointer(np.float64, flags="C")
        fp = np.ctypeslib.ndpointer(np.float32, flags="C")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C")
        up = np.ctypeslib.ndpointer(np.uint32, flags="C")
        cfgp = C.POINTER(abi.Config)
        L.oracle_env_create.restype = P
        L.oracle_env_create.argtypes = [cfgp]
        L.oracle_env_destroy.argtypes = [P]
        L.oracle_env_set_log.argtypes = [P, C.c_int, dp, C.c_int]
        L.oracle_env_log_len.argtypes = [P, C.c_int]
        L.oracle_env_set_raw.argtypes = [P, C.c_int, dp, C.c_int]
        L.oracle_env_raw_len.argtypes = [P, C.c_int]
        L.oracle_env_set_rtick.argtypes = [P, dp, C.c_int]
        L.oracle_env_rtick_len.argtypes = [P]
        L.oracle_env_reset.argtypes = [P, fp]
        L.oracle_env_step.argtypes = [P, C.c_float, C.c_int, fp, C.POINTER(C.c_double), C.POINTER(C.c_int),
                                      C.POINTER(C.c_uint32)]
        L.oracle_single_run.argtypes = [P, C.c_int]
        L.oracle_legacy_step.argtypes = [P, dp, C.POINTER(C.c_uint32)]
        L.oracle_c1_run.argtypes = [P, C.c_int, up, ip]
        L.oracle_c2_run.argtypes = [cfgp, C.c_int, dp, C.c_int, C.c_void_p, dp, C.c_int]
        L.oracle_ast_rollouts.restype = C.c_longlong
        L.oracle_ast_rollouts.argtypes = [cfgp, C.c_int, C.c_int, fp, ip, ip, dp, up, C.c_int]
        L.oracle_env_get_ship.argtypes = [P, C.c_int, dp]
        L.oracle_env_get_env.argtypes = [P, dp]
        L.oracle_env_get_route.argtypes = [P, dp, dp]
        L.oracle_sbmpc.argtypes = [C.c_double, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_double,
                                   C.c_double, dp, dp, C.c_double, C.c_double, dp]
        L.oracle_sbmpc_multi.argtypes = [C.c_double, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                         C.c_double, C.c_double, dp, C.c_int, dp, dp]
        L.oracle_map_query.argtypes = [cfgp, C.c_int, dp, ip, dp]
        L.oracle_encounter.argtypes = [C.c_int, dp, dp]
        L.oracle_reward_terms.argtypes = [C.c_int, dp, dp]
        L.oracle_termination_reward.restype = C.c_double
        L.oracle_termination_reward.argtypes = [C.c_double, C.c_double, ip]
    return L


LOG_COLS = ["time", "north", "east", "yaw_deg", "rudder_deg", "u", "v", "r_deg", "shaft_rpm", "thrust", "e_ct",
            "heading_err", "fuel"]


class OracleEnv:
    """One reference env (AST, NONIW or SINGLE) in the oracle."""

    def __init__(self, cfg, log_cap=0):
        self.cfg = cfg
        self.h = lib().oracle_env_create(C.byref(cfg))
        self.logs = []
        self.raws = []
        self.rtick = None
        if log_cap:
            for s in range(cfg.n_ships):
                buf = np.zeros((log_cap, 13))
                lib().oracle_env_set_log(self.h, s, buf, log_cap)
                self.logs.append(buf)
                raw = np.zeros((log_cap, abi.TRAJ_SHIP_COLS))
                lib().oracle_env_set_raw(self.h, s, raw, log_cap)
                self.raws.append(raw)
            self.rtick = np.zeros(log_cap)
            lib().oracle_env_set_rtick(self.h, self.rtick, log_cap)

    def __del__(self):
        try:
            lib().oracle_env_destroy(self.h)
        except Exception:
            pass

    def log(self, ship):
        return self.logs[ship][:lib().oracle_env_log_len(self.h, ship)].copy()

    def raw_rows(self, ship):
        """Raw rows in the device trajectory layout (include/shipsim.h SHIPSIM_TS_*)."""
        return self.raws[ship][:lib().oracle_env_raw_len(self.h, ship)].copy()

    def rewards_per_tick(self):
        return self.rtick[:lib().oracle_env_rtick_len(self.h)].copy()

    def reset(self):
        o = np.zeros(8, np.float32)
        lib().oracle_env_reset(self.h, o)
        return o

    def step(self, a, max_ticks=0):
        o = np.zeros(8, np.float32)
        r = C.c_double()
        d = C.c_int()
        b = C.c_uint32()
        ticks = lib().oracle_env_step(self.h, float(np.float32(a)), max_ticks, o, C.byref(r), C.byref(d),
                                      C.byref(b))
        return o, r.value, bool(d.value), int(b.value), ticks

    def legacy_step(self):
        """legacy MultiShipEnv.step(): (next_states (8,) float64, done, termination bits)."""
        out = np.zeros(8)
        b = C.c_uint32()
        d = lib().oracle_legacy_step(self.h, out, C.byref(b))
        return out, bool(d), int(b.value)

    def run_single(self, k):
        return lib().oracle_single_run(self.h, k)

    def run_c1(self, max_ticks=100000):
        bits = np.zeros(max_ticks, np.uint32)
        stops = np.zeros(2 * max_ticks, np.int32)
        k = lib().oracle_c1_run(self.h, max_ticks, bits, stops)
        return bits[:k], stops[:2 * k].reshape(k, 2)

    def ship_state(self, ship):
        out = np.zeros(20)
        lib().oracle_env_get_ship(self.h, ship, out)
        return out

    def env_state(self):
        out = np.zeros(12)
        lib().oracle_env_get_env(self.h, out)
        return out

    def route(self):
        n = int(self.env_state()[8])
        north, east = np.zeros(abi.MAX_ROUTE), np.zeros(abi.MAX_ROUTE)
        lib().oracle_env_get_route(self.h, north, east)
        return np.stack([north[:n], east[:n]], 1)


def c2_run(cfg, init, max_ticks=4000, trace=True, n_threads=1, L=None):
    init = np.ascontiguousarray(init, np.float64)
    n = init.shape[0]
    tr = np.zeros((n, max_ticks, 12)) if trace else None
    fin = np.zeros((n, 7))
    T = (L or lib()).oracle_c2_run(C.byref(cfg), n, init, max_ticks, tr.ctypes.data if trace else None, fin, n_threads)
    return (tr[:, :T] if trace else None), fin


def ast_rollouts(cfg, actions, n_threads=1, L=None):
    actions = np.ascontiguousarray(actions, np.float32)
    n, d = actions.shape
    ticks = np.zeros(n, np.int32)
    dec = np.zeros(n, np.int32)
    ret = np.zeros(n)
    bits = np.zeros(n, np.uint32)
    total = (L or lib()).oracle_ast_rollouts(C.byref(cfg), n, d, actions, ticks, dec, ret, bits, n_threads)
    return total, ticks, dec, ret, bits


def sbmpc(p_last, chi_last, u_d, chi_d, os_state, ob, obs_l=80, obs_w=16, tf=1000, dt=20):
    p = C.c_double(p_last)
    c = C.c_double(chi_last)
    out = np.zeros(3)
    lib().oracle_sbmpc(tf, dt, C.byref(p), C.byref(c), u_d, chi_d, np.ascontiguousarray(os_state, np.float64),
                       np.ascontiguousarray(ob, np.float64), obs_l, obs_w, out)
    return out, p.value, c.value


def sbmpc_multi(p_last, chi_last, u_d, chi_d, os_state, obs, tf=1000, dt=20):
    """get_optimal_ctrl_offset over a do_list: obs (K, 7) rows [x, y, psi, u, v, length, width]. Returns
    ([speed factor, course offset, active], P_ca_last_, Chi_ca_last_)."""
    p = C.c_double(p_last)
    c = C.c_double(chi_last)
    out = np.zeros(3)
    obs = np.ascontiguousarray(obs, np.float64).reshape(-1, 7)
    lib().oracle_sbmpc_multi(tf, dt, C.byref(p), C.byref(c), u_d, chi_d, np.ascontiguousarray(os_state, np.float64),
                             obs.shape[0], obs, out)
    return out, p.value, c.value


def map_query(cfg, ne):
    ne = np.ascontiguousarray(ne, np.float64)
    n = ne.shape[0]
    inside = np.zeros(n, np.int32)
    dist = np.zeros(n)
    lib().oracle_map_query(C.byref(cfg), n, ne, inside, dist)
    return inside, dist
