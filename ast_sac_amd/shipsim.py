"""Python binding of libshipsim.so (include/shipsim.h) over torch device tensors.

The library is the product path: there is no CPU fallback. If the shared library is missing or
cannot be loaded, importing/constructing raises — build it with `python -c "import
__graft_entry__ as g; g.build()"` (hipcc --offload-arch=gfx950).
"""
import ctypes as C
import os

import torch  # noqa: F401  (loads torch's HIP runtime first; libshipsim binds to the same libamdhip64.so.7)

from . import shipsim_abi as abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SHIPSIM_LIB") or os.path.join(_HERE, "lib", "libshipsim.so")

_lib = None


class ShipSimError(RuntimeError):
    pass


class ShipSimNonFiniteError(ShipSimError):
    """shipsim_synchronize: env decisions ended on a NaN/Inf ship state (SHIPSIM_EV_NONFINITE)."""


def load_library(path=LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ShipSimError(f"native library {path} not found: build it first (__graft_entry__.build())")
    L = C.CDLL(path)
    P = C.c_void_p
    cfgp = C.POINTER(abi.Config)
    L.shipsim_abi_version.restype = C.c_int32
    L.shipsim_build_info.restype = C.c_char_p
    L.shipsim_default_config.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_double, cfgp]
    L.shipsim_create.argtypes = [cfgp, C.c_int32, C.c_int32, C.c_int32, P, C.POINTER(P)]
    L.shipsim_destroy.argtypes = [P]
    L.shipsim_last_error.argtypes = [P]
    L.shipsim_last_error.restype = C.c_char_p
    L.shipsim_set_stream.argtypes = [P, P]
    L.shipsim_num_envs.argtypes = [P]
    L.shipsim_num_envs.restype = C.c_int32
    L.shipsim_lanes_per_env.argtypes = [P]
    L.shipsim_lanes_per_env.restype = C.c_int32
    L.shipsim_reset.argtypes = [P, P, P]
    L.shipsim_step.argtypes = [P, P, P, C.c_int32, P, P, P, P, P, P]
    L.shipsim_tick.argtypes = [P, C.c_int32, P]
    L.shipsim_get_state.argtypes = [P, C.c_int32, P]
    L.shipsim_set_state.argtypes = [P, C.c_int32, P]
    L.shipsim_synchronize.argtypes = [P]
    L.shipsim_nonfinite_count.argtypes = [P]
    L.shipsim_nonfinite_count.restype = C.c_int32
    L.shipsim_set_trajectory.argtypes = [P, P, P, C.c_int32, P]
    L.shipsim_sbmpc_eval.argtypes = [C.c_int32, C.c_double, C.c_double, P, P, P]
    L.shipsim_legacy_step.argtypes = [P, C.c_int32, P, P, P]
    L.shipsim_run_table.argtypes = [P, P, C.c_int32, C.c_int32, C.c_int32, P, P, P, P, P, C.c_int32, P]
    L.shipsim_set_stream_tail.argtypes = [P, C.c_int32]
    # entry points added in later ABI versions: each bound on its own, so an explicitly chosen older build (SHIPSIM_LIB,
    # A/B timing only) that lacks one still gets the argument types of every other
    for name, argtypes in (("shipsim_div_check", [C.c_int32, P, P, P, P, P]),
                           ("shipsim_diag_lane_faults", [P]),
                           ("shipsim_run_policy", [P, P, P, C.c_int32, C.c_int32, C.c_int32, C.c_uint64, P, C.c_int32,
                                                   C.c_int32, P, P, P, P, P, C.c_int32, P]),
                           ("shipsim_sbmpc_eval_multi", [C.c_int32, C.c_int32, C.c_double, C.c_double, P, P, P])):
        try:
            getattr(L, name).argtypes = argtypes
        except AttributeError:
            if "SHIPSIM_LIB" not in os.environ:
                raise
    if L.shipsim_abi_version() != abi.ABI_VERSION:
        raise ShipSimError(f"ABI mismatch: library {L.shipsim_abi_version()} vs binding {abi.ABI_VERSION}")
    from .build_hash import check_library
    try:
        check_library("shipsim", L.shipsim_build_info().decode(), path, explicit="SHIPSIM_LIB" in os.environ)
    except RuntimeError as e:
        raise ShipSimError(str(e)) from None
    _lib = L
    return L


EXPORTED_SYMBOLS = ("shipsim_abi_version", "shipsim_build_info", "shipsim_default_config", "shipsim_create",
                    "shipsim_destroy", "shipsim_last_error", "shipsim_num_envs", "shipsim_reset", "shipsim_step",
                    "shipsim_tick", "shipsim_get_state", "shipsim_set_state", "shipsim_synchronize",
                    "shipsim_set_trajectory", "shipsim_sbmpc_eval", "shipsim_legacy_step", "shipsim_run_table",
                    "shipsim_nonfinite_count", "shipsim_lanes_per_env", "shipsim_set_stream",
                    "shipsim_run_policy", "shipsim_diag_lane_faults", "shipsim_set_stream_tail", "shipsim_div_check",
                    "shipsim_sbmpc_eval_multi")


def diag_lane_faults():
    """Lane / index check violations of a diagnostics build (-DSHIPSIM_LANECHECK) since the last call:
    dict(violations, site, exec), or None for the default build."""
    out = (C.c_uint32 * 32)()
    if load_library().shipsim_diag_lane_faults(out) != 0:
        return None
    return dict(violations=int(out[0]), site=int(out[1]), exec=(int(out[3]) << 32) | int(out[2]),
                per_site={i: int(out[8 + i]) for i in range(16) if out[8 + i]})


def default_config(kind=abi.KIND_AST, machinery=abi.MACH_DETAILED, collav=abi.COLLAV_SBMPC, time_step=4.0):
    cfg = abi.Config()
    rc = load_library().shipsim_default_config(kind, machinery, collav, time_step, C.byref(cfg))
    if rc:
        raise ShipSimError(f"shipsim_default_config failed ({rc})")
    return cfg


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class ShipSim:
    """N independent environments on one device, state resident in HBM."""

    def __init__(self, cfg, n_envs, device=None, n_obs_ships=0):
        """n_obs_ships: obstacle ships per env (AST; 0 = cfg.n_ships - 1, see shipsim_create)."""
        if not torch.cuda.is_available():
            raise ShipSimError("ShipSim needs a HIP device (torch.cuda.is_available() is False)")
        self.L = load_library()
        # a private copy: the caller's config is left as it was (n_obs_ships only applies to this handle)
        cfg = abi.Config.from_buffer_copy(cfg)
        self.n_envs = int(n_envs)
        if n_obs_ships > 0 and cfg.kind == abi.KIND_AST:
            cfg.n_ships = 1 + int(n_obs_ships)
        self.cfg = cfg
        self.n_ships = int(cfg.n_ships)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else torch.device(device).index or 0)
        with torch.cuda.device(self.device):
            self.stream = torch.cuda.current_stream(self.device)
            h = C.c_void_p()
            rc = self.L.shipsim_create(C.byref(cfg), self.n_envs, int(n_obs_ships), self.device.index,
                                       C.c_void_p(self.stream.cuda_stream), C.byref(h))
            if rc:
                msg = self.L.shipsim_last_error(h if h.value else None).decode()
                if h.value:
                    self.L.shipsim_destroy(h)
                raise ShipSimError(f"shipsim_create failed ({rc}): {msg}")
        self.h = h
        self._stream_ptr = self.stream.cuda_stream
        self.lanes_per_env = int(self.L.shipsim_lanes_per_env(h))

    def _follow_stream(self):
        """Launch on torch's current stream of the device (e.g. a graph-capturing one): shipsim_set_stream
        when it changed since the last call."""
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != self._stream_ptr:
            self._check(self.L.shipsim_set_stream(self.h, C.c_void_p(s)), "shipsim_set_stream")
            self._stream_ptr = s

    def _check(self, rc, what):
        if rc:
            raise ShipSimError(f"{what} failed ({rc}): {self.L.shipsim_last_error(self.h).decode()}")

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.L.shipsim_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, x, dtype):
        if x is None:
            return None
        t = torch.as_tensor(x, dtype=dtype, device=self.device).contiguous()
        return t

    def reset(self, mask=None, obs_out=None):
        m = self._dev(mask, torch.uint8) if mask is not None else None
        obs = obs_out if obs_out is not None else torch.empty((self.n_envs, 8), dtype=torch.float32, device=self.device)
        self._follow_stream()
        self._check(self.L.shipsim_reset(self.h, _ptr(m), _ptr(obs)), "shipsim_reset")
        return obs

    def step(self, action, active=None, max_ticks=0, out=None):
        """One sliced decision step (shipsim_step). action: (N,) or (N,1) float32 scoping angles
        [rad] (already denormalized); consumed only by envs waiting for a decision. With
        max_ticks <= 0 every active env runs to its decision point (out['ready'] all ones)."""
        a = self._dev(action, torch.float32).reshape(-1)
        if a.numel() != self.n_envs:
            raise ShipSimError(f"action has {a.numel()} entries, expected {self.n_envs}")
        act = self._dev(active, torch.uint8) if active is not None else None
        if out is None:
            out = dict(obs=torch.empty((self.n_envs, 8), dtype=torch.float32, device=self.device),
                       reward=torch.empty(self.n_envs, dtype=torch.float64, device=self.device),
                       done=torch.empty(self.n_envs, dtype=torch.uint8, device=self.device),
                       events=torch.empty(self.n_envs, dtype=torch.int32, device=self.device),
                       ticks=torch.empty(self.n_envs, dtype=torch.int32, device=self.device),
                       ready=torch.empty(self.n_envs, dtype=torch.uint8, device=self.device))
        self._follow_stream()
        self._check(self.L.shipsim_step(self.h, _ptr(a), _ptr(act), int(max_ticks), _ptr(out["obs"]), _ptr(out["reward"]),
                                        _ptr(out["done"]), _ptr(out["events"]), _ptr(out["ticks"]),
                                        _ptr(out.get("ready"))), "shipsim_step")
        self._keep = (a, act)
        return out

    def tick(self, k=1, events=None):
        """k raw ticks of the loop body (shipsim_tick: SINGLE, and NONIW's MultiShipNonIWEnv._step). events: an
        optional (N,) int32 / uint32 device tensor for the env_info bits of the last tick (NONIW)."""
        self._follow_stream()
        self._check(self.L.shipsim_tick(self.h, int(k), _ptr(events)), "shipsim_tick")

    def set_stream_tail(self, extra_ticks):
        """Work-conserving launch tail of run_table / run_policy (shipsim_set_stream_tail): a wave whose envs met
        max_ticks keeps ticking, 32 ticks at a time, while any wave of the launch has not, up to extra_ticks more
        (0: off). Per-env results are unchanged; only where launches end moves."""
        self._check(self.L.shipsim_set_stream_tail(self.h, int(extra_ticks)), "shipsim_set_stream_tail")
        self.stream_tail = int(extra_ticks)

    def run_table(self, table, max_ticks, ep_idx, dec_idx, out=None, log=None, log_len=None):
        """Open-loop decision stream (shipsim_run_table): table (n_eps, n_dec, N) float32 scoping angles
        on the device; ep_idx / dec_idx (N,) int32 device counters, updated in place. Returns
        dict(ticks=(N,) int32, decisions=(N,) int32). log: optional (N, cap, DECLOG_COLS) float64 with
        log_len (N,) int32."""
        t = self._dev(table, torch.float32)
        if t.dim() != 3 or t.shape[2] != self.n_envs:
            raise ValueError(f"table must be (n_eps, n_dec, {self.n_envs})")
        for x in (ep_idx, dec_idx):
            if x.dtype != torch.int32 or x.device != self.device or x.numel() != self.n_envs:
                raise ValueError("ep_idx / dec_idx must be int32 device tensors of n_envs elements")
        if out is None:
            out = dict(ticks=torch.zeros(self.n_envs, dtype=torch.int32, device=self.device),
                       decisions=torch.zeros(self.n_envs, dtype=torch.int32, device=self.device))
        cap = int(log.shape[1]) if log is not None else 0
        self._follow_stream()
        self._check(self.L.shipsim_run_table(self.h, _ptr(t), int(t.shape[0]), int(t.shape[1]), int(max_ticks),
                                             _ptr(ep_idx), _ptr(dec_idx), _ptr(out["ticks"]), _ptr(out["decisions"]),
                                             _ptr(log), cap, _ptr(log_len)), "shipsim_run_table")
        self._keep_table = t
        return out

    def run_policy(self, policy, max_ticks, n_dec, ep_idx, dec_idx, deterministic=False, seed=0, counter=None,
                   out=None, log=None, log_len=None):
        """The decision stream with the policy in the loop (shipsim_run_policy). policy: (params_ptr, w2t_ptr,
        obs_dim, hidden) as SacFused.policy_weights() returns; counter: (1,) int64 device tensor read by the
        launch (the caller advances it between calls); n_dec: decisions per episode (max_path_length).
        Other arguments and the result as run_table."""
        params, w2t, obs_dim, hidden = policy
        for x in (ep_idx, dec_idx):
            if x.dtype != torch.int32 or x.device != self.device or x.numel() != self.n_envs:
                raise ValueError("ep_idx / dec_idx must be int32 device tensors of n_envs elements")
        if counter is not None and (counter.dtype != torch.int64 or counter.device != self.device):
            raise ValueError("counter must be an int64 device tensor")
        if out is None:
            out = dict(ticks=torch.zeros(self.n_envs, dtype=torch.int32, device=self.device),
                       decisions=torch.zeros(self.n_envs, dtype=torch.int32, device=self.device))
        cap = int(log.shape[1]) if log is not None else 0
        self._follow_stream()
        self._check(self.L.shipsim_run_policy(self.h, C.c_void_p(params), C.c_void_p(w2t), int(obs_dim), int(hidden),
                                              int(bool(deterministic)), int(seed) & ((1 << 64) - 1), _ptr(counter),
                                              int(n_dec), int(max_ticks), _ptr(ep_idx), _ptr(dec_idx),
                                              _ptr(out["ticks"]), _ptr(out["decisions"]), _ptr(log), cap,
                                              _ptr(log_len)), "shipsim_run_policy")
        return out

    def legacy_step(self, k=1, out=None):
        """k legacy MultiShipEnv.step() ticks of every env (shipsim_legacy_step): dict(states=(N, 8) f64
        next_states, done=(N,) u8, status=(N,) i32 termination bits LT_*) of each env's last tick."""
        N = self.n_envs
        if out is None:
            out = dict(states=torch.zeros((N, 8), dtype=torch.float64, device=self.device),
                       done=torch.zeros(N, dtype=torch.uint8, device=self.device),
                       status=torch.zeros(N, dtype=torch.int32, device=self.device))
        self._follow_stream()
        self._check(self.L.shipsim_legacy_step(self.h, int(k), _ptr(out["states"]), _ptr(out["done"]),
                                               _ptr(out["status"])), "shipsim_legacy_step")
        return out

    def _field_shape(self, field):
        S, N = self.n_envs * self.n_ships, self.n_envs
        if field < abi.N_SHIP_FIELDS:
            return (S,), torch.int32 if field in abi.INT_FIELDS else torch.float64
        if field == abi.E_ROUTE_LEN:
            return (S,), torch.int32
        if field in (abi.E_ROUTE_NORTH, abi.E_ROUTE_EAST):
            return (S, abi.MAX_ROUTE), torch.float64
        return (N,), torch.int32 if field in abi.INT_FIELDS else torch.float64

    def get(self, field):
        shape, dt = self._field_shape(field)
        t = torch.empty(shape, dtype=dt, device=self.device)
        self._follow_stream()
        self._check(self.L.shipsim_get_state(self.h, int(field), _ptr(t)), "shipsim_get_state")
        return t

    def set(self, field, value):
        shape, dt = self._field_shape(field)
        t = self._dev(value, dt).reshape(shape)
        self._follow_stream()
        self._check(self.L.shipsim_set_state(self.h, int(field), _ptr(t)), "shipsim_set_state")
        self._keep_set = t

    # -- trajectory recording (include/shipsim.h: shipsim_set_trajectory) --
    def set_trajectory(self, capacity, env_rows=True):
        """Record every tick's simulation_results row (both ships) and RewardTracker row into device
        tensors of `capacity` rows per env; returns dict(ship=(N*2, cap, 20) f64, env=(N, cap, 8) f64,
        len=(N,) int32, cap). Rows start at the next reset."""
        S = self.n_envs * self.n_ships
        cap = int(capacity)
        t = dict(ship=torch.zeros((S, cap, abi.TRAJ_SHIP_COLS), dtype=torch.float64, device=self.device),
                 env=torch.zeros((self.n_envs, cap, abi.TRAJ_ENV_COLS), dtype=torch.float64, device=self.device)
                 if env_rows else None,
                 len=torch.zeros(self.n_envs, dtype=torch.int32, device=self.device), cap=cap)
        self._check(self.L.shipsim_set_trajectory(self.h, _ptr(t["ship"]), _ptr(t["env"]), cap, _ptr(t["len"])),
                    "shipsim_set_trajectory")
        self.traj = t
        return t

    def clear_trajectory(self):
        self._check(self.L.shipsim_set_trajectory(self.h, None, None, 0, None), "shipsim_set_trajectory")
        self.traj = None

    def synchronize(self):
        """Wait for the handle's stream; raises ShipSimNonFiniteError when env decisions ended on a
        non-finite ship state since the previous call (those envs report SHIPSIM_EV_NONFINITE, done)."""
        rc = self.L.shipsim_synchronize(self.h)
        if rc == abi.ENONFINITE:
            raise ShipSimNonFiniteError(self.L.shipsim_last_error(self.h).decode())
        self._check(rc, "shipsim_synchronize")

    def nonfinite_count(self):
        """Decisions flagged SHIPSIM_EV_NONFINITE since create (as of the last synchronize)."""
        return int(self.L.shipsim_nonfinite_count(self.h))


def div_check(num, den, device="cuda"):
    """The kernels' fp64 division by a reused divisor (reciprocal formed once) beside the plain division, on the
    device: (fast, ref) float64 tensors of num / den (shipsim_div_check)."""
    L = load_library()
    a = torch.as_tensor(num, dtype=torch.float64, device=device).contiguous().reshape(-1)
    d = torch.as_tensor(den, dtype=torch.float64, device=device).contiguous().reshape(-1)
    if a.shape != d.shape:
        raise ShipSimError("num and den must have the same size")
    fast, ref = torch.empty_like(a), torch.empty_like(a)
    stream = torch.cuda.current_stream(a.device)
    rc = L.shipsim_div_check(int(a.numel()), _ptr(a), _ptr(d), _ptr(fast), _ptr(ref), C.c_void_p(stream.cuda_stream))
    if rc:
        raise ShipSimError(f"shipsim_div_check failed ({rc})")
    return fast, ref


def sbmpc_eval(requests, tf=1000.0, dt=20.0, device="cuda"):
    """SBMPC.get_optimal_ctrl_offset on the device for a batch of (n, 17) requests
    [P_ca_last, Chi_ca_last, u_d, chi_d, os_state(6), obstacle(5), obs_l, obs_w] -> (n, 3) tensor
    [speed factor, course offset, active] (shipsim_sbmpc_eval)."""
    L = load_library()
    x = torch.as_tensor(requests, dtype=torch.float64, device=device).contiguous()
    if x.dim() != 2 or x.shape[1] != abi.SBMPC_IN:
        raise ShipSimError(f"requests must be (n, {abi.SBMPC_IN})")
    out = torch.empty((x.shape[0], 3), dtype=torch.float64, device=x.device)
    stream = torch.cuda.current_stream(x.device)
    rc = L.shipsim_sbmpc_eval(int(x.shape[0]), float(tf), float(dt), _ptr(x), _ptr(out), C.c_void_p(stream.cuda_stream))
    if rc:
        raise ShipSimError(f"shipsim_sbmpc_eval failed ({rc})")
    return out


def sbmpc_eval_multi(requests, n_obs, tf=1000.0, dt=20.0, device="cuda"):
    """SBMPC.get_optimal_ctrl_offset over a do_list of n_obs obstacles on the device, for a batch of
    (n, SBMPC_MULTI_IN) requests [P_ca_last, Chi_ca_last, u_d, chi_d, os_state(6), then per obstacle slot
    (SHIPSIM_MAX_OBS of them) x, y, psi, u, v, length, width] -> (n, 3) tensor [speed factor, course offset, active]
    (shipsim_sbmpc_eval_multi)."""
    L = load_library()
    x = torch.as_tensor(requests, dtype=torch.float64, device=device).contiguous()
    if x.dim() != 2 or x.shape[1] != abi.SBMPC_MULTI_IN:
        raise ShipSimError(f"requests must be (n, {abi.SBMPC_MULTI_IN})")
    out = torch.empty((x.shape[0], 3), dtype=torch.float64, device=x.device)
    stream = torch.cuda.current_stream(x.device)
    rc = L.shipsim_sbmpc_eval_multi(int(x.shape[0]), int(n_obs), float(tf), float(dt), _ptr(x), _ptr(out),
                                    C.c_void_p(stream.cuda_stream))
    if rc:
        raise ShipSimError(f"shipsim_sbmpc_eval_multi failed ({rc}): n_obs must be 1..{abi.MAX_OBS}")
    return out
