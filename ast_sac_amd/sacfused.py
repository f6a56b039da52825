"""ctypes binding of libsacfused.so (include/sac_fused.h): the fused SAC update kernels.

No fallback: if the library is missing, `load_library` raises (build with __graft_entry__.build()).
"""
import ctypes as C
import os

import torch  # noqa: F401  (HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SACFUSED_LIB") or os.path.join(_HERE, "lib", "libsacfused.so")
ABI_VERSION = 4
CHAIN_STAGE_NEXT, CHAIN_FROM_STAGED, CHAIN_NO_GRADS = 1, 2, 4  # sacf_grads_chain flags
EXPORTED_SYMBOLS = ("sacf_abi_version", "sacf_build_info", "sacf_create", "sacf_destroy", "sacf_last_error", "sacf_set_stream",
                    "sacf_param_count", "sacf_target_count", "sacf_stats_count", "sacf_bind", "sacf_sync_params",
                    "sacf_set_replay", "sacf_grads", "sacf_grads_chain", "sacf_apply", "sacf_policy_reserve", "sacf_policy_act",
                    "sacf_policy_weights", "sacf_hidden_supported")
_lib = None


class SacFusedError(RuntimeError):
    pass


class Config(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("obs_dim", C.c_int32), ("hidden", C.c_int32), ("batch", C.c_int32),
                ("discount", C.c_float), ("reward_scale", C.c_float), ("soft_target_tau", C.c_float),
                ("action_reg_coeff", C.c_float), ("clip_val", C.c_float), ("target_entropy", C.c_float),
                ("policy_lr", C.c_float), ("qf_lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float),
                ("adam_eps", C.c_float), ("auto_entropy", C.c_int32), ("world_size", C.c_int32),
                ("split_update", C.c_int32), ("reserved", C.c_int32 * 5)]


def load_library(path=LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SacFusedError(f"native library {path} not found: build it first (__graft_entry__.build())")
    L = C.CDLL(path)
    P = C.c_void_p
    L.sacf_abi_version.restype = C.c_int32
    L.sacf_create.argtypes = [C.POINTER(Config), C.c_int, P, C.POINTER(P)]
    L.sacf_destroy.argtypes = [P]
    L.sacf_last_error.argtypes = [P]
    L.sacf_last_error.restype = C.c_char_p
    L.sacf_set_stream.argtypes = [P, P]
    for f in ("sacf_param_count", "sacf_target_count", "sacf_stats_count"):
        getattr(L, f).argtypes = [P]
        getattr(L, f).restype = C.c_int64
    L.sacf_bind.argtypes = [P] * 8
    L.sacf_sync_params.argtypes = [P]
    L.sacf_set_replay.argtypes = [P, P, P, P, P, P, P, C.c_int64, C.c_uint64]
    L.sacf_grads.argtypes = [P] * 7
    L.sacf_grads_chain.argtypes = [P, P, C.c_int32]
    L.sacf_apply.argtypes = [P]
    L.sacf_policy_reserve.argtypes = [P, C.c_int64]
    L.sacf_hidden_supported.argtypes = [C.c_int32]
    L.sacf_policy_act.argtypes = [P, P, C.c_int64, C.c_int32, P, C.c_int32, C.c_uint64, P, P, P]
    L.sacf_policy_weights.argtypes = [P, C.POINTER(P), C.POINTER(P), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    if L.sacf_abi_version() != ABI_VERSION:
        raise SacFusedError("libsacfused ABI mismatch")
    L.sacf_build_info.restype = C.c_char_p
    from .build_hash import check_library
    try:
        check_library("sacfused", L.sacf_build_info().decode(), path, explicit="SACFUSED_LIB" in os.environ)
    except RuntimeError as e:
        raise SacFusedError(str(e)) from None
    _lib = L
    return L


def hidden_supported(hidden):
    """True if libsacfused has kernels for this hidden width (sacf_hidden_supported)."""
    return bool(load_library().sacf_hidden_supported(int(hidden)))


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class SacFused:
    """One handle = one device + the caller's flat fp32 buffers (see sac_fused.h)."""

    def __init__(self, obs_dim, hidden, batch, device, discount, reward_scale, tau, action_reg, clip_val,
                 target_entropy, policy_lr, qf_lr, auto_entropy=True, world_size=1, betas=(0.9, 0.999), eps=1e-8,
                 split_update=False):
        self.L = load_library()
        cfg = Config(abi_version=ABI_VERSION, obs_dim=obs_dim, hidden=hidden, batch=batch, discount=discount,
                     reward_scale=reward_scale, soft_target_tau=tau, action_reg_coeff=action_reg or 0.0,
                     clip_val=clip_val, target_entropy=target_entropy, policy_lr=policy_lr, qf_lr=qf_lr,
                     beta1=betas[0], beta2=betas[1], adam_eps=eps, auto_entropy=int(bool(auto_entropy)),
                     world_size=world_size, split_update=int(bool(split_update)))
        self.device = torch.device(device)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            rc = self.L.sacf_create(C.byref(cfg), self.device.index or 0,
                                    C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream), C.byref(h))
        if rc:
            msg = self.L.sacf_last_error(h).decode() if h.value else "invalid config"
            if h.value:
                self.L.sacf_destroy(h)
            raise SacFusedError(f"sacf_create failed ({rc}): {msg}")
        self.h = h
        self.n_params = self.L.sacf_param_count(h)
        self.n_targets = self.L.sacf_target_count(h)
        self.n_stats = self.L.sacf_stats_count(h)

    def _check(self, rc, what):
        if rc:
            raise SacFusedError(f"{what} failed ({rc}): {self.L.sacf_last_error(self.h).decode()}")

    def set_stream(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._check(self.L.sacf_set_stream(self.h, C.c_void_p(s.cuda_stream)), "sacf_set_stream")

    def bind(self, params, targets, grads, m, v, step, stats):
        self._bound = (params, targets, grads, m, v, step, stats)
        self._check(self.L.sacf_bind(self.h, *[_p(t) for t in self._bound]), "sacf_bind")

    def sync_params(self):
        self._check(self.L.sacf_sync_params(self.h), "sacf_sync_params")

    def set_replay(self, obs, act, rew, term, next_obs, size_t, capacity, seed):
        self._replay = (obs, act, rew, term, next_obs, size_t)
        self._check(self.L.sacf_set_replay(self.h, _p(obs), _p(act), _p(rew), _p(term), _p(next_obs), _p(size_t),
                                           int(capacity), int(seed) & ((1 << 64) - 1)), "sacf_set_replay")

    def grads(self, batch=None, eps=None):
        b = [None] * 5 if batch is None else [batch[k] for k in ("observations", "actions", "rewards", "terminals",
                                                                    "next_observations")]
        self._check(self.L.sacf_grads(self.h, *[_p(t) for t in b], _p(eps)), "sacf_grads")

    def grads_chain(self, flags, eps=None):
        """A replay-sampled step of a chain (sacf_grads_chain): CHAIN_STAGE_NEXT stages the next step's batch,
        CHAIN_FROM_STAGED starts from the batch the previous call staged (no replay change in between),
        CHAIN_NO_GRADS leaves the gradient buffer unwritten when the update is applied in the same call."""
        self._check(self.L.sacf_grads_chain(self.h, _p(eps), int(flags)), "sacf_grads_chain")

    def apply(self):
        self._check(self.L.sacf_apply(self.h), "sacf_apply")

    def policy_reserve(self, n):
        self._check(self.L.sacf_policy_reserve(self.h, int(n)), "sacf_policy_reserve")

    def policy_act(self, obs, act, mask=None, deterministic=False, seed=0, counter=None, eps_out=None):
        """Actions of the current policy for obs (n, obs_dim) float32 into act (n,) / (n, 1) float32 on
        the handle's stream (sacf_policy_act); rows with mask == 0 keep their action."""
        n, stride = int(obs.shape[0]), int(obs.stride(0))
        self._check(self.L.sacf_policy_act(self.h, _p(obs), n, stride, _p(mask), int(bool(deterministic)),
                                           int(seed) & ((1 << 64) - 1), _p(counter), _p(act), _p(eps_out)),
                    "sacf_policy_act")

    def policy_weights(self):
        """(params_ptr, w2t_ptr, obs_dim, hidden): the device policy parameters and the library's current
        W2ᵀ copy (sacf_policy_weights), for shipsim_run_policy."""
        p, t, o, hdn = C.c_void_p(), C.c_void_p(), C.c_int32(), C.c_int32()
        self._check(self.L.sacf_policy_weights(self.h, C.byref(p), C.byref(t), C.byref(o), C.byref(hdn)),
                    "sacf_policy_weights")
        return p.value, t.value, o.value, hdn.value

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.L.sacf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
