"""Minimal gymnasium-compatible spaces (gymnasium is not a dependency of the build).

Uses gymnasium.spaces.Box when gymnasium is importable, otherwise a small Box with the same
attributes the reference touches: low, high, shape, dtype, sample() (env.py:86-104,
ast_sac/env_wrapper/normalized_box_env.py:34-35, env_replay_buffer.py:20-35, sac.py:64-65).
"""
import numpy as np

try:  # pragma: no cover - depends on the environment
    from gymnasium.spaces import Box as _GymBox
except Exception:  # noqa: BLE001
    _GymBox = None


class _Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        low = np.asarray(low)
        high = np.asarray(high)
        if shape is not None:
            low = np.broadcast_to(low, shape)
            high = np.broadcast_to(high, shape)
        self.dtype = np.dtype(dtype)
        self.low = np.array(low, dtype=self.dtype)
        self.high = np.array(high, dtype=self.dtype)
        self.shape = self.low.shape
        self._rng = np.random.default_rng()

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"


Box = _GymBox if _GymBox is not None else _Box


class Discrete:
    def __init__(self, n):
        self.n = n
