"""Parity tolerances shared by the oracle and GPU tests.

North-star tolerance: trajectories within 1e-5 relative of the CPU reference. "Relative" is taken
per column against |ref| plus a floor of 1 % of the column's largest magnitude (so that values
crossing zero — rudder angle, sway speed, yaw rate — are judged on the column's own scale).
Integer / event quantities (tick counts, event bits, done flags, waypoint indices) must match
exactly.
"""
import numpy as np

RTOL = 1e-5


def rel_err(got, ref, floor_frac=0.01):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    if ref.ndim >= 2:
        scale = np.max(np.abs(ref.reshape(-1, ref.shape[-1])), axis=0)
    else:
        scale = np.max(np.abs(ref)) if ref.size else 0.0
    return np.abs(got - ref) / (np.abs(ref) + floor_frac * scale + 1e-12)


def assert_close(got, ref, rtol=RTOL, what=""):
    e = rel_err(got, ref)
    worst = float(e.max()) if e.size else 0.0
    assert worst <= rtol, f"{what}: worst relative error {worst:.3e} > {rtol:.1e} at {np.unravel_index(e.argmax(), e.shape)}"
    return worst
