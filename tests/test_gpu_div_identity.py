"""The env kernels divide by a reused divisor with its refined reciprocal formed once (`div_rcp` / `div_by`,
csrc/shipsim_device.hpp): the ship's machinery constants r_me / r_hsg / jp, the step dt in the PIDs, the reward
scales and the shared ω + 0.1 of the two torque quotients (ship_engine.py:416-443, controllers.py:106-118,
reward_designs.py:33-55). These tests pin that this is the same fp64 division, bit for bit, as the compiler's `/`
on the device, over the operand ranges the ship model reaches and far beyond (shipsim_div_check)."""
import numpy as np
import pytest
import torch

from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import div_check, default_config

pytestmark = pytest.mark.gpu


def _rand_doubles(rng, n, e0, e1):
    """n doubles with random sign and mantissa, exponent uniform in [e0, e1]"""
    mant = rng.integers(0, 1 << 52, n, dtype=np.uint64)
    exp = rng.integers(e0 + 1023, e1 + 1024, n).astype(np.uint64)
    sign = rng.integers(0, 2, n).astype(np.uint64)
    return ((sign << np.uint64(63)) | (exp << np.uint64(52)) | mant).view(np.float64)


def _assert_same_bits(num, den):
    fast, ref = div_check(num, den)
    torch.cuda.synchronize()
    f = fast.cpu().numpy().view(np.uint64)
    r = ref.cpu().numpy().view(np.uint64)
    bad = np.flatnonzero(f != r)
    assert bad.size == 0, (f"{bad.size} of {f.size} quotients differ, first: "
                           f"{np.asarray(num).ravel()[bad[0]]!r} / {np.asarray(den).ravel()[bad[0]]!r}")
    # and both are the correctly rounded quotient where numpy can check it (finite, normal results)
    q = np.asarray(num, dtype=np.float64) / np.asarray(den, dtype=np.float64)
    ok = np.isfinite(q) & (np.abs(q) > 2.0 ** -1000)
    np.testing.assert_array_equal(r[ok], q[ok].view(np.uint64))


def test_ship_model_divisors():
    """the divisors the kernels actually reuse (the default AST configuration's ship constants, dt, the reward
    scales), against numerators over the ship model's magnitudes, signs and exact zeros"""
    cfg = default_config(abi.KIND_AST, abi.MACH_DETAILED, abi.COLLAV_SBMPC, 4.0)
    dens = [4.0, 30.0, 0.01, 200000000.0, 175000.0, 1250000.0, 50000.0, 12500.0]
    for k in range(2):
        sh = cfg.ship[k]
        for name in dir(sh):
            if name.startswith("_"):
                continue
            v = getattr(sh, name)
            if isinstance(v, float) and v != 0.0 and np.isfinite(v):
                dens.append(float(v))
    rng = np.random.default_rng(20251018)
    nums = np.concatenate([_rand_doubles(rng, 200_000, -60, 60), np.zeros(100), -np.zeros(100),
                           rng.uniform(-1e6, 1e6, 100_000)])
    for d in sorted(set(dens)):
        _assert_same_bits(nums, np.full_like(nums, d))


def test_wide_operand_ranges():
    """random numerators over 2^-900 .. 2^900 and divisors over 2^-60 .. 2^60, plus the shared-denominator case
    ω + 0.1 over the shaft speeds a ship reaches"""
    rng = np.random.default_rng(7)
    n = 4_000_000
    _assert_same_bits(_rand_doubles(rng, n, -900, 900), _rand_doubles(rng, n, -60, 60))
    omega = rng.uniform(0.0, 40.0, n)
    _assert_same_bits(_rand_doubles(rng, n, -30, 30), omega + 0.1)
