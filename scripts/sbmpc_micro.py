"""Micro-benchmark of the wave-cooperative SBMPC (shipsim_sbmpc_eval): cycles per optimisation pass."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ast_sac_amd.shipsim import sbmpc_eval, load_library  # noqa: E402
import ctypes as C  # noqa: E402
L = load_library()
timing = hasattr(L, "shipsim_debug_phase_cycles")
if timing:
    L.shipsim_debug_phase_cycles.argtypes = [C.c_void_p]
    buf = (C.c_ulonglong * 8)()

rng = np.random.Generator(np.random.PCG64(5))
n = 65536
for rad_hi, tag in ((2000, "encounters within D_INIT"), (1000, "close (< 1 km)")):
    os_ = np.stack([rng.uniform(0, 20000, n), rng.uniform(0, 10000, n), rng.uniform(-np.pi, np.pi, n),
                    rng.uniform(0, 6, n), rng.uniform(-0.5, 0.5, n), rng.uniform(-0.01, 0.01, n)], 1)
    ang, rad = rng.uniform(-np.pi, np.pi, n), rng.uniform(20, rad_hi, n)
    ob = np.stack([os_[:, 0] + rad * np.cos(ang), os_[:, 1] + rad * np.sin(ang), rng.uniform(-np.pi, np.pi, n),
                   rng.uniform(0, 6, n), rng.uniform(-0.5, 0.5, n)], 1)
    last = np.stack([rng.choice([0.4, 0.6, 0.8, 1.0], n), np.deg2rad(rng.choice(np.arange(-30, 31, 10), n))], 1)
    req = np.concatenate([last, rng.uniform(3, 5, (n, 1)), rng.uniform(-4, 4, (n, 1)), os_, ob,
                          np.full((n, 1), 80.0), np.full((n, 1), 16.0)], 1)
    x = torch.from_numpy(req).cuda()
    for _ in range(3):
        sbmpc_eval(x)
    torch.cuda.synchronize()
    if timing:
        L.shipsim_debug_phase_cycles(buf)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        sbmpc_eval(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    passes = 32  # 64 requests per wave, two per pass; 1024 waves = one per SIMD
    print(f"{tag}: {ms:.3f} ms for {n} requests -> {ms * 1e3 / passes:.2f} us "
          f"({ms * 1e-3 / passes * 2.4e9:.0f} cycles at 2.4 GHz) per pass")
    if timing:
        L.shipsim_debug_phase_cycles(buf)
        cyc = np.array(buf[4:8], dtype=np.float64)
        print("   scenario split: setup+skip %.1f%%, sample0 %.1f%%, horizon loop %.1f%%, final/fallback %.1f%%"
              % tuple(100 * cyc / max(cyc.sum(), 1)))
