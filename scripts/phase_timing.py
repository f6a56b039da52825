"""Per-phase cycle split of ast_step_kernel (timing build, -DSHIPSIM_PHASE_TIMING).

    SHIPSIM_LIB=ast_sac_amd/lib/abl/lib_TIMING.so python scripts/phase_timing.py none 16
Phases: 0 partner exchange + SBMPC, 1 control + integrate (both ships), 2 map queries,
3 reward / termination / decision logic.
"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ast_sac_amd import shipsim_abi as abi  # noqa: E402
from ast_sac_amd.shipsim import ShipSim, load_library  # noqa: E402

collav = sys.argv[1] if len(sys.argv) > 1 else "none"
lpe = int(sys.argv[2]) if len(sys.argv) > 2 else 16
N = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
L = load_library()
L.shipsim_debug_phase_cycles.argtypes = [C.c_void_p]
cfg = abi.ast_config(collav)
cfg.lanes_per_env = lpe
sim = ShipSim(cfg, N)
tab = torch.from_numpy(abi.normalized_to_scoping(abi.ast_action_table(N)).T.copy()).cuda()
dec = torch.zeros(N, dtype=torch.long, device="cuda")
ar = torch.arange(N, device="cuda")
sim.reset()
buf = (C.c_ulonglong * 8)()
ticks = 0
for it in range(60):
    if it == 10:
        torch.cuda.synchronize()
        L.shipsim_debug_phase_cycles(buf)
        ticks = 0
        t0 = time.perf_counter()
    o = sim.step(tab[dec.clamp(max=8), ar], max_ticks=64)
    ready = o["ready"].bool()
    ticks += int(o["ticks"].sum())
    end = ready & (o["done"].bool() | (dec >= 8))
    dec = torch.where(ready, dec + 1, dec).masked_fill(end, 0)
    sim.reset(mask=end.to(torch.uint8))
torch.cuda.synchronize()
dt = time.perf_counter() - t0
L.shipsim_debug_phase_cycles(buf)
cyc = np.array(buf[:4], dtype=np.float64)
print(f"{collav} lpe{lpe} N={N}: {ticks / dt / 1e6:.1f} M env-ticks/s (timing build)")
for k, name in enumerate(["exchange+sbmpc", "control+integrate", "map queries", "reward+termination+decision"]):
    print(f"  phase {k} {name:30s} {100 * cyc[k] / cyc.sum():5.1f} %")
sb = np.array(buf[4:8], dtype=np.float64)
if sb.sum() > 0:  # SbTimer: per-scenario split of sbmpc_scenario_cost (summed over lanes)
    print("  SBMPC scenario split:", ", ".join(f"{n} {100 * v / sb.sum():.1f} %" for n, v in
                                             zip(["setup+skip", "sample0", "horizon loop", "final/fallback"], sb)))
    print(f"  SBMPC share of phase 0 (lane-cycles / 32 per half-wave): {sb.sum() / 32 / max(cyc[0], 1):.2f}")
