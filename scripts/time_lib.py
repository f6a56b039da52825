"""Time the AST step kernel for one library build (SHIPSIM_LIB) — diagnostics for ablations."""
import os, sys, time, json
R = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import numpy as np, torch
from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import ShipSim
collav = sys.argv[1] if len(sys.argv) > 1 else "none"
lpe = int(sys.argv[2]) if len(sys.argv) > 2 else 8
N = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
sl = int(sys.argv[4]) if len(sys.argv) > 4 else 32
cfg = abi.ast_config(collav); cfg.lanes_per_env = lpe
sim = ShipSim(cfg, N)
dev = sim.device
table = torch.from_numpy(abi.normalized_to_scoping(np.random.default_rng(1).uniform(-1, 1, (9, N)).astype(np.float32))).to(dev)
dec = torch.zeros(N, dtype=torch.long, device=dev); ar = torch.arange(N, device=dev)
out = None
sim.reset()
ticks = torch.zeros((), dtype=torch.int64, device=dev)
def step():
    global out
    out = sim.step(table[dec, ar], max_ticks=sl, out=out)
    ready = out["ready"].bool()
    end = ready & (out["done"].bool() | (dec + 1 >= 9))
    ticks.add_(out["ticks"].sum())
    dec.add_(ready.long()); dec.masked_fill_(end, 0)
    sim.reset(mask=end.to(torch.uint8))
for _ in range(20): step()
torch.cuda.synchronize(); ticks.zero_()
t = time.perf_counter()
for _ in range(60): step()
torch.cuda.synchronize(); el = time.perf_counter() - t
print(json.dumps(dict(lib=os.path.basename(os.environ.get("SHIPSIM_LIB", "libshipsim.so")), collav=collav, lpe=lpe, N=N, slice=sl,
                      ticks_per_s=float(ticks.item()) / el, ms_per_step=el / 60 * 1e3)))
