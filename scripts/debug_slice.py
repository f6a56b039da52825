import sys, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
os.environ["SHIPSIM_LIB"] = os.path.join(R, "ast_sac_amd/lib/libshipsim_dbg.so")
sys.path.insert(0, R)
import numpy as np, torch
from ast_sac_amd import shipsim_abi as abi
from ast_sac_amd.shipsim import ShipSim
for lpe in (8,):
    cfg = abi.ast_config("sbmpc"); cfg.lanes_per_env = lpe
    sim = ShipSim(cfg, 4)
    sim.reset()
    for call in range(3):
        print("---- call", call, flush=True)
        out = sim.step(torch.zeros(4), max_ticks=1)
        torch.cuda.synchronize()
        print("n_base", sim.get(104).cpu().numpy(), flush=True)
