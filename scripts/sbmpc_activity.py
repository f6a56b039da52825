"""Fraction of env-ticks (and of 4-env wave-ticks at LPE 16) with SBMPC active, bench workload.
Uses the trajectory record's imminent flag (= SBMPC.is_stephen_useful in sbmpc mode)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ast_sac_amd import shipsim_abi as abi  # noqa: E402
from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, default_args  # noqa: E402

N = 4096
env = BatchedMultiShipRLEnv(default_args(collav_mode="sbmpc"), N)
tr = env.record_trajectories()
env.reset()
tab = torch.from_numpy(abi.normalized_to_scoping(abi.ast_action_table(N)).T.copy()).cuda()
dec = torch.zeros(N, dtype=torch.long, device="cuda")
ar = torch.arange(N, device="cuda")
done_env = torch.zeros(N, dtype=torch.bool, device="cuda")
for it in range(200):
    o = env.step_async(tab[dec.clamp(max=8), ar], max_ticks=64, active=(~done_env).to(torch.uint8))
    ready = o["ready"].bool() & ~done_env
    end = ready & (o["done"].bool() | (dec >= 8))
    dec = torch.where(ready, dec + 1, dec)
    done_env |= end
    if bool(done_env.all()):
        break
L = tr["len"].cpu().numpy()
flags = tr["env"][:, :, abi.TE_FLAGS].cpu().numpy().astype(np.int64)
T = L.max() - 1
act = np.zeros((N, T), bool)
for i in range(N):
    act[i, :L[i] - 1] = (flags[i, :L[i] - 1] & abi.TE_FLAG_IMMINENT) != 0
valid = np.zeros((N, T), bool)
for i in range(N):
    valid[i, :L[i] - 1] = True
print("episodes: mean ticks", (L - 1).mean(), "env-tick active fraction", act.sum() / valid.sum())
w = act.reshape(N // 4, 4, T)
wv = valid.reshape(N // 4, 4, T)
print("wave-ticks with >=1 active env", (w.any(1) & wv.any(1)).sum() / wv.any(1).sum(),
      "mean active envs per active wave-tick", w.sum(1)[w.any(1)].mean())
