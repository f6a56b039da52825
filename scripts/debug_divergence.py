"""Diagnostics: first state divergence between two builds of libshipsim on the same sliced replay.

    SHIPSIM_LIB=<lib A> python scripts/debug_divergence.py dump  OUT.npz  [collav lpe max_ticks n]
    SHIPSIM_LIB=<lib B> python scripts/debug_divergence.py check OUT.npz  [collav lpe max_ticks n]

`dump` replays tests/gpu_harness.make_tables(n, 2, seed 7) through ShipSim.step with `max_ticks`
slices (as tests/test_gpu_parity.py::test_layout_and_slicing_matrix) and stores every ship / env
state field after every call; `check` replays with the other library and reports the first call,
env, ship and field whose bits differ, with both values and the outputs of that call.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_harness as H  # noqa: E402
from ast_sac_amd import shipsim_abi as abi  # noqa: E402
from ast_sac_amd.shipsim import ShipSim  # noqa: E402

mode, path = sys.argv[1], sys.argv[2]
collav = sys.argv[3] if len(sys.argv) > 3 else "sbmpc"
lpe = int(sys.argv[4]) if len(sys.argv) > 4 else 8
mt = int(sys.argv[5]) if len(sys.argv) > 5 else 3
n = int(sys.argv[6]) if len(sys.argv) > 6 else 192
FIELDS = list(range(abi.N_SHIP_FIELDS)) + list(range(abi.E_SAMPLING_COUNT, abi.E_ROUTE_LEN + 1))
NAMES = {v: k for k, v in vars(abi).items() if (k.startswith("F_") or k.startswith("E_")) and isinstance(v, int)}

cfg = abi.ast_config(collav, machinery=abi.MACH_DETAILED)
cfg.lanes_per_env = lpe
tables = H.make_tables(n, 2, seed=7)
sim = ShipSim(cfg, n)
sim.reset()
ep = np.zeros(n, int)
dec = np.zeros(n, int)
n_eps = np.array([len(t) for t in tables])
snaps = []
ref = dict(np.load(path)) if mode == "check" else None
call = 0
while True:
    active = ep < n_eps
    if not active.any() or call >= 4000:
        break
    acts = np.zeros(n, np.float32)
    for i in np.nonzero(active)[0]:
        acts[i] = abi.normalized_to_scoping(tables[i][ep[i]][dec[i]])
    out = sim.step(torch.from_numpy(acts), active=torch.from_numpy(active.astype(np.uint8)), max_ticks=mt)
    rd = out["ready"].cpu().numpy().astype(bool)
    d = out["done"].cpu().numpy().astype(bool)
    st = {f: sim.get(f).cpu().numpy() for f in FIELDS}
    st["ticks"] = out["ticks"].cpu().numpy()
    st["ready"] = rd.astype(np.int32)
    if mode == "dump":
        for k, v in st.items():
            snaps.append((f"{call}/{k}", v))
    else:
        for k, v in st.items():
            key = f"{call}/{k}"
            if key not in ref:
                print("reference run ended at call", call)
                sys.exit(0)
            w = ref[key]
            a = np.ascontiguousarray(v).view(np.uint8).reshape(len(v), -1)
            b = np.ascontiguousarray(w).view(np.uint8).reshape(len(w), -1)
            bad = np.nonzero((a != b).any(axis=1))[0]
            if len(bad):
                name = NAMES.get(k, k) if isinstance(k, int) else k
                print(f"first divergence: call {call}, field {name}, rows {bad[:8].tolist()} ({len(bad)} rows)")
                for r in bad[:4]:
                    print(f"  row {r}: A {w[r]!r}  B {v[r]!r}")
                for f in FIELDS:
                    vv, ww = st[f], ref[f"{call}/{f}"]
                    diff = np.nonzero((np.ascontiguousarray(vv).view(np.uint8).reshape(len(vv), -1) !=
                                       np.ascontiguousarray(ww).view(np.uint8).reshape(len(ww), -1)).any(axis=1))[0]
                    if len(diff):
                        print(f"  field {NAMES.get(f, f)}: rows {diff[:8].tolist()}")
                prev = call - 1
                if prev >= 0:
                    r0 = int(bad[0])
                    env = r0 // 2 if isinstance(k, int) and k < abi.N_SHIP_FIELDS else r0
                    print(f"  env {env} state before the call (A):",
                          {NAMES.get(f, f): ref[f'{prev}/{f}'][2 * env if f < abi.N_SHIP_FIELDS else env].tolist()
                           for f in FIELDS if f not in (abi.E_ROUTE_NORTH, abi.E_ROUTE_EAST)})
                    print(f"  ticks A {ref[f'{call}/ticks'][env]} B {st['ticks'][env]}; ready A "
                          f"{ref[f'{call}/ready'][env]} B {st['ready'][env]}")
                sys.exit(0)
    call += 1
    need_reset = np.zeros(n, bool)
    for i in np.nonzero(active)[0]:
        if not rd[i]:
            continue
        dec[i] += 1
        if d[i] or dec[i] >= len(tables[i][ep[i]]):
            ep[i] += 1
            dec[i] = 0
            need_reset[i] = ep[i] < n_eps[i]
    if need_reset.any():
        sim.reset(mask=torch.from_numpy(need_reset.astype(np.uint8)))
if mode == "dump":
    np.savez_compressed(path, **dict(snaps))
    print("dumped", call, "calls")
else:
    print("no divergence over", call, "calls")
