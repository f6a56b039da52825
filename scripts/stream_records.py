"""Decision records of the headline stream for bitwise comparison of two libshipsim builds (a kernel change that
must not move any result):
    SHIPSIM_LIB=A.so python scripts/stream_records.py run OUT_A.npz   (and again for B)
    python scripts/stream_records.py compare OUT_A.npz OUT_B.npz
C3 sbmpc, 4096 envs, the bench's action table, two 2048-tick launches without the launch tail (fixed launch
boundaries), every decision logged; compare reports the records, tick counts and final states that differ."""
import os
import sys

import numpy as np


def run(out):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ast_sac_amd import shipsim_abi as abi
    from ast_sac_amd.shipsim import ShipSim
    N, cap = 4096, 96
    cfg = abi.ast_config("sbmpc")
    sim = ShipSim(cfg, N)
    sim.reset()
    n_dec = cfg.max_sampling_frequency
    a_norm = np.random.Generator(np.random.PCG64(20251015)).uniform(-1, 1, (8, n_dec, N)).astype(np.float32)
    table = torch.from_numpy(abi.normalized_to_scoping(a_norm)).cuda()
    ep = torch.zeros(N, dtype=torch.int32, device="cuda")
    dec = torch.zeros(N, dtype=torch.int32, device="cuda")
    log = torch.zeros((N, cap, abi.DECLOG_COLS), dtype=torch.float64, device="cuda")
    log_len = torch.zeros(N, dtype=torch.int32, device="cuda")
    ticks = []
    for _ in range(2):
        o = sim.run_table(table, 2048, ep, dec, log=log, log_len=log_len)
        ticks.append(o["ticks"].cpu().numpy())
    fields = [abi.F_NORTH, abi.F_EAST, abi.F_YAW, abi.F_U, abi.F_V, abi.F_R, abi.F_OMEGA, abi.F_TIME]
    state = np.stack([sim.get(f).cpu().numpy().astype(np.float64) for f in fields], 1)
    np.savez(out, log=log.cpu().numpy(), log_len=log_len.cpu().numpy(), ticks=np.stack(ticks), state=state,
             lib=os.environ.get("SHIPSIM_LIB", "in-tree"))
    print(out, int(log_len.cpu().sum()), "records")


def compare(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in ("log_len", "ticks", "state", "log"):
        x, y = A[k], B[k]
        same = np.array_equal(x.view(np.uint8), y.view(np.uint8)) if x.dtype.kind == "f" else np.array_equal(x, y)
        n_diff = int((x != y).sum()) if x.shape == y.shape else -1
        print(f"{k:8s} {'bitwise equal' if same else 'DIFFERS'} ({n_diff} elements differ)")
        ok &= same
    print("IDENTICAL" if ok else "DIFFERENT", str(A["lib"]), str(B["lib"]))


if __name__ == "__main__":
    run(sys.argv[2]) if sys.argv[1] == "run" else compare(sys.argv[2], sys.argv[3])
