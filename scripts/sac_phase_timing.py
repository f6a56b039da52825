"""Where a SAC grad step's time goes, per kernel and block kind: a diagnostics build of libsacfused
(-DSACF_PHASE_TIMING: wave 0 of every block stamps the device wall clock at entry, operands ready, products
done and exit) runs graph-replayed steps, and the last step's stamps are summarised relative to each kernel's
first block entry (median / max over the blocks of each kind, µs).

  python scripts/sac_phase_timing.py --build          # here: compile ast_sac_amd/lib/diag/libsacfused_timing.so
  python scripts/sac_phase_timing.py [--batch 256]    # on the GPU box
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = os.path.join(ROOT, "ast_sac_amd", "lib", "diag", "libsacfused_timing.so")
KSTAMP, NST = 8192, 8


def diag_path(variant=None):
    return DIAG if not variant else DIAG.replace(".so", f"_{variant}.so")


def build(variant=None, flags=()):
    sys.path.insert(0, ROOT)
    from __graft_entry__ import HIPCC, HIPFLAGS, SAC_SRC
    from ast_sac_amd.build_hash import LIB_FLAGS
    os.makedirs(os.path.dirname(DIAG), exist_ok=True)
    subprocess.check_call([HIPCC] + HIPFLAGS + LIB_FLAGS["sacfused"] + ["-mllvm", "-amdgpu-sched-strategy=max-ilp"] + ["-DSACF_PHASE_TIMING", '-DSACF_SRC_HASH="diag"']
                          + list(flags) + SAC_SRC + ["-o", diag_path(variant)])
    print("built", diag_path(variant))


def kinds(kernel, nblocks, bt, cb, n_mfma, n_valu):
    """Block kind of each block id (mirrors tile_of and the kernels' dispatch)."""
    out = []
    for b in range(nblocks):
        if kernel == 2:
            out.append("mfma_tile" if b < n_mfma else ("valu" if b < n_mfma + n_valu else "scalar"))
            continue
        bx = b // cb
        if kernel == 0:
            out.append("actor_fwd" if bx < 2 * bt else "critic_data_fwd" if bx < 4 * bt else "target_pre")
        else:
            out.append("critic_tangent" if bx < 2 * bt else "targets" if bx < 4 * bt else
                       "critic_factors" if bx < 6 * bt else "actor_factors")
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--build", action="store_true")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--out", default=None)
    p.add_argument("--variant", default=None, help="diagnostics build name suffix (libsacfused_timing_<v>.so)")
    p.add_argument("--flags", default="", help="--build: extra hipcc flags, e.g. -DSACF_WT=0")
    a = p.parse_args()
    if a.build:
        return build(a.variant, a.flags.split())
    os.environ["SACFUSED_LIB"] = diag_path(a.variant)
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from ast_sac_amd import sacfused
    dev = torch.device("cuda", 0)
    r = bench.bench_sac(dev, 1, None, a.steps, a.batch, eager_steps=0, graph=True)
    torch.cuda.synchronize()
    L = sacfused.load_library()
    buf = (C.c_ulonglong * (3 * KSTAMP * NST))()
    assert L.sacf_debug_stamps(buf, len(buf)) == 0
    import numpy as np
    st = np.frombuffer(buf, dtype=np.uint64).reshape(3, KSTAMP, NST).astype(np.float64)
    bp = (a.batch + 31) // 32 * 32
    bt, cb = bp // 32, a.hidden // 32
    grids = [6 * bt * cb, 8 * bt * cb, 3 * cb * cb + 3 * (a.hidden // 16) + 1]
    names = ["fwd (P1)", "mid (P2)", "wgrad (P3)"]
    res = {"step_us": r["ms_per_grad_step"] * 1e3, "batch": a.batch, "hidden": a.hidden, "kernels": {}}
    for k in range(3):
        s = st[k, :grids[k]]
        t0 = s[:, 0].min()
        rel = (s - t0) / 100.0  # 100 MHz ticks -> µs
        ks = kinds(k, grids[k], bt, cb, 3 * cb * cb, 3 * (a.hidden // 16))
        per = {}
        for kind in dict.fromkeys(ks):
            m = rel[[i for i, x in enumerate(ks) if x == kind]]
            per[kind] = {"blocks": int(m.shape[0]),
                         "entry_med": float(np.median(m[:, 0])), "entry_max": float(m[:, 0].max()),
                         "operands_ready_med": float(np.median(m[:, 1] - m[:, 0])),
                         "operands_ready_max": float((m[:, 1] - m[:, 0]).max()),
                         "products_med": float(np.median(m[:, 2] - m[:, 1])),
                         "products_max": float((m[:, 2] - m[:, 1]).max()),
                         "epilogue_med": float(np.median(m[:, 3] - m[:, 2])),
                         "epilogue_max": float((m[:, 3] - m[:, 2]).max()),
                         "exit_med": float(np.median(m[:, 3])), "exit_max": float(m[:, 3].max())}
            for q in range(4, NST):  # prologue points stamped by this kind (0 = not stamped)
                got = st[k, :grids[k]][[i for i, x in enumerate(ks) if x == kind], q] > 0
                if got.all():
                    per[kind][f"p{q}_since_entry_med"] = float(np.median(m[:, q] - m[:, 0]))
                    per[kind][f"p{q}_since_entry_max"] = float((m[:, q] - m[:, 0]).max())
        res["kernels"][names[k]] = {"span_us": float(rel[:, 3].max()), "kinds": per}
        # per block (relative to the kernel's first entry, µs): entry, operands ready, products done, exit, p4
        res.setdefault("blocks", {})[names[k]] = {
            "kind": ks, "entry": [round(float(x), 2) for x in rel[:, 0]], "ready": [round(float(x), 2) for x in rel[:, 1]],
            "products": [round(float(x), 2) for x in rel[:, 2]], "exit": [round(float(x), 2) for x in rel[:, 3]],
            "p4": [round(float(x), 2) if st[k, i, 4] > 0 else None for i, x in enumerate(rel[:, 4])]}
    gaps = [(st[k + 1, :grids[k + 1], 0].min() - st[k, :grids[k], 3].max()) / 100.0 for k in range(2)]
    res["gaps_us"] = {"fwd_exit_to_mid_entry": gaps[0], "mid_exit_to_wgrad_entry": gaps[1]}
    txt = json.dumps(res, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "blocks"}, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
