"""Per-block start offsets and durations of the SAC weight-gradient pass (timing build, -DSACF_PHASE_TIMING):
MFMA tiles by matrix, VALU blocks, the scalar block; median over steps. Diagnostics only.
Usage: SACFUSED_LIB=ast_sac_amd/lib/abl/libsac_TIMING.so python scripts/sac_wg_blocks.py [B]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SACFUSED_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ast_sac_amd",
                                                   "lib", "abl", "libsac_TIMING.so"))
from ast_sac_amd import sacfused  # noqa: E402
from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp  # noqa: E402
from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy  # noqa: E402
from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer  # noqa: E402
from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer  # noqa: E402

MHZ = 100.0


class _Env:
    class action_space:
        shape = (1,)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    q = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[256, 256]).to(dev) for _ in range(4)]
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[256, 256]).to(dev)
    rb = DeviceReplayBuffer(100000, 8, 1, dev)
    n = 20000
    rb.add_batch(torch.randn(n, 8, device=dev) * 1000, torch.rand(n, 1, device=dev) * 2 - 1, torch.randn(n, 1, device=dev),
                 torch.randn(n, 8, device=dev) * 1000, (torch.rand(n, 1, device=dev) < 0.1).float())
    tr = FusedSACTrainer(env=_Env, policy=pol, qf1=q[0], qf2=q[1], target_qf1=q[2], target_qf2=q[3], batch_size=B,
                         use_graph=True, backend="hip", discount=0.965, soft_target_tau=1e-3, policy_lr=8e-5,
                         qf_lr=8e-5, reward_scale=0.75, action_reg_coeff=0.01, clip_val=100.0)
    L = sacfused.load_library()
    L.sacf_debug_wg_blocks.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_void_p]
    wbuf = (C.c_ulonglong * (1024 * 16))()
    wst = []
    buf = (C.c_ulonglong * 3072)()
    nm, nb = C.c_int(), C.c_int()
    starts, ends, xcc = [], [], None
    tr.train_from_buffer(rb, 5)
    for it in range(40):
        tr.train_from_buffer(rb, 1)
        torch.cuda.synchronize()
        assert L.sacf_debug_wg_blocks(tr._sf.h, C.cast(buf, C.c_void_p), C.byref(nm), C.byref(nb), C.cast(wbuf, C.c_void_p)) == 0
        a = np.array(buf[:], dtype=np.int64).reshape(-1, 3)[:nb.value]
        t0 = a[:, 0].min()
        starts.append((a[:, 0] - t0) / MHZ)
        ends.append((a[:, 1] - t0) / MHZ)
        xcc = a[:, 2]
        w = np.array(wbuf[:], dtype=np.int64).reshape(1024, 4, 4)[:nm.value]
        wst.append((w - t0) / MHZ)
    s, e = np.median(np.array(starts), 0), np.median(np.array(ends), 0)
    d = e - s
    n_mfma, n_blocks = nm.value, nb.value
    tiles = n_mfma // 3
    groups = {"mfma actor W2": range(0, tiles), "mfma Q1 W2": range(tiles, 2 * tiles),
              "mfma Q2 W2": range(2 * tiles, 3 * tiles), "valu": range(n_mfma, n_blocks - 1),
              "scalar": range(n_blocks - 1, n_blocks)}
    print(f"B={B}: weight-gradient pass, {n_blocks} blocks ({n_mfma} MFMA tiles), us (median of {len(starts)} steps)")
    print(f"  kernel span (first start -> last end): {e.max():.2f}")
    for k, r in groups.items():
        r = list(r)
        print(f"  {k:14s} n {len(r):4d} start med {np.median(s[r]):6.2f} max {s[r].max():6.2f} | dur med "
              f"{np.median(d[r]):6.2f} max {d[r].max():6.2f} | end max {e[r].max():6.2f}")
    slow = np.argsort(-e)[:8]
    print("  last-ending blocks:", [(int(b), round(float(s[b]), 2), round(float(d[b]), 2), int(xcc[b])) for b in slow])
    per_x = [round(float(np.median(d[xcc == x])), 2) if (xcc == x).any() else None for x in range(8)]
    print("  median duration by XCC:", per_x)
    W = np.median(np.array(wst), 0)  # [block][wave][stage] from the pass's first start
    for wv in range(4):
        print(f"  MFMA tiles wave {wv}: loaded {np.median(W[:, wv, 0]):6.2f} mfma issued {np.median(W[:, wv, 1]):6.2f} "
              f"split-K read {np.median(W[:, wv, 2]):6.2f} done {np.median(W[:, wv, 3]):6.2f} (max {W[:, wv, 3].max():6.2f})")


if __name__ == "__main__":
    main()
