"""Phase breakdown of the SAC kernels (timing build: scripts/build_timing.sh, -DSACF_PHASE_TIMING):
per kernel, wall-clock deltas of block (0, 0)'s first wave between the SAC_T stamps, median over steps.
Diagnostics only. Usage: SACFUSED_LIB=ast_sac_amd/lib/abl/libsac_TIMING.so python scripts/sac_phase_timing.py"""
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

NAMES = ["actor_fwd", "critic_fwd", "critic_bwd", "actor_bwd", "wgrad"]
MHZ = 100.0  # gfx9 wall clock (s_memrealtime) rate


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
                         use_graph=False, backend="hip", discount=0.965, soft_target_tau=1e-3, policy_lr=8e-5,
                         qf_lr=8e-5, reward_scale=0.75, action_reg_coeff=0.01, clip_val=100.0)
    L = sacfused.load_library()
    L.sacf_debug_stamps.argtypes = [C.c_void_p]
    buf = (C.c_ulonglong * 64)()
    rows = []
    for it in range(60):
        torch.cuda.synchronize()
        assert L.sacf_debug_reset() == 0
        tr.train_from_buffer(rb, 1)
        torch.cuda.synchronize()
        assert L.sacf_debug_stamps(C.cast(buf, C.c_void_p)) == 0
        if it >= 10:
            rows.append(np.array(buf[:], dtype=np.int64))
    st = np.array(rows)
    print(f"B={B}: per-phase wall time of block (0,0) wave 0, us (median of {len(rows)} steps)")
    for k, name in enumerate(NAMES):
        s = st[:, k * 12:(k + 1) * 12]
        idx = [i for i in range(12) if (s[:, i] != 0).all()]
        if name == "wgrad":
            groups = [[0, 1, 2, 3], [6, 7, 8]]
        elif name == "critic_fwd":
            groups = [[0, 6, 7, 8, 1, 2, 3, 4, 5]]
        else:
            groups = [[i for i in idx if i < 9]]
        for g in groups:
            g = [i for i in g if i in idx]
            d = [float(np.median(s[:, g[j + 1]] - s[:, g[j]])) / MHZ for j in range(len(g) - 1)]
            tot = float(np.median(s[:, g[-1]] - s[:, g[0]])) / MHZ
            print(f"  {name:10s} stamps {g}: " + " ".join(f"{x:6.2f}" for x in d) + f"  | total {tot:6.2f}")
        span = float(np.median(s[:, 10] - s[:, 9])) / MHZ
        last = np.bincount((s[:, 11] & 4095).astype(np.int64)).argmax() if name == "wgrad" else -1
        print(f"  {name:10s} all blocks: first start -> last end {span:6.2f}" +
              (f" (most often last: block {last})" if last >= 0 else ""))
    t0 = st[:, 9]
    print("  kernel starts relative to actor_fwd, us: " + " ".join(
        f"{NAMES[k]} {float(np.median(st[:, k * 12 + 9] - t0)) / MHZ:6.2f}" for k in range(5)))


if __name__ == "__main__":
    main()
