"""SAC grad-step rate with the Adam update fused into the weight-gradient kernel (default, one rank) vs a
separate apply kernel (split_update=True), B = 64 / 256. Timing only. Usage: python scripts/sac_wg_ab.py [steps]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp  # noqa: E402
from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy  # noqa: E402
from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer  # noqa: E402
from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer  # noqa: E402


class _Env:
    class action_space:
        shape = (1,)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    only = sys.argv[2] if len(sys.argv) > 2 else None
    dev = torch.device("cuda", 0)
    rb = DeviceReplayBuffer(300000, 8, 1, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    n = 65536
    rb.add_batch(torch.randn(n, 8, device=dev, generator=g) * 1000, torch.rand(n, 1, device=dev, generator=g) * 2 - 1,
                 torch.randn(n, 1, device=dev, generator=g), torch.randn(n, 8, device=dev, generator=g) * 1000,
                 (torch.rand(n, 1, device=dev, generator=g) < 0.1).float())
    res = {}
    for B in (256, 64):
        for split in (False, True, False, True):
            if only is not None and str(split) != only:
                continue
            torch.manual_seed(0)
            q = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[256, 256]).to(dev) for _ in range(4)]
            pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[256, 256]).to(dev)
            tr = FusedSACTrainer(env=_Env, policy=pol, qf1=q[0], qf2=q[1], target_qf1=q[2], target_qf2=q[3],
                                 discount=0.965, soft_target_tau=1e-3, policy_lr=8e-5, qf_lr=8e-5, reward_scale=0.75,
                                 action_reg_coeff=0.01, clip_val=100.0, batch_size=B, backend="hip", split_update=split)
            tr.train_from_buffer(rb, 20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.train_from_buffer(rb, steps)
            torch.cuda.synchronize()
            res.setdefault(f"B{B}_{'split' if split else 'fused'}", []).append(steps / (time.perf_counter() - t0))
    print(json.dumps({k: dict(grad_steps_per_s=max(v), us_per_step=1e6 / max(v)) for k, v in res.items()}))


if __name__ == "__main__":
    main()
