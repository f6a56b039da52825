"""SAC grad-steps/s of the hip backend, five launches vs the persistent single launch (libsacfused
step_kernel 0 / 1), graph-replayed steps from a 300k DeviceReplayBuffer, runner networks 2x256.
Usage: python scripts/sac_ab.py [steps] > out.json"""
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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    dev = torch.device("cuda", 0)
    rb = DeviceReplayBuffer(300000, 8, 1, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    n = 65536
    rb.add_batch(torch.randn(n, 8, device=dev, generator=g) * 1000, torch.rand(n, 1, device=dev, generator=g) * 2 - 1,
                 torch.randn(n, 1, device=dev, generator=g), torch.randn(n, 8, device=dev, generator=g) * 1000,
                 (torch.rand(n, 1, device=dev, generator=g) < 0.1).float())
    res, status = {}, {}
    for B in (256, 64, 1024):
        for variant in ("five_launches", "persistent", "persistent_full_barrier", "five_launches", "persistent"):
            persistent = variant != "five_launches"
            if variant == "persistent_full_barrier":
                os.environ["SACF_FULL_BARRIER"] = "1"
            else:
                os.environ.pop("SACF_FULL_BARRIER", None)
            torch.manual_seed(0)
            q = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[256, 256]).to(dev) for _ in range(4)]
            pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[256, 256]).to(dev)
            tr = FusedSACTrainer(env=_Env, policy=pol, qf1=q[0], qf2=q[1], target_qf1=q[2], target_qf2=q[3],
                                 discount=0.965, soft_target_tau=1e-3, policy_lr=8e-5, qf_lr=8e-5, reward_scale=0.75,
                                 action_reg_coeff=0.01, clip_val=100.0, batch_size=B, backend="hip",
                                 persistent_kernel=persistent)
            tr.train_from_buffer(rb, 20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.train_from_buffer(rb, steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            key = f"B{B}_{variant}"
            try:
                tr._sf.step_kernel_status()
            except Exception as e:  # noqa: BLE001  (reported, the timing kept)
                status[key] = str(e)
            res.setdefault(key, []).append(steps / dt)
    print(json.dumps({k: dict(grad_steps_per_s=max(v), runs=v, us_per_step=1e6 / max(v), status=status.get(k, "ok"))
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
