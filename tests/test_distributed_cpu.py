"""Data-parallel SAC on CPU with gloo, world_size 2.

Each rank holds half of a global batch; FusedSACTrainer averages the flat gradient bucket with one
all-reduce per step. The result must equal a single-process update on the whole batch (the mean
loss over 2B rows is the average of the two B-row means), and the ranks must stay identical.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

H, B, STEPS = 32, 16, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Env:
    class action_space:
        shape = (1,)


def _make(seed):
    from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    torch.manual_seed(seed)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[H, H])
    qs = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[H, H]) for _ in range(4)]
    return pol, qs


def _data(world):
    g = torch.Generator().manual_seed(5)
    Bg = B * world
    batches, eps = [], []
    for _ in range(STEPS):
        batches.append(dict(observations=torch.randn(Bg, 8, generator=g) * 100,
                            actions=torch.rand(Bg, 1, generator=g) * 2 - 1,
                            rewards=torch.randn(Bg, 1, generator=g),
                            terminals=(torch.rand(Bg, 1, generator=g) < 0.3).float(),
                            next_observations=torch.randn(Bg, 8, generator=g) * 100))
        eps.append((torch.randn(Bg, 1, generator=g), torch.randn(Bg, 1, generator=g)))
    return batches, eps


def _trainer(pol, qs, batch_size, pg=None):
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    return FusedSACTrainer(env=_Env, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2], target_qf2=qs[3],
                           discount=0.965, reward_scale=0.75, policy_lr=3e-3, qf_lr=3e-3, soft_target_tau=0.05,
                           action_reg_coeff=0.01, clip_val=100.0, batch_size=batch_size, use_graph=False,
                           process_group=pg)


def _params(tr):
    return torch.cat([p.detach().reshape(-1) for p in tr.pi_params + tr.q_params + tr.t_params]).numpy()


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pol, qs = _make(seed=100 + rank)  # different init per rank: broadcast must fix it
    tr = _trainer(pol, qs, B, dist.group.WORLD)
    tr.broadcast_parameters(0)
    batches, eps = _data(world)
    cur = {}
    tr.noise_fn = lambda shape: cur["eps"]
    sl = slice(rank * B, (rank + 1) * B)
    for s in range(STEPS):
        cur["eps"] = torch.cat([eps[s][0][sl], eps[s][1][sl]], 0)
        tr.train_from_torch({k: v[sl] for k, v in batches[s].items()})
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), _params(tr))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_sac_matches_single_process_full_batch(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = np.load(tmp_path / "rank0.npy")
    r1 = np.load(tmp_path / "rank1.npy")
    np.testing.assert_array_equal(r0, r1)

    pol, qs = _make(seed=100)
    tr = _trainer(pol, qs, B * world)
    batches, eps = _data(world)
    cur = {}
    tr.noise_fn = lambda shape: cur["eps"]
    for s in range(STEPS):
        cur["eps"] = torch.cat([eps[s][0], eps[s][1]], 0)
        tr.train_from_torch(batches[s])
    np.testing.assert_allclose(r0, _params(tr), rtol=2e-5, atol=2e-6)
