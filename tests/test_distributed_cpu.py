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


# ------------------------------------------------------------------------------------------------
# replicated data parallel: every rank trains on the union of all ranks' transitions
# ------------------------------------------------------------------------------------------------
N_ROWS, RB_SEED, BG = 40, 11, 2 * B


def _rank_rows(rank):
    g = torch.Generator().manual_seed(1000 + rank)
    return (torch.randn(N_ROWS, 8, generator=g) * 100, torch.rand(N_ROWS, 1, generator=g) * 2 - 1,
            torch.randn(N_ROWS, 1, generator=g), torch.randn(N_ROWS, 8, generator=g) * 100,
            (torch.rand(N_ROWS, 1, generator=g) < 0.3).float())


def _noise():
    g = torch.Generator().manual_seed(77)
    return [torch.randn(2 * BG, 1, generator=g) for _ in range(STEPS)]


def _replicated_worker(rank, world, port, out_dir):
    from ast_sac_amd.ast_sac.data_management.replay_buffer import ReplicatedReplayBuffer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pol, qs = _make(seed=100 + rank)
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    tr = FusedSACTrainer(env=_Env, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2], target_qf2=qs[3],
                         discount=0.965, reward_scale=0.75, policy_lr=3e-3, qf_lr=3e-3, soft_target_tau=0.05,
                         action_reg_coeff=0.01, clip_val=100.0, batch_size=BG, use_graph=False,
                         process_group=dist.group.WORLD, replicated=True)
    assert tr.world == 1 and not tr.split
    tr.broadcast_parameters(0)
    rb = ReplicatedReplayBuffer(1000, 8, 1, "cpu", dist.group.WORLD, stage_size=64,
                                generator=torch.Generator().manual_seed(RB_SEED))
    o, a, r, no, t = _rank_rows(rank)
    keep = torch.arange(N_ROWS) % 4 != rank  # a masked add, as the collector's
    rb.add_batch(o, a, r, no, t, mask=keep)
    assert rb.num_steps_can_sample() == 0  # staged only
    n = rb.sync()
    assert n == rb.num_steps_can_sample() == 2 * int(keep.sum())
    noise = _noise()
    cur = {}
    tr.noise_fn = lambda shape: cur["eps"]
    for s in range(STEPS):
        cur["eps"] = noise[s]
        tr.train_from_buffer(rb, 1)
    np.save(os.path.join(out_dir, f"rep{rank}.npy"), _params(tr))
    np.save(os.path.join(out_dir, f"rows{rank}.npy"), rb._observations[:n].numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_replicated_dp_sac_equals_single_process_on_the_union():
    """Two gloo ranks with different local transitions and different initial networks: after sync() both hold
    the union (rank order) and, with the broadcast parameters and the common batch seed, their SAC steps give
    bitwise the parameters of ONE process training on that union with the whole global batch."""
    import tempfile
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_replicated_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        r0, r1 = np.load(os.path.join(d, "rep0.npy")), np.load(os.path.join(d, "rep1.npy"))
        rows0, rows1 = np.load(os.path.join(d, "rows0.npy")), np.load(os.path.join(d, "rows1.npy"))
    np.testing.assert_array_equal(r0, r1)
    np.testing.assert_array_equal(rows0, rows1)
    pol, qs = _make(seed=100)
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    tr = FusedSACTrainer(env=_Env, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2], target_qf2=qs[3],
                         discount=0.965, reward_scale=0.75, policy_lr=3e-3, qf_lr=3e-3, soft_target_tau=0.05,
                         action_reg_coeff=0.01, clip_val=100.0, batch_size=BG, use_graph=False)
    rb = DeviceReplayBuffer(1000, 8, 1, "cpu", generator=torch.Generator().manual_seed(RB_SEED))
    for rank in range(world):
        o, a, r, no, t = _rank_rows(rank)
        rb.add_batch(o, a, r, no, t, mask=torch.arange(N_ROWS) % 4 != rank)
    np.testing.assert_array_equal(rows0, rb._observations[:rb.num_steps_can_sample()].numpy())
    noise = _noise()
    cur = {}
    tr.noise_fn = lambda shape: cur["eps"]
    for s in range(STEPS):
        cur["eps"] = noise[s]
        tr.train_from_buffer(rb, 1)
    np.testing.assert_array_equal(r0, _params(tr))
