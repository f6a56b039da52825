"""Data-parallel SAC on the device with the product (hip) backend: two ranks (gloo, both on the one
GPU of the box) each hold half of a global batch; FusedSACTrainer all-reduces the flat gradient
between its two HIP-graph halves (libsacfused: sacf_grads | all-reduce | sacf_apply, which divides by
world_size). After three steps both ranks must hold identical parameters equal to a single-process
hip update on the whole batch. Needs an MI355X."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

H, B, STEPS = 256, 64, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Env:
    class action_space:
        shape = (1,)


def _make(seed, dev):
    from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    torch.manual_seed(seed)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[H, H]).to(dev)
    qs = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[H, H]).to(dev) for _ in range(4)]
    return pol, qs


def _data(world):
    g = torch.Generator().manual_seed(11)
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


def _trainer(pol, qs, batch_size, pg=None, use_graph=True):
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    return FusedSACTrainer(env=_Env, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2], target_qf2=qs[3],
                           discount=0.965, reward_scale=0.75, policy_lr=3e-3, qf_lr=3e-3, soft_target_tau=0.05,
                           action_reg_coeff=0.01, clip_val=100.0, batch_size=batch_size, use_graph=use_graph,
                           process_group=pg, backend="hip")


def _params(tr):
    return torch.cat([tr.flat_param, tr.flat_target]).detach().cpu().numpy()


def _run(tr, batches, eps, sl, dev):
    cur = {}
    tr.noise_fn = lambda shape: cur["eps"]
    for s in range(STEPS):
        cur["eps"] = torch.cat([eps[s][0][sl], eps[s][1][sl]], 0).to(dev)
        tr.train_from_torch({k: v[sl].to(dev) for k, v in batches[s].items()})
    torch.cuda.synchronize(dev)


def _worker(rank, world, port, out_dir, use_graph):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pol, qs = _make(seed=100 + rank, dev=dev)  # different init per rank: the broadcast must fix it
    tr = _trainer(pol, qs, B, dist.group.WORLD, use_graph)
    assert tr.backend == "hip" and tr.world == world
    tr.broadcast_parameters(0)
    batches, eps = _data(world)
    _run(tr, batches, eps, slice(rank * B, (rank + 1) * B), dev)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), _params(tr))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("use_graph", [True, False])
def test_hip_dp_sac_matches_single_process_full_batch(tmp_path, use_graph):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), use_graph), nprocs=world, join=True)
    r0 = np.load(tmp_path / "rank0.npy")
    r1 = np.load(tmp_path / "rank1.npy")
    np.testing.assert_array_equal(r0, r1)

    dev = torch.device("cuda", 0)
    pol, qs = _make(seed=100, dev=dev)
    tr = _trainer(pol, qs, B * world, use_graph=use_graph)
    batches, eps = _data(world)
    _run(tr, batches, eps, slice(0, B * world), dev)
    ref = _params(tr)
    # same math, different fp32 summation order over the rows (B + B vs 2B)
    # (Adam normalises each step: an element whose gradient is ~1e-8 moves by up to lr either way, so
    # the bound is 1e-5 absolute = 0.3 % of one step of lr 3e-3)
    np.testing.assert_allclose(r0, ref, rtol=2e-5, atol=1e-5)
