"""The data-parallel SAC step through RCCL on the hardware: a world-size-1 "nccl"
process group (RCCL) drives FusedSACTrainer's split path — libsacfused sacf_grads | torch.distributed all_reduce of the flat
gradient | sacf_apply, captured in one HIP graph (and eagerly, use_graph False) — the exact code N ranks run, and it must equal the fused single-rank step (where Adam
runs inside the weight-gradient kernel). SURVEY.md §8(e); sac.py:102-154. Needs an MI355X."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from test_gpu_distributed import _data, _make, _params, _run, B

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _trainer(pol, qs, pg, split, use_graph):
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    return FusedSACTrainer(env=_Env, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2],
                           target_qf2=qs[3], discount=0.965, reward_scale=0.75, policy_lr=3e-3, qf_lr=3e-3,
                           soft_target_tau=0.05, action_reg_coeff=0.01, clip_val=100.0, batch_size=B,
                           use_graph=use_graph, process_group=pg, backend="hip", split_update=split)


class _Env:
    class action_space:
        shape = (1,)


def _worker(rank, port, out_dir, use_graph):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    calls = []
    real = dist.all_reduce

    def counting(t, *a, **k):
        calls.append(t.numel())
        return real(t, *a, **k)

    dist.all_reduce = counting
    pol, qs = _make(seed=100, dev=dev)
    tr = _trainer(pol, qs, dist.group.WORLD, True, use_graph)
    assert tr.split and tr.world == 1
    tr.broadcast_parameters(0)
    batches, eps = _data(1)
    _run(tr, batches, eps, slice(0, B), dev)
    if use_graph:  # sacf_grads | all_reduce | sacf_apply captured in ONE HIP graph (replays run no Python)
        assert tr.capture_collective and len(tr._graphs[1]) == 1, "grads | all-reduce | apply in one graph"
        assert calls[-1] == tr.flat_grad.numel(), calls
    else:
        assert len(calls) >= 3 and calls[-1] == tr.flat_grad.numel(), calls
    np.save(os.path.join(out_dir, "rccl.npy"), _params(tr))
    dist.all_reduce = real
    dist.destroy_process_group()


@pytest.mark.parametrize("use_graph", [True, False])
def test_rccl_split_step_equals_fused_step(tmp_path, use_graph):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    mp.spawn(_worker, args=(_free_port(), str(tmp_path), use_graph), nprocs=1, join=True)
    got = np.load(tmp_path / "rccl.npy")
    dev = torch.device("cuda", 0)
    pol, qs = _make(seed=100, dev=dev)
    tr = _trainer(pol, qs, None, False, use_graph)
    assert not tr.split
    batches, eps = _data(1)
    _run(tr, batches, eps, slice(0, B), dev)
    ref = _params(tr)
    # same kernels for the gradient; the update runs in sac_apply_kernel instead of inside the weight-
    # gradient kernel: identical fp32 expressions, so equal up to the last bit
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-7)
    print("rccl split step vs fused step: max |diff| %.3g, bitwise %s" % (np.abs(got - ref).max(),
                                                                         bool((got == ref).all())))
