"""The default multi-rank C4 shape on the hardware: replicated data parallel —
every rank keeps the union of all ranks' transitions in a ReplicatedReplayBuffer (the graph-captured collector
stages its rows, sync() all-gathers them after every collect) and runs the same global-batch FusedSACTrainer step
(replicated=True, hip backend) with the broadcast seed; reference: data_management/simple_replay_buffer.py:70-84,
core/batch_rl_algorithm.py:81-106, run/ast-sac_runner.py:55,66-72.

* RCCL, world size 1: the runner's device experiment (ast_sac_runner.experiment_device with an "nccl" process
  group, so the replicated buffer, its RCCL syncs and the replicated trainer are the ones N ranks run) through
  DeviceBatchRLAlgorithm equals the same experiment in one process without a group, bit for bit: parameters,
  targets, Adam moments, step counter and the replay ring.
* two ranks (gloo, both on the one GPU of the box): different seeds, so the ranks collect different transitions;
  after training (runs of 8 grad steps replay the multi-step graph) both ranks hold the same ring and bitwise the
  same parameters, targets and Adam state.
Needs an MI355X."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_ENVS = 256


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _args(seed):
    from ast_sac_amd.run.ast_sac_runner import parse_cli_args
    return parse_cli_args(["--n_envs", str(N_ENVS), "--num_epochs", "2", "--min_num_steps_before_training", "512",
                           "--num_expl_steps_per_train_loop", "256", "--num_eval_steps_per_epoch", "64",
                           "--do_logging", "false", "--seed", str(seed)])


def _train(seed, dev, pg):
    """The runner's device experiment for `seed` (main(): torch / numpy seeded with seed + rank), trained."""
    from ast_sac_amd.run.ast_sac_runner import make_variant, experiment_device
    args = _args(seed)
    torch.manual_seed(seed)
    np.random.seed(seed)
    algo = experiment_device(make_variant(args), args, dev, pg)
    algo.log_stats = False
    algo.train()
    torch.cuda.synchronize(dev)
    tr, rb = algo.trainer, algo.replay_buffer
    n = rb.num_steps_can_sample()
    st = {k: v.detach().cpu().numpy() for k, v in (("param", tr.flat_param), ("target", tr.flat_target),
                                                   ("m", tr._adam_m), ("v", tr._adam_v), ("step", tr._step_t))}
    st["rows"] = torch.cat([rb._observations[:n], rb._actions[:n], rb._rewards[:n], rb._next_obs[:n],
                            rb._terminals[:n]], 1).cpu().numpy()
    st["grad_steps"] = np.array([algo.num_train_steps_total])
    return algo, st


def _noise_seed(algo):
    return algo.expl_data_collector._device_policy.seed


def _rccl_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from ast_sac_amd.ast_sac.data_management.replay_buffer import ReplicatedReplayBuffer
    algo, st = _train(5, dev, dist.group.WORLD)
    assert isinstance(algo.replay_buffer, ReplicatedReplayBuffer) and algo.trainer.replicated
    assert dist.get_backend(algo.replay_buffer.pg) == "nccl"
    assert algo.expl_data_collector.fused and algo.expl_data_collector.use_graph
    np.savez(os.path.join(out_dir, "rccl.npz"), **st)
    dist.destroy_process_group()


def test_replicated_rccl_world1_equals_single_process(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    mp.spawn(_rccl_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    got = dict(np.load(tmp_path / "rccl.npz"))
    from ast_sac_amd.ast_sac.data_management.replay_buffer import ReplicatedReplayBuffer
    algo, ref = _train(5, torch.device("cuda", 0), None)
    assert not isinstance(algo.replay_buffer, ReplicatedReplayBuffer) and not algo.trainer.replicated
    assert ref["grad_steps"][0] >= 2 * algo.trainer.GRAPH_STEPS
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    print(f"\n[replicated, RCCL world 1] {ref['rows'].shape[0]} ring rows, {ref['grad_steps'][0]} grad steps: "
          f"bitwise equal to the single-process run")


def _gloo_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    algo, st = _train(5 + rank, dev, dist.group.WORLD)  # main(): seed + rank (different policy noise and nets)
    assert algo.trainer.replicated and algo.trainer.world == 1 and not algo.trainer.split
    np.save(os.path.join(out_dir, f"noise{rank}.npy"), np.array([_noise_seed(algo)], dtype=np.int64))
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **st)
    dist.barrier()
    dist.destroy_process_group()


def test_replicated_two_ranks_stay_bitwise_equal(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    world = 2
    mp.spawn(_gloo_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [dict(np.load(tmp_path / f"rank{k}.npz")) for k in range(world)]
    for k in r[0]:
        np.testing.assert_array_equal(r[0][k], r[1][k], err_msg=k)
    rows = r[0]["rows"]
    assert r[0]["grad_steps"][0] >= 2 * 8  # the multi-step graph ran
    # the ring is the union of two different collections (each rank's exploration noise has its own seed)
    assert np.load(tmp_path / "noise0.npy")[0] != np.load(tmp_path / "noise1.npy")[0]
    assert rows.shape[0] >= 2 * 512
    print(f"\n[replicated, 2 gloo ranks on one GPU] {rows.shape[0]} ring rows, {r[0]['grad_steps'][0]} grad steps: "
          f"ranks bitwise equal (parameters, targets, Adam m / v, step, ring)")
