"""C4 combined loop: the runner's device experiment on one GPU — 8192 envs
(the per-GPU shard of C4's 65,536), collav sbmpc, PTI machinery, policy sampling on the device,
device replay buffer, FusedSACTrainer (B = 256) — timed phase by phase:

  collect   exploration decisions with the policy in the loop (env-ticks/s, decisions/s)
  sac       grad steps alone (grad-steps/s)
  runner    DeviceBatchRLAlgorithm's train loop as configured (collect >= 256 decisions, 240 grad steps)
  ratio     the reference ratio held exactly: after every collection pass of D decisions,
            round(D * 240 / 256) grad steps (runner :66-72) — decisions/s and env-ticks/s of the loop

Usage: python scripts/c4_loop.py [n_envs] > out.json   (one JSON line)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ast_sac_amd.ast_sac.torch.utils import pytorch_util as ptu  # noqa: E402
from ast_sac_amd.run.ast_sac_runner import experiment_device, make_variant, parse_cli_args  # noqa: E402


def progress(msg):
    print(f"[c4 {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    n_envs = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    args = parse_cli_args(["--n_envs", str(n_envs), "--do_logging", "False", "--seed", "0"])
    ptu.set_gpu_mode(True, 0)
    torch.cuda.set_device(0)
    algo = experiment_device(make_variant(args), args, ptu.device)
    coll, rb, tr = algo.expl_data_collector, algo.replay_buffer, algo.trainer

    def counters():
        d = coll.get_diagnostics()
        return d["num steps total"], coll.device_diagnostics()["num env ticks total"]

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return r, time.perf_counter() - t0

    ticks0 = coll.max_ticks
    res = dict(workload=f"C4 shard: {n_envs} envs/GPU, collav sbmpc, PTI, dt 4, {ticks0}-tick "
                        f"{'fused' if coll.fused else 'sliced'} passes, SAC B={args.batch_size} 2x{args.layer_size}")
    # epoch-0 initial exploration (min_num_steps_before_training) fills the buffer; also warms up
    coll.collect(args.min_num_steps_before_training, rb)
    tr.train_from_buffer(rb, 20)
    # collect alone
    s0, k0 = counters()
    _, t = timed(lambda: coll.collect(8 * n_envs, rb))
    s1, k1 = counters()
    res["collect"] = dict(decisions=s1 - s0, env_ticks=k1 - k0, seconds=t, decisions_per_s=(s1 - s0) / t,
                          env_ticks_per_s=(k1 - k0) / t)
    res["collect"]["fused"] = coll.fused
    fused0 = coll.fused
    # sliced passes (policy launch + env slice; an env idles after its decision until the pass ends) and,
    # when the env library can run the policy, fused passes (policy inside the env launch)
    for fused in ([False, True] if fused0 else [False]):
        coll.fused = fused
        for sl in ((128, 256, 512, 1024, 2048) if fused else (32, 64, 128, 256, 512)):
            coll.max_ticks = sl
            coll.collect(4 * n_envs, rb)  # warm-up (graph capture of this slice length)
            s0, k0 = counters()
            _, t = timed(lambda: coll.collect(32 * n_envs, rb))
            s1, k1 = counters()
            progress(f"collect {'fused' if fused else 'sliced'} {sl}")
            res[f"collect_{'fused' if fused else 'sliced'}{sl}"] = dict(
                decisions=s1 - s0, env_ticks=k1 - k0, seconds=t, decisions_per_s=(s1 - s0) / t,
                env_ticks_per_s=(k1 - k0) / t)
        if fused:  # the launch tail (shipsim_set_stream_tail): envs of waves that met the pass's ticks tick on
            for sl, tail in ((1024, 512), (1024, 1024)):
                coll.max_ticks, coll.stream_tail = sl, tail
                coll.collect(4 * n_envs, rb)
                s0, k0 = counters()
                _, t = timed(lambda: coll.collect(32 * n_envs, rb))
                s1, k1 = counters()
                progress(f"collect fused {sl} tail {tail}")
                res[f"collect_fused{sl}_tail{tail}"] = dict(
                    decisions=s1 - s0, env_ticks=k1 - k0, seconds=t, decisions_per_s=(s1 - s0) / t,
                    env_ticks_per_s=(k1 - k0) / t)
            coll.stream_tail = 0
    coll.fused = fused0
    coll.max_ticks = ticks0
    # SAC alone
    n_sac = 2400
    _, t = timed(lambda: tr.train_from_buffer(rb, n_sac))
    res["sac"] = dict(grad_steps=n_sac, seconds=t, grad_steps_per_s=n_sac / t)
    progress(f"sac {n_sac / t:.0f} grad steps/s")
    # the runner's train loop as configured
    loops = 20
    s0, k0 = counters()
    _, t = timed(lambda: [(coll.collect(args.num_expl_steps_per_train_loop, rb),
                           tr.train_from_buffer(rb, args.num_trains_per_train_loop)) for _ in range(loops)])
    s1, k1 = counters()
    g = loops * args.num_trains_per_train_loop
    res["runner"] = dict(loops=loops, decisions=s1 - s0, env_ticks=k1 - k0, grad_steps=g, seconds=t,
                         decisions_per_s=(s1 - s0) / t, env_ticks_per_s=(k1 - k0) / t, grad_steps_per_s=g / t)
    # the reference ratio held exactly
    s0, k0 = counters()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = 0
    while True:
        before = counters()[0]
        coll.collect(1, rb)
        d = counters()[0] - before
        n = int(round(d * args.num_trains_per_train_loop / args.num_expl_steps_per_train_loop))
        tr.train_from_buffer(rb, n)
        g += n
        if time.perf_counter() - t0 > 20.0:
            break
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    s1, k1 = counters()
    res["ratio"] = dict(decisions=s1 - s0, env_ticks=k1 - k0, grad_steps=g, seconds=t,
                        decisions_per_s=(s1 - s0) / t, env_ticks_per_s=(k1 - k0) / t, grad_steps_per_s=g / t,
                        grad_steps_per_decision=g / max(1, s1 - s0))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
