"""Headline benchmark: batched two-ship AST env-steps/sec (BASELINE.json metric) on 1..8 MI355X.

A "step" is one launch over every env of every rank in which each env runs `--slice` (4096, about
four episodes) `_step` ticks of the C3 decision stream: decisions (tick until RoA + 1 tick,
or done; ≈130 env-ticks per decision at dt = 4 s) with scoping angles from a device-resident
synthetic table U(-1, 1) (PCG64 seeded per rank, NormalizedBoxEnv's float32 rule), 9 decisions per
episode (max_path_length), auto-reset on episode end. Default --mode table runs it with
shipsim_run_table (a completed decision is followed at once by the next, episodes reset inside
the kernel, every decision's result written to a per-env record ring); --mode step drives the
same stream from the host with shipsim_step slices + masked shipsim_reset between launches (the
RL collector's call pattern, where the policy picks the next action). Both give identical
per-decision results (tests/test_gpu_table.py). Launch length matters because the launch ends
with its slowest wave: per-wave cost varies with SBMPC activity (waves whose envs are inside 2 km
of the obstacle ship do ~2x the work), and that variance averages out over longer launches
(sbmpc: 128 ticks 251 M, 512 369 M, 1024 446 M, 2048 483 M, 4096 511-513 M env-ticks/s;
profiles/round1_sweeps.md).

value = env-ticks (one `_step` of one env, both ships + reward/termination) summed over all ranks
        / max-over-ranks wall time of the K timed steps.

Workload (config C3, BASELINE.json configs[2]): 4096 two-ship AST envs per GPU, ShipModelAST
with PTI machinery, HeadingBySampledRouteController, reward_designs, collav = sbmpc (the runner
default, run/ast-sac_runner.py:35), dt = 4 s. Weak scaling: envs per GPU fixed.

Launch:  python bench.py                       (N = 1)
         python bench.py --gpus N              (spawns N ranks itself: a child torch.distributed.run;
                                                this parent process never touches the GPU)
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
One rank per GPU over RCCL ("nccl"); `--dist-backend gloo` rehearses N ranks on fewer devices, and the
line then reports `ranks` (processes) and `n_gpus` (distinct physical devices) separately.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X FP64 vector spec (the resource the env kernel actually spends)
ALGO_BYTES_PER_ENV_TICK = 616  # C3/C5 detailed dynamics, one obstacle ship


def algo_bytes_per_env_tick(n_obs_ships=1):
    """SURVEY.md §8(d)'s 616 B = 2·(2·112 + 84) (ship state 112 B per ship, env state 84 B, read and
    written once per tick), for 1 + K ships."""
    return 2 * ((1 + n_obs_ships) * 112 + 84)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=6)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--envs-per-gpu", type=int, default=4096)
    p.add_argument("--collav", default="sbmpc", choices=["none", "simple", "sbmpc"])
    p.add_argument("--machinery", default="detailed", choices=["detailed", "simplified"])
    p.add_argument("--slice", type=int, default=4096,
                   help="max ticks per env per step call (0 = whole decision); table mode: ticks per env per launch")
    p.add_argument("--mode", default="table", choices=["table", "step"],
                   help="table: shipsim_run_table, decisions chained and episodes reset inside the kernel (the "
                        "C3 open-loop decision stream); step: shipsim_step slices + host-side table lookup and "
                        "masked shipsim_reset between calls (the RL collector's call pattern)")
    p.add_argument("--obs-ships", type=int, default=1,
                   help="obstacle ships per env (C5 multi-obstacle generalisation; 1 = the reference env)")
    p.add_argument("--lpe", type=int, default=0, help="device lanes per env (0 = library choice from envs per GPU)")
    p.add_argument("--tail-ticks", type=int, default=1024,
                   help="table mode: work-conserving launch tail (shipsim_set_stream_tail): waves that met --slice "
                        "keep ticking while the launch's slowest wave has not, up to this many more ticks (0 = off)")
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-c2", action="store_true", help="skip the configs[1] single-ship secondary line")
    p.add_argument("--no-policy-stream", action="store_true",
                   help="skip the secondary line of the same envs with the policy in the loop (shipsim_run_policy)")
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "round6", "r6fin_pmc_traffic.json"))
    p.add_argument("--pmc-fp64-json", default=os.path.join(ROOT, "profiles", "round6", "r6fin_pmc_fp64.json"))
    p.add_argument("--sac-steps", type=int, default=300, help="timed SAC grad steps (0 = skip the SAC line)")
    p.add_argument("--sac-global-batch", type=int, default=256,
                   help="SAC batch summed over all ranks (runner: 256); each rank samples global / N rows "
                        "(SURVEY.md §8(e))")
    p.add_argument("--dist-backend", default="nccl", help="nccl (RCCL, one GPU per rank) | gloo (rehearsal)")
    p.add_argument("--no-c4", action="store_true", help="skip the C4 leg (runner experiment at the reference ratio)")
    p.add_argument("--c4-envs", type=int, default=8192, help="C4 leg: envs per rank (C4: 65,536 over 8 GPUs)")
    p.add_argument("--c4-loops", type=int, default=3, help="C4 leg: timed train loops")
    p.add_argument("--no-c5", action="store_true", help="skip the C5 legs (K = 2 and 4 obstacle ships, sbmpc)")
    return p.parse_args()


def host_threads():
    """Threads for the CPU baseline: every core this process may run on (the box's CPU share,
    OMP_NUM_THREADS when the launcher sets it)."""
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return (omp or avail), avail


def cpu_baseline(cfg, seconds, n_threads, n_envs=4096):
    """BASELINE.md CPU-baseline plan: the oracle (the fixture-pinned C restatement) compiled here
    with -O3 -march=native, OpenMP one env per thread over every available core, on a bounded sample
    of the same workload: C3 = batches of `n_envs` two-ship AST envs x one episode each (9 decisions
    from the PCG64 table, as the GPU stream runs them), and C2 = `n_envs` single ships over the whole
    10,000 s horizon at dt 30 and dt 4 (the c2_single_ship line's workload)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_ffi as O
    from ast_sac_amd import shipsim_abi as abi
    L = O.native_lib()
    n = n_envs
    while True:
        acts = abi.normalized_to_scoping(abi.ast_action_table(n))
        t0 = time.perf_counter()
        total, ticks, dec, ret, bits = O.ast_rollouts(cfg, acts, n_threads=n_threads, L=L)
        dt = time.perf_counter() - t0
        if dt >= seconds * 0.5 or n >= 64 * n_envs:
            break
        n = n_envs * max(2 * (n // n_envs), int(np.ceil(n / n_envs * seconds * 0.6 / max(dt, 1e-3))))
    # thread scaling on a smaller sample of the same stream (one thread, then the lease's threads), for the
    # all-core figure below: envs are independent, so the rate per thread is what the extra cores would add
    small = abi.normalized_to_scoping(abi.ast_action_table(512))
    per_thread = {}
    for k in sorted({1, n_threads}):
        t0 = time.perf_counter()
        tot_k = O.ast_rollouts(cfg, small, n_threads=k, L=L)[0]
        per_thread[k] = tot_k / (time.perf_counter() - t0) / k
    eff = per_thread[n_threads] / per_thread[1]
    affinity = host_threads()[1]
    c2 = {}
    init = abi.c2_initial_states(n_envs)
    for step in (30, 4):
        c2cfg = abi.c2_config(step)
        n_ticks = int(np.ceil(c2cfg.simulation_time / step))
        t0 = time.perf_counter()
        O.c2_run(c2cfg, init, max_ticks=n_ticks, trace=False, n_threads=n_threads, L=L)
        c2[f"dt{step}"] = n_envs * n_ticks / (time.perf_counter() - t0)
    return dict(value=total / dt, unit="env-ticks/s", cores=n_threads, kind="port",
                nproc=os.cpu_count(), affinity_cpus=affinity,
                all_affinity_cores=dict(
                    value=total / dt / n_threads * affinity, cores=affinity, kind="extrapolated",
                    thread_scaling={"threads": sorted(per_thread), "env_ticks_per_s_per_thread":
                                    [per_thread[k] for k in sorted(per_thread)], "efficiency": eff},
                    note=f"measured rate per thread at {n_threads} threads x the {affinity} CPUs in affinity: the box "
                         f"leases {n_threads} threads (OMP_NUM_THREADS) and running more is not allowed there; "
                         f"envs share nothing, and per-thread efficiency {n_threads} vs 1 thread on a 512-env sample "
                         f"was {eff:.2f}"),
                sample=f"C3: {n // n_envs} x {n_envs} two-ship AST envs x 1 episode each (<=9 decisions from the "
                       f"PCG64 table), {int(total)} env-ticks in {dt:.1f} s; oracle/shipsim_oracle.c built -O3 "
                       f"-march=native, OpenMP {n_threads} threads",
                c2_ship_ticks_per_s=c2, c2_sample=f"{n_envs} single ships x whole 10,000 s horizon (dt 30, dt 4)")


MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense, = FP32 vector rate


def sac_flops_per_step(B, H, O):
    """Matrix flops (2 per multiply-add) of one SAC grad step with two hidden layers of width H, obs_dim O,
    act_dim 1 (sac.py compute_loss :156-270): forward over 2B actor rows (obs, next_obs) and 6B critic rows
    (Q1/Q2 at (obs, a) and (obs, ã), targets at (next_obs, ã')); backward through the critics at (obs, a)
    for the Q losses and (obs, ã) for the policy loss (4B rows, down to dQ/dã), through the actor at obs
    (B rows); weight gradients of policy (B rows) and both critics (B rows each)."""
    mac_fwd = 2 * B * (H * O + H * H + 2 * H) + 6 * B * (H * (O + 1) + H * H + H)
    mac_bwd = 4 * B * (H + H * H + H) + B * (2 * H + H * H)
    mac_wg = B * (H * O + H * H + 2 * H) + 2 * B * (H * (O + 1) + H * H + H)
    return 2 * (mac_fwd + mac_bwd + mac_wg)


def bench_sac(dev, world, pg, steps, global_batch, eager_steps=40, graph=True, dp_mode="replicated"):
    """SAC grad-steps/s (secondary metric): FusedSACTrainer HIP-graph step (runner networks: 2x256 hidden, global
    batch `global_batch`, on-device uniform sampling from a 300k-row DeviceReplayBuffer), beside the reference-order
    eager SACTrainer. With world > 1: dp_mode "replicated" (the runner's default) runs the whole
    global batch on every rank over the same buffer rows (the union a ReplicatedReplayBuffer holds: filled here
    with the same seed on every rank) with no per-step collective; "allreduce" gives each rank global / world rows
    and all-reduces the flat gradient every step over RCCL (captured in the step's HIP graph)."""
    import torch
    import torch.distributed as dist
    from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac_amd.ast_sac.torch.sac.sac import SACTrainer
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer

    class _Env:
        class action_space:
            shape = (1,)

    def nets():
        torch.manual_seed(0)
        q = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[256, 256]).to(dev) for _ in range(4)]
        return TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[256, 256]).to(dev), q

    hp = dict(discount=0.965, soft_target_tau=1e-3, policy_lr=8e-5, qf_lr=8e-5, reward_scale=0.75,
              action_reg_coeff=0.01, clip_val=100.0)
    replicated = world > 1 and dp_mode == "replicated"
    batch = global_batch if (world == 1 or replicated) else global_batch // world
    rb = DeviceReplayBuffer(300000, 8, 1, dev)
    # rank-specific rows for the all-reduce shape (own shards); the same rows everywhere when replicated
    g = torch.Generator(device=dev).manual_seed(1 if replicated or world == 1 else 1 + dist.get_rank())
    n = 65536
    rb.add_batch(torch.randn(n, 8, device=dev, generator=g) * 1000, torch.rand(n, 1, device=dev, generator=g) * 2 - 1,
                 torch.randn(n, 1, device=dev, generator=g), torch.randn(n, 8, device=dev, generator=g) * 1000,
                 (torch.rand(n, 1, device=dev, generator=g) < 0.1).float())

    def timed(fn, k):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        fn(k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt)

    def fused(backend):
        pol, q = nets()
        tr = FusedSACTrainer(env=_Env, policy=pol, qf1=q[0], qf2=q[1], target_qf1=q[2], target_qf2=q[3],
                             batch_size=batch, process_group=pg, backend=backend, use_graph=graph,
                             replicated=replicated, **hp)
        tr.broadcast_parameters(0)
        tr.train_from_buffer(rb, 10)  # captures the graph
        return timed(lambda k: tr.train_from_buffer(rb, k), steps)

    dt = fused("hip")
    H, O = 256, 8
    backend = dist.get_backend(pg) if world > 1 else None
    ar = {"nccl": "RCCL all-reduce", "gloo": "gloo all-reduce (rehearsal, not RCCL)"}.get(backend, f"{backend} all-reduce")
    flops = sac_flops_per_step(batch, H, O)
    if world == 1:
        shape = "single rank"
    elif replicated:
        shape = (f"replicated x{world}: every rank runs the global-batch step over the same rows, no per-step "
                 "collective (the runner's default; its per-loop row all-gather is not in this timing)")
    else:
        shape = f"gradient all-reduce x{world}: {batch} rows per rank, {ar} of the flat gradient every step"
    res = {"grad_steps_per_s": steps / dt, "ms_per_grad_step": dt / steps * 1e3, "batch_per_gpu": batch,
           "global_batch": global_batch, "hidden": [H, H], "dtype": "f32", "dist_backend": backend,
           "dp_mode": dp_mode if world > 1 else None, "shape": shape,
           "impl": "FusedSACTrainer hip backend (csrc/sac_kernels.hip: three launches per grad step — forward, "
                   "critics on the sampled action with the action tangent + backward factors, weight gradients "
                   "with Adam / soft update / W2T refresh fused in" +
                   ("; the gradient all-reduce and a separate Adam launch inside the same HIP graph)"
                    if (world > 1 and not replicated) else "; one HIP graph)"),
           "roofline": {"bound": "mfma", "unit": "TFLOP/s", "peak": MFMA_F32_PEAK_TFLOPS,
                        "flops_per_step": flops,
                        "achieved": flops / (dt / steps) / 1e12,
                        "frac": flops / (dt / steps) / 1e12 / MFMA_F32_PEAK_TFLOPS,
                        "note": "algorithmic matrix flops of one grad step (2 per multiply-add: forward, "
                                "backward and weight-gradient products of every layer of the reference's "
                                "formulation, per rank) / whole-step wall time (every launch of the step); "
                                "v_mfma_f32_32x32x2_f32 dense f32 peak"}}
    if replicated:  # the per-train-loop cost the step timing leaves out: ReplicatedReplayBuffer.sync()
        from ast_sac_amd.ast_sac.data_management.replay_buffer import ReplicatedReplayBuffer
        per_rank = 32768  # one fused collector pass of 4096 envs stages ~8 decisions per env
        rbr = ReplicatedReplayBuffer(300000, 8, 1, dev, pg, stage_size=65536)

        def stage_and_sync(k):
            for _ in range(k):
                rbr.add_batch(torch.randn(per_rank, 8, device=dev), torch.rand(per_rank, 1, device=dev),
                              torch.randn(per_rank, 1, device=dev), torch.randn(per_rank, 8, device=dev),
                              torch.zeros(per_rank, 1, device=dev))
                rbr.sync()
        stage_and_sync(2)
        t_sync = timed(stage_and_sync, 10) / 10
        loop_steps = per_rank * world * 240 / 256  # grad steps one such loop runs at the reference's ratio
        res["replicated_sync"] = {"rows_per_rank": per_rank, "ms_per_sync": t_sync * 1e3,
                                  "us_per_grad_step": t_sync / loop_steps * 1e6,
                                  "note": "staging + two all-gathers (counts, rows) + the ring append, once per train "
                                          "loop; amortised over the loop's grad steps at the reference's 240:256 ratio"}
    if world == 1 and eager_steps:
        res["torch_ops_graph_grad_steps_per_s"] = steps / fused("torch")
    if world == 1 and eager_steps:
        pol, q = nets()
        ref = SACTrainer(env=_Env, policy=pol, qf1=q[0], qf2=q[1], target_qf1=q[2], target_qf2=q[3], **hp)

        def eager(k):
            for _ in range(k):
                ref.train_from_torch(rb.random_batch(batch))
        eager(3)
        res["reference_order_eager_grad_steps_per_s"] = eager_steps / timed(eager, eager_steps)
    return res


def bench_policy_stream(dev, cfg, n_envs, slice_ticks, launches=3, warmup=1, tail_ticks=0, hidden=256):
    """The C3 envs with the policy in the loop (secondary line): shipsim_run_policy, every decision's action
    sampled inside the launch from a TanhGaussianPolicy (runner networks 2 x `hidden`, random init, stochastic) held
    by a FusedSACTrainer — the collector's fused pass without the replay bookkeeping. env-ticks/s over
    `launches` launches of `slice_ticks` ticks (HIP events on the launch stream), with the table line's
    work-conserving launch tail of `tail_ticks` (shipsim_set_stream_tail; 0: off)."""
    import torch
    from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    from ast_sac_amd.shipsim import ShipSim
    from ast_sac_amd import shipsim_abi as abi

    class _Env:
        class action_space:
            shape = (1,)

    torch.manual_seed(0)
    q = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[hidden, hidden]).to(dev) for _ in range(4)]
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[hidden, hidden]).to(dev)
    tr = FusedSACTrainer(env=_Env, policy=pol, qf1=q[0], qf2=q[1], target_qf1=q[2], target_qf2=q[3],
                         discount=0.965, soft_target_tau=1e-3, policy_lr=8e-5, qf_lr=8e-5, reward_scale=0.75,
                         batch_size=256, backend="hip")
    dp = tr.device_policy(deterministic=False, seed=20251017)
    sim = ShipSim(cfg, n_envs, device=dev)
    sim.reset()
    if tail_ticks > 0:
        sim.set_stream_tail(tail_ticks)
    n_dec = cfg.max_sampling_frequency
    ep = torch.zeros(n_envs, dtype=torch.int32, device=dev)
    dec = torch.zeros(n_envs, dtype=torch.int32, device=dev)
    out = dict(ticks=torch.zeros(n_envs, dtype=torch.int32, device=dev),
               decisions=torch.zeros(n_envs, dtype=torch.int32, device=dev))
    ticks = torch.zeros((), dtype=torch.int64, device=dev)
    decs = torch.zeros((), dtype=torch.int64, device=dev)
    e0 = [torch.cuda.Event(enable_timing=True) for _ in range(launches)]
    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(launches)]
    for i in range(warmup + launches):
        if i == warmup:
            torch.cuda.synchronize()
            ticks.zero_()
            decs.zero_()
            t0 = time.perf_counter()
        if i >= warmup:
            e0[i - warmup].record()
        sim.run_policy(dp.weights(), slice_ticks, n_dec, ep, dec, deterministic=False, seed=dp.seed,
                       counter=dp.counter, out=out)
        if i >= warmup:
            e1[i - warmup].record()
        dp.counter.add_(1)
        ticks.add_(out["ticks"].sum())
        decs.add_(out["decisions"].sum())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms = sum(a.elapsed_time(b) for a, b in zip(e0, e1)) / launches
    res = {"env_ticks_per_s": float(ticks.item()) / dt, "decisions_per_s": float(decs.item()) / dt,
           "kernel_ms": kms, "envs": n_envs, "slice_ticks": slice_ticks, "tail_ticks": tail_ticks,
           "launches": launches,
           "lanes_per_env": sim.lanes_per_env,
           "impl": "shipsim_run_policy (ast_step_kernel CHAIN 2: TanhGaussianPolicy sample per decision in-kernel, "
                   "NormalizedBoxEnv mapping, in-place episode resets)"}
    sim.close()
    return res


def bench_c4(dev, world, rank, pg, n_envs=8192, slice_ticks=128, loops=3, warmup_loops=1, dp_mode="replicated"):
    """configs[3] (C4) as the runner runs it, at whatever N the job has: the runner's device experiment
    (ast_sac_amd/run/ast_sac_runner.py experiment_device: `n_envs` two-ship AST envs per rank, sbmpc, PTI, dt 4,
    policy sampled inside the env launch, device replay, FusedSACTrainer 2 x 256, global batch 256), then `loops`
    train loops at the reference's update ratio (run/ast-sac_runner.py:66-72, batch_rl_algorithm.py:81-106: 240 grad
    steps per 256 collected decisions, counted over ALL ranks): per loop every rank collects one fused pass of
    `slice_ticks` ticks, the replicated buffers all-gather the new rows (ReplicatedReplayBuffer.sync, RCCL over xGMI
    with nccl), and every rank runs round(decisions_all_ranks x 240 / 256) identical global-batch grad steps
    (DESIGN.md §6). Reports the job's grad steps/s (one chain, whatever N), env-ticks/s and decisions/s summed over
    the ranks, and the sync's share; the timed region is bracketed by barriers, times are the max over ranks."""
    import torch
    import torch.distributed as dist
    from ast_sac_amd.run.ast_sac_runner import experiment_device, make_variant, parse_cli_args
    argv = ["--n_envs", str(n_envs), "--do_logging", "False", "--seed", "0", "--slice_ticks", str(slice_ticks),
            "--dp_mode", dp_mode]
    args = parse_cli_args(argv)
    algo = experiment_device(make_variant(args), args, dev, pg)
    coll, rb, tr = algo.expl_data_collector, algo.replay_buffer, algo.trainer
    ak = make_variant(args)["algorithm_kwargs"]

    def counters():
        return coll.get_diagnostics()["num steps total"], coll.device_diagnostics()["num env ticks total"]

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    # epoch 0's initial exploration fills the buffers (every rank's rows into every replica)
    coll.collect(ak["min_num_steps_before_training"], rb)
    algo._sync_buffer()
    tr.train_from_buffer(rb, 20)

    def loop(k):
        t_sync = 0.0
        for _ in range(k):
            got = coll.collect(1, rb)  # one pass
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            algo._sync_buffer()
            torch.cuda.synchronize()
            t_sync += time.perf_counter() - t0
            n = algo._n_grad_steps(got)  # all ranks' decisions x 240 / 256 (an all-reduce of the count)
            if n:
                tr.train_from_buffer(rb, n)
            algo.num_train_steps_total += n
        return t_sync

    loop(warmup_loops)
    g0 = algo.num_train_steps_total
    s0, k0 = counters()
    barrier()
    t0 = time.perf_counter()
    t_sync = loop(loops)
    barrier()
    el = time.perf_counter() - t0
    s1, k1 = counters()
    grad = algo.num_train_steps_total - g0
    v = torch.tensor([el, t_sync, float(s1 - s0), float(k1 - k0)], dtype=torch.float64, device=dev)
    if world > 1:
        mx, sm = v.clone(), v.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        v = torch.stack([mx[0], mx[1], sm[2], sm[3]])
    el, t_sync, dec, ticks = (float(x) for x in v)
    res = {"grad_steps_per_s": grad / el, "env_ticks_per_s": ticks / el, "decisions_per_s": dec / el,
           "grad_steps": grad, "decisions": dec, "env_ticks": ticks, "seconds": el, "loops": loops,
           "sync_ms_per_loop": t_sync / loops * 1e3, "sync_frac": t_sync / el,
           "grad_steps_per_decision": grad / max(dec, 1.0), "ranks": world, "envs_per_rank": n_envs,
           "global_envs": n_envs * world, "slice_ticks": slice_ticks, "dp_mode": dp_mode if world > 1 else None,
           "global_batch": ak["batch_size"],
           "note": "the runner's device experiment at the reference's update ratio (240 grad steps per 256 decisions "
                   "over all ranks); per loop one fused collector pass per rank, the replicated buffers' row "
                   "all-gather, then the identical global-batch grad steps on every rank; grad steps are one serial "
                   "chain for the whole job, so they do not add up over ranks"}
    del algo, coll, rb, tr
    torch.cuda.empty_cache()
    return res


def bench_c5(dev, world, n_envs, n_obs, collav="sbmpc", slice_ticks=4096, tail_ticks=1024, launches=3, warmup=1,
             rank=0):
    """configs[4] (C5) multi-obstacle envs: the headline's decision stream (shipsim_run_table, PTI machinery, dt 4,
    bench.py's PCG64 table) with K = `n_obs` obstacle ships per env (the test ship's SBMPC over all of them,
    sbmpc.py:149-178). env-ticks/s summed over the ranks / max-over-ranks time of `launches` timed launches."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from ast_sac_amd import shipsim_abi as abi
    from ast_sac_amd.shipsim import ShipSim
    cfg = abi.ast_config(collav, machinery=abi.MACH_DETAILED, n_obs_ships=n_obs)
    sim = ShipSim(cfg, n_envs, device=dev, n_obs_ships=n_obs)
    n_dec = cfg.max_sampling_frequency
    gen = np.random.Generator(np.random.PCG64(20251015 + rank))
    table = torch.from_numpy(abi.normalized_to_scoping(gen.uniform(-1, 1, (8, n_dec, n_envs)).astype(np.float32))).to(dev)
    ep = torch.zeros(n_envs, dtype=torch.int32, device=dev)
    dec = torch.zeros(n_envs, dtype=torch.int32, device=dev)
    out = dict(ticks=torch.empty(n_envs, dtype=torch.int32, device=dev),
               decisions=torch.empty(n_envs, dtype=torch.int32, device=dev))
    cap = max(8, (slice_ticks + tail_ticks) // 32 + 16)
    log = torch.zeros((n_envs, cap, abi.DECLOG_COLS), dtype=torch.float64, device=dev)
    log_len = torch.zeros(n_envs, dtype=torch.int32, device=dev)
    sim.reset()
    if tail_ticks > 0:
        sim.set_stream_tail(tail_ticks)
    ticks = torch.zeros((), dtype=torch.int64, device=dev)
    for i in range(warmup + launches):
        if i == warmup:
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            ticks.zero_()
            t0 = time.perf_counter()
        log_len.zero_()
        sim.run_table(table, slice_ticks, ep, dec, out=out, log=log, log_len=log_len)
        ticks.add_(out["ticks"].sum())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    v = torch.tensor([time.perf_counter() - t0, float(ticks.item())], dtype=torch.float64, device=dev)
    if world > 1:
        mx, sm = v.clone(), v.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        v = torch.stack([mx[0], sm[1]])
    lpe = sim.lanes_per_env
    sim.close()
    return {"env_ticks_per_s": float(v[1]) / float(v[0]), "ms_per_launch": float(v[0]) / launches * 1e3,
            "obs_ships": n_obs, "collav": collav, "envs_per_gpu": n_envs, "slice_ticks": slice_ticks,
            "tail_ticks": tail_ticks, "launches": launches, "lanes_per_env": lpe,
            "parity": "K = 1 is the reference env; K > 1 generalises it (include/shipsim.h shipsim_create); its "
                      "SBMPC over K obstacles is pinned to the reference (tests/golden/sbmpc_multi.npz)"}


def bench_c2(dev, n_ships=4096, per_launch=None):
    """configs[1] (C2): 4096 single ships, SimpleShipModel + ThrustFromSpeedSetPoint +
    HeadingByRouteController, PCG64-perturbed initial states, the whole 10,000 s
    horizon in one shipsim_tick launch (single_tick_pipe_kernel: three waves per 64 ships); secondary line,
    ship-ticks/s."""
    import numpy as np
    import torch
    from ast_sac_amd import shipsim_abi as abi
    from ast_sac_amd.shipsim import ShipSim
    res = {"ships": n_ships, "unit": "ship-ticks/s", "kernel": "single_tick_pipe_kernel"}
    init = abi.c2_initial_states(n_ships)
    for dt in (30, 4):
        cfg = abi.c2_config(dt)
        n_ticks = int(np.ceil(cfg.simulation_time / dt))
        per = (per_launch or {})[dt] if per_launch else n_ticks  # ticks per shipsim_tick launch (default: all)
        best = None
        for rep in range(2):  # first pass warms up
            sim = ShipSim(cfg, n_ships, device=dev)
            for f, col in ((abi.F_NORTH, 0), (abi.F_EAST, 1), (abi.F_YAW, 2), (abi.F_U, 3)):
                sim.set(f, torch.from_numpy(np.ascontiguousarray(init[:, col])))
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            done = 0
            while done < n_ticks:
                k = min(per, n_ticks - done)
                sim.tick(k)
                done += k
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            sim.close()
            best = el if best is None else min(best, el)
        res[f"dt{dt}"] = n_ships * n_ticks / best
        res[f"dt{dt}_ticks"] = n_ticks
    return res


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`bench.py --gpus N` run directly: start the N ranks as ONE child process
    (torch.distributed.run, rendezvous on 127.0.0.1) and return its exit status. Nothing here has
    touched the GPU (no torch import), and the child is a fresh process, never an exec of this one."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def device_identity(torch, dev):
    """A string naming the physical GPU behind `dev`: its UUID, else its PCI domain:bus:device."""
    p = torch.cuda.get_device_properties(dev)
    uuid = str(getattr(p, "uuid", "") or "")
    if uuid and uuid.strip("0-"):
        return "uuid:" + uuid
    pci = tuple(getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if any(v is not None for v in pci):
        return "pci:%s" % (pci,)
    return "host:%s/ordinal:%d" % (os.uname().nodename, dev.index)


def rank_layout(args, torch):
    """(world, rank, local device index) of this process, checked against --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch with --gpus N alone "
                         f"(it spawns the ranks) or under torch.distributed.run --nproc-per-node {args.gpus}")
    n_dev = torch.cuda.device_count()
    if args.dist_backend == "nccl":
        if local >= n_dev:
            raise SystemExit(f"bench.py: rank {rank} needs device {local}, only {n_dev} visible (one GPU per rank "
                             f"over RCCL; use --dist-backend gloo to rehearse more ranks than devices)")
    else:  # multi-rank rehearsal on fewer GPUs than ranks
        local = local % max(1, n_dev)
    return world, rank, local


def progress(msg):
    """A phase line on stderr (the GPU box takes a run silent for minutes to be hung)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import numpy as np
    import torch
    import torch.distributed as dist
    from ast_sac_amd import shipsim_abi as abi
    from ast_sac_amd.shipsim import ShipSim

    world, rank, local = rank_layout(args, torch)
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # distinct physical devices behind the ranks (= world over RCCL; fewer under a gloo rehearsal), by
    # device identity (UUID / PCI location), not by local ordinal (a launcher may give each rank
    # HIP_VISIBLE_DEVICES=<one GPU>, where every rank sees its GPU as device 0)
    ids = [device_identity(torch, dev)]
    if world > 1:
        ids = [None] * world
        dist.all_gather_object(ids, device_identity(torch, dev))
    n_devices = len(set(ids))
    mach = abi.MACH_DETAILED if args.machinery == "detailed" else abi.MACH_SIMPLIFIED
    cfg = abi.ast_config(args.collav, machinery=mach, n_obs_ships=args.obs_ships)
    cfg.lanes_per_env = args.lpe
    N = args.envs_per_gpu
    sim = ShipSim(cfg, N, device=dev, n_obs_ships=args.obs_ships)
    bytes_per_tick = algo_bytes_per_env_tick(args.obs_ships)

    # device-resident synthetic decision table: 9 decisions per episode, new table row per episode
    n_dec = cfg.max_sampling_frequency
    table_eps = 8
    gen = np.random.Generator(np.random.PCG64(20251015 + rank))
    a_norm = gen.uniform(-1, 1, (table_eps, n_dec, N)).astype(np.float32)
    table = torch.from_numpy(abi.normalized_to_scoping(a_norm)).to(dev)  # (eps, dec, N)
    ep_idx = torch.zeros(N, dtype=torch.long, device=dev)
    dec_idx = torch.zeros(N, dtype=torch.long, device=dev)
    ar = torch.arange(N, device=dev)
    out = dict(obs=torch.empty((N, 8), dtype=torch.float32, device=dev),
               reward=torch.empty(N, dtype=torch.float64, device=dev),
               done=torch.empty(N, dtype=torch.uint8, device=dev),
               events=torch.empty(N, dtype=torch.int32, device=dev),
               ticks=torch.empty(N, dtype=torch.int32, device=dev),
               ready=torch.empty(N, dtype=torch.uint8, device=dev))
    obs_reset = torch.empty((N, 8), dtype=torch.float32, device=dev)
    total_ticks = torch.zeros((), dtype=torch.int64, device=dev)
    total_decisions = torch.zeros((), dtype=torch.int64, device=dev)
    n_ev = args.steps + args.warmup  # every launch is bracketed (warmup ones too, to compare with rocprof)
    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)]

    ep32 = torch.zeros(N, dtype=torch.int32, device=dev)
    dec32 = torch.zeros(N, dtype=torch.int32, device=dev)
    tout = dict(ticks=out["ticks"], decisions=torch.empty(N, dtype=torch.int32, device=dev))
    if args.mode == "table" and args.slice <= 0:
        raise SystemExit("--mode table needs --slice >= 1")
    # every completed decision's result (reward, events, done, obs: what MultiShipRLEnv.step returns) is
    # written to a per-env record ring, as shipsim_step writes its outputs
    # (sized for every decision of a launch: decisions average ~130 ticks at dt 4 s and the measured
    # maximum is ~slice / 76; the largest per-launch count is reported as decision_log.max_per_launch)
    dlog_cap = max(8, (args.slice + max(args.tail_ticks, 0)) // 32 + 16)
    if args.tail_ticks > 0:  # launches end on the slowest wave's quota, the others tick on meanwhile
        sim.set_stream_tail(args.tail_ticks)
    dlog = torch.zeros((N, dlog_cap, abi.DECLOG_COLS), dtype=torch.float64, device=dev)
    dlog_len = torch.zeros(N, dtype=torch.int32, device=dev)
    dlog_max = torch.zeros((), dtype=torch.int32, device=dev)

    def one_step_table(timed_i=None):
        dlog_len.zero_()
        if timed_i is not None:
            ev0[timed_i].record()
        sim.run_table(table, args.slice, ep32, dec32, out=tout, log=dlog, log_len=dlog_len)
        torch.maximum(dlog_max, dlog_len.max(), out=dlog_max)
        if timed_i is not None:
            ev1[timed_i].record()
        total_ticks.add_(tout["ticks"].sum())
        total_decisions.add_(tout["decisions"].sum())

    def one_step(timed_i=None):
        if args.mode == "table":
            return one_step_table(timed_i)
        act = table[ep_idx % table_eps, dec_idx, ar]
        if timed_i is not None:
            ev0[timed_i].record()
        sim.step(act, max_ticks=args.slice, out=out)
        if timed_i is not None:
            ev1[timed_i].record()
        ready = out["ready"].bool()
        end = ready & (out["done"].bool() | (dec_idx + 1 >= n_dec))
        total_ticks.add_(out["ticks"].sum())
        total_decisions.add_(ready.sum())
        dec_idx.add_(ready.long())
        dec_idx.masked_fill_(end, 0)
        ep_idx.add_(end.long())
        sim.reset(mask=end.to(torch.uint8), obs_out=obs_reset)

    progress("headline stream: warmup + timed launches")
    sim.reset(obs_out=obs_reset)
    for i in range(args.warmup):
        one_step(args.steps + i)
    total_ticks.zero_()
    total_decisions.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    # the same stream without the launch tail (the training collector's default, FUSED_TAIL = 0), beside the
    # headline, which runs with it (--tail-ticks): the same number of launches, continuing the same envs
    tail_off = None
    if args.mode == "table" and args.tail_ticks > 0:
        progress("headline stream without the launch tail")
        sim.set_stream_tail(0)
        off_ticks = torch.zeros((), dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t_off = time.perf_counter()
        for i in range(args.steps):
            dlog_len.zero_()
            sim.run_table(table, args.slice, ep32, dec32, out=tout, log=dlog, log_len=dlog_len)
            off_ticks.add_(tout["ticks"].sum())
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        off = torch.tensor([time.perf_counter() - t_off, float(off_ticks.item())], dtype=torch.float64, device=dev)
        if world > 1:
            mx, sm = off.clone(), off.clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(sm, op=dist.ReduceOp.SUM)
            off = torch.stack([mx[0], sm[1]])
        tail_off = {"value": float(off[1]) / float(off[0]), "ms_per_step": float(off[0]) / args.steps * 1e3,
                    "tail_ticks": 0, "note": "the same C3 stream and launches with the work-conserving launch tail "
                                             "off (the training collector's default); the headline runs with it"}
        sim.set_stream_tail(args.tail_ticks)

    all_ms = np.array([a.elapsed_time(b) for a, b in zip(ev0, ev1)])
    kern_ms = all_ms[:args.steps]
    local_ticks = int(total_ticks.item())
    stats = torch.tensor([elapsed, float(local_ticks), float(total_decisions.item()), float(kern_ms.mean())],
                         dtype=torch.float64, device=dev)
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, kmean = float(mx[0]), float(mx[3])
        all_ticks, all_dec = float(sm[1]), float(sm[2])
    else:
        all_ticks, all_dec, kmean = float(local_ticks), float(total_decisions.item()), float(kern_ms.mean())

    if rank == 0:
        value = all_ticks / elapsed
        ticks_per_launch = local_ticks / args.steps
        achieved = bytes_per_tick * ticks_per_launch / (kmean * 1e-3) / 1e9
        def pmc_record(path):
            # a separate rocprofv3 --pmc pass of this same bench command (profiles/), used only when it was
            # taken on this workload
            try:
                with open(path) as f:
                    rec = json.load(f)
            except (OSError, ValueError):
                return None
            same = (rec.get("collav") == args.collav and rec.get("envs") == N and rec.get("slice") == args.slice
                    and rec.get("obs_ships", 1) == args.obs_ships and rec.get("machinery", "detailed") == args.machinery)
            return rec if same else None
        pmc = pmc_record(args.pmc_json)
        traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
        fp64 = pmc_record(args.pmc_fp64_json)
        fp64_valu = None
        if fp64:
            flops = fp64["fp64_flops_per_launch"]
            tflops = flops / (kmean * 1e-3) / 1e12
            fp64_valu = {"flops_per_launch": flops, "achieved_tflops": tflops, "peak_tflops": FP64_VALU_PEAK_TFLOPS,
                         "frac": tflops / FP64_VALU_PEAK_TFLOPS,
                         "flops_per_env_tick_all_lanes": flops / ticks_per_launch,
                         "flops_per_env_tick_distinct": flops / ticks_per_launch * 2 / sim.lanes_per_env,
                         "fp64_wave_instructions_per_env_tick": fp64["fp64_wave_instructions_per_launch"]
                         / ticks_per_launch,
                         "source": os.path.relpath(args.pmc_fp64_json, ROOT),
                         "note": "64 lanes x SQ_INSTS_VALU_FLOPS_FP64 (= 2 FMA + ADD + MUL + TRANS f64 wave-"
                                 "instructions) per launch / this run's mean launch time: the FP64 VALU rate the "
                                 "kernel issues; 'distinct' counts each ship's chain once (its LPE/2 sub-lanes "
                                 "repeat it)"}
    progress("c2 single ships")
    c2 = bench_c2(dev) if (rank == 0 and not args.no_c2) else None
    progress("policy stream")
    pstream = (bench_policy_stream(dev, cfg, N, args.slice if args.mode == "table" else 4096,
                                   tail_ticks=max(args.tail_ticks, 0) if args.mode == "table" else 0)
               if (rank == 0 and not args.no_policy_stream and args.obs_ships == 1) else None)
    if pstream is not None:  # the runner's --layer_size 512: the in-kernel fc1 in two 256-unit slices
        p512 = bench_policy_stream(dev, cfg, N, args.slice if args.mode == "table" else 4096, launches=1,
                                   tail_ticks=max(args.tail_ticks, 0) if args.mode == "table" else 0, hidden=512)
        pstream["hidden_512"] = {k: p512[k] for k in ("env_ticks_per_s", "decisions_per_s", "kernel_ms", "launches")}
    progress("sac")
    sac = sac_ar = None
    if args.sac_steps > 0:
        if args.sac_global_batch % world:
            raise SystemExit(f"--sac-global-batch {args.sac_global_batch} is not a multiple of {world} ranks")
        pgw = dist.group.WORLD if world > 1 else None
        sac = bench_sac(dev, world, pgw, args.sac_steps, args.sac_global_batch, dp_mode="replicated")
        if world > 1:  # the alternative data-parallel shape, for DESIGN.md §6's comparison
            sac_ar = bench_sac(dev, world, pgw, args.sac_steps, args.sac_global_batch, eager_steps=0,
                               dp_mode="allreduce")
    c4 = None
    if not args.no_c4:
        progress("c4 loop")
        c4 = bench_c4(dev, world, rank, dist.group.WORLD if world > 1 else None, n_envs=args.c4_envs,
                      loops=args.c4_loops)
    c5 = None
    if not args.no_c5 and args.obs_ships == 1:
        progress("c5 multi-obstacle")
        c5 = {f"k{k}": bench_c5(dev, world, N, k, rank=rank, tail_ticks=max(args.tail_ticks, 0)) for k in (2, 4)}
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N = 1 figure
            progress("cpu baseline")
            cpu = cpu_baseline(cfg, args.cpu_baseline_seconds, host_threads()[0], N)
        line = {
            "metric": "batched env-steps/sec (two-ship AST)",
            "value": value,
            "unit": "env-ticks/s",
            "n_gpus": n_devices,
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded PCG64 scoping-angle table, reference scenario of record)",
            "config": {"workload": ("C3: two-ship AST envs (ShipModelAST PTI machinery, sampled-route LOS, "
                                    "reward_designs), dt 4 s") if args.obs_ships == 1 else
                                   (f"C5 multi-obstacle: test ship + {args.obs_ships} obstacle ships per env "
                                    "(parity unpinned beyond 1), otherwise C3"),
                       "obs_ships": args.obs_ships,
                       "envs_per_gpu": N, "global_envs": N * world, "collav": args.collav,
                       "machinery": args.machinery, "slice_ticks": args.slice, "lanes_per_env": sim.lanes_per_env,
                       "mode": args.mode, "tail_ticks": args.tail_ticks if args.mode == "table" else 0,
                       "parallelism": f"env-shard x{world}" + (f" on {n_devices} device(s), {args.dist_backend}"
                                                                  if n_devices != world else "")},
            "launch_tail": ({"headline_with_tail_ticks": args.tail_ticks, "without_tail": tail_off}
                            if tail_off else None),
            "decisions_per_s": all_dec / elapsed,
            "env_ticks_per_decision": all_ticks / max(all_dec, 1),
            "decision_log": {"cap": dlog_cap, "max_per_launch": int(dlog_max.item())} if args.mode == "table" else None,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": f"ast_step_kernel (avg {kmean:.3f} ms/launch, "
                                   f"{ticks_per_launch:.0f} env-ticks x {bytes_per_tick} B)",
                         "kernel_ms_timed": kmean, "kernel_ms_all_launches": float(all_ms.mean()),
                         "launches": int(len(all_ms)), "fp64_valu": fp64_valu},
            "cpu_baseline": cpu,
            "sac": sac,
            "sac_allreduce": sac_ar,
            "c2_single_ship": c2,
            "policy_stream": pstream,
            "c4": c4,
            "c5": c5,
        }
        print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    sim.close()


if __name__ == "__main__":
    main()
