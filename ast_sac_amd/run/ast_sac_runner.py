"""AST-SAC training launcher (run/ast-sac_runner.py).

Same CLI and variant as the reference. Two execution shapes:

* `--n_envs 0`: the reference object graph — one MultiShipRLEnv (N=1 view of the device env),
  NormalizedBoxEnv, MdpPathCollector(ast_sac_rollout), EnvReplayBuffer, SACTrainer,
  TorchBatchRLAlgorithm — for drop-in use and side-by-side comparison.
* `--n_envs N` (default 4096): the MI355X shape — N device-resident envs per GPU stepped in
  slices, transitions written straight into a DeviceReplayBuffer, FusedSACTrainer (HIP-graph
  step) and DeviceBatchRLAlgorithm. Under torch.distributed.run every rank owns N envs. With
  --dp_mode replicated (default) every rank keeps the union of all ranks' transitions (RCCL
  all-gathers of the row counts and the new rows once per train loop) and runs the same global-batch SAC step, so no
  collective runs per grad step; --dp_mode allreduce gives each rank a local buffer and averages
  the SAC gradients with one RCCL all-reduce per grad step.

    python -m ast_sac_amd.run.ast_sac_runner --num_epochs 2
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m ast_sac_amd.run.ast_sac_runner
"""
import argparse
import os

import numpy as np
import torch


def _bool(s):
    return str(s).lower() in ("1", "true", "yes", "y")


def build_parser():
    p = argparse.ArgumentParser(description="Ship Transit Soft Actor-Critic Args")
    # environment (run/ast-sac_runner.py:27-43)
    p.add_argument("--max_sampling_frequency", type=int, default=9)
    p.add_argument("--time_step", type=int, default=4)
    p.add_argument("--radius_of_acceptance", type=int, default=300)
    p.add_argument("--lookahead_distance", type=int, default=1000)
    p.add_argument("--collav_mode", type=str, default="sbmpc")
    p.add_argument("--ship_draw", type=_bool, default=True)
    p.add_argument("--time_since_last_ship_drawing", default=30)
    p.add_argument("--normalize_action", type=_bool, default=False)
    # algorithm (:46-80)
    p.add_argument("--do_logging", type=_bool, default=True)
    p.add_argument("--algorithm", type=str, default="SAC")
    p.add_argument("--version", type=str, default="normal")
    p.add_argument("--layer_size", type=int, default=256)
    p.add_argument("--replay_buffer_size", type=int, default=300000)
    p.add_argument("--batch_size", type=int, default=256)
    p.add_argument("--num_epochs", type=int, default=500)
    p.add_argument("--num_eval_steps_per_epoch", type=int, default=180)
    p.add_argument("--num_trains_per_train_loop", type=int, default=240)
    p.add_argument("--num_expl_steps_per_train_loop", type=int, default=256)
    p.add_argument("--min_num_steps_before_training", type=int, default=8192)
    p.add_argument("--max_path_length", type=int, default=9)
    # trainer (:83-104)
    p.add_argument("--discount", type=float, default=0.965)
    p.add_argument("--soft_target_tau", type=float, default=1e-3)
    p.add_argument("--target_update_period", type=int, default=1)
    p.add_argument("--policy_lr", type=float, default=8e-5)
    p.add_argument("--qf_lr", type=float, default=8e-5)
    p.add_argument("--reward_scale", type=float, default=0.75)
    p.add_argument("--use_automatic_entropy_tuning", type=_bool, default=True)
    p.add_argument("--action_reg_coeff", type=float, default=0.01)
    p.add_argument("--clip_val", type=float, default=100)
    # MI355X execution shape
    p.add_argument("--n_envs", type=int, default=4096, help="device envs per GPU (0 = reference single-env graph)")
    p.add_argument("--eval_envs", type=int, default=0,
                   help="0 (default): evaluation on the exploration envs, one env object as the reference (Q10); "
                        "N > 0: a separate evaluation shard of N envs")
    p.add_argument("--slice_ticks", type=int, default=0,
                   help="env ticks per collector pass; 0: the collector's measured best for its pass kind "
                        "(1024 with the policy inside the env launch, 128 for sliced passes; DESIGN §9)")
    p.add_argument("--fused_collect", type=_bool, default=True,
                   help="the policy inside the env launch (shipsim_run_policy) where the networks allow it")
    p.add_argument("--stream_tail", type=int, default=-1,
                   help="fused passes: the env launch's work-conserving tail (shipsim_set_stream_tail) — envs whose "
                        "wave met the pass's ticks tick on, up to this many more, while the slowest wave has not; "
                        "-1/0: off (the default: runs repeat bit for bit); 512: +11.6 %% collection rate (DESIGN §9), with launch "
                        "boundaries (and so a stochastic policy's noise draws) depending on timing")
    p.add_argument("--match_update_ratio", type=_bool, default=True,
                   help="grad steps per train loop = collected decisions (all ranks) x num_trains / num_expl_steps "
                        "(the reference's ratio); false: num_trains_per_train_loop per loop")
    p.add_argument("--dp_mode", type=str, default="replicated", choices=["replicated", "allreduce"],
                   help="multi-rank SAC: replicated = every rank trains on the union of all ranks' transitions (one "
                        "row all-gather (after a count all-gather) per train loop, no per-step collective); allreduce = local buffers, one gradient "
                        "all-reduce per grad step")
    p.add_argument("--machinery", type=str, default="detailed", choices=["detailed", "simplified"])
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--log_dir", type=str, default=None)
    return p


def parse_cli_args(argv=None):
    return build_parser().parse_args(argv)


def make_variant(args):
    return dict(
        algorithm=args.algorithm, version=args.version, layer_size=args.layer_size,
        replay_buffer_size=args.replay_buffer_size,
        algorithm_kwargs=dict(num_epochs=args.num_epochs, num_eval_steps_per_epoch=args.num_eval_steps_per_epoch,
                              num_trains_per_train_loop=args.num_trains_per_train_loop,
                              num_expl_steps_per_train_loop=args.num_expl_steps_per_train_loop,
                              min_num_steps_before_training=args.min_num_steps_before_training,
                              max_path_length=args.max_path_length, batch_size=args.batch_size),
        trainer_kwargs=dict(discount=args.discount, soft_target_tau=args.soft_target_tau,
                            target_update_period=args.target_update_period, policy_lr=args.policy_lr,
                            qf_lr=args.qf_lr, reward_scale=args.reward_scale,
                            use_automatic_entropy_tuning=args.use_automatic_entropy_tuning,
                            action_reg_coeff=args.action_reg_coeff, clip_val=args.clip_val),
        n_envs=args.n_envs, slice_ticks=args.slice_ticks, machinery=args.machinery,
        match_update_ratio=args.match_update_ratio, dp_mode=args.dp_mode)


def _networks(obs_dim, act_dim, M, device):
    from ..ast_sac.torch.networks.mlp import ConcatMlp
    from ..ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    qs = [ConcatMlp(input_size=obs_dim + act_dim, output_size=1, hidden_sizes=[M, M]).to(device) for _ in range(4)]
    policy = TanhGaussianPolicy(obs_dim=obs_dim, action_dim=act_dim, hidden_sizes=[M, M]).to(device)
    return policy, qs


def experiment_reference(variant, args, device):
    """run/ast-sac_runner.py:experiment, object for object."""
    from .env_setup import prepare_multiship_rl_env
    from ..ast_sac.env_wrapper.normalized_box_env import NormalizedBoxEnv
    from ..ast_sac.data_management.replay_buffer import EnvReplayBuffer
    from ..ast_sac.samplers.data_collector.path_collector import MdpPathCollector
    from ..ast_sac.samplers.data_collector.rollout_functions import ast_sac_rollout
    from ..ast_sac.torch.sac.policies.base import MakeDeterministic
    from ..ast_sac.torch.sac.sac import SACTrainer
    from ..ast_sac.torch.core.torch_rl_algorithm import TorchBatchRLAlgorithm

    env, _ = prepare_multiship_rl_env(args, device=device, machinery=args.machinery)
    expl_env = NormalizedBoxEnv(env, reward_scale=args.reward_scale)
    eval_env = NormalizedBoxEnv(env, reward_scale=args.reward_scale)  # shared env object, as the reference (Q10)
    obs_dim = expl_env.observation_space.low.size
    act_dim = expl_env.action_space.low.size
    policy, (qf1, qf2, tq1, tq2) = _networks(obs_dim, act_dim, variant["layer_size"], device)
    eval_coll = MdpPathCollector(eval_env, MakeDeterministic(policy), rollout_fn=ast_sac_rollout)
    expl_coll = MdpPathCollector(expl_env, policy, rollout_fn=ast_sac_rollout)
    rb = EnvReplayBuffer(variant["replay_buffer_size"], expl_env)
    trainer = SACTrainer(env=eval_env, policy=policy, qf1=qf1, qf2=qf2, target_qf1=tq1, target_qf2=tq2,
                         **variant["trainer_kwargs"])
    algo = TorchBatchRLAlgorithm(trainer=trainer, exploration_env=expl_env, evaluation_env=eval_env,
                                 exploration_data_collector=expl_coll, evaluation_data_collector=eval_coll,
                                 replay_buffer=rb, **variant["algorithm_kwargs"])
    algo.to(device)
    return algo


def replicated_stage_rows(args, ak):
    """Rows the replicated buffer's staging ring must hold between two syncs (one per collect): the largest
    collect's decisions plus the overshoot of its last batch of passes, which the collector bounds to the ring's
    free rows (batched_collector.py collect) — at least two passes of the widest kind (fused: N x the log cap)."""
    from ..ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector as C
    ticks = args.slice_ticks or C.FUSED_TICKS
    tail = C.FUSED_TAIL if args.stream_tail < 0 else args.stream_tail
    per_pass = args.n_envs * C.log_cap_for(ticks, tail)
    return max(65536, max(ak["min_num_steps_before_training"], ak["num_expl_steps_per_train_loop"]) + 2 * per_pass)


def experiment_device(variant, args, device, process_group=None):
    from ..rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, config_from_args
    from ..ast_sac.env_wrapper.normalized_box_env import BatchedNormalizedBoxEnv
    from ..ast_sac.data_management.replay_buffer import DeviceReplayBuffer, ReplicatedReplayBuffer
    from ..ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector
    from ..ast_sac.torch.sac.policies.base import MakeDeterministic
    from ..ast_sac.torch.sac.sac_fused import FusedSACTrainer
    from ..ast_sac.core.device_rl_algorithm import DeviceBatchRLAlgorithm

    cfg = config_from_args(args, args.machinery)
    env = BatchedMultiShipRLEnv(args, args.n_envs, device=device, cfg=cfg)
    expl_env = BatchedNormalizedBoxEnv(env, reward_scale=args.reward_scale)
    if args.eval_envs > 0:  # a separate evaluation env shard (not the reference's shape, see below)
        eval_env = BatchedNormalizedBoxEnv(BatchedMultiShipRLEnv(args, args.eval_envs, device=device,
                                                                 cfg=config_from_args(args, args.machinery)),
                                           reward_scale=args.reward_scale)
    else:  # default: one env object under both wrappers, as run/ast-sac_runner.py:113-114 (quirk Q10): the
        # evaluation episodes reset and advance the exploration envs, whose SBMPC memory carries over (Q7)
        eval_env = BatchedNormalizedBoxEnv(env, reward_scale=args.reward_scale)
    obs_dim = expl_env.observation_space.low.size
    act_dim = expl_env.action_space.low.size
    policy, (qf1, qf2, tq1, tq2) = _networks(obs_dim, act_dim, variant["layer_size"], device)
    ak = variant["algorithm_kwargs"]
    # --batch_size is the GLOBAL batch (the reference's 256, run/ast-sac_runner.py:55)
    world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
    # (a process group of one rank takes the replicated path too: the N-rank code, an identity on the data)
    replicated = process_group is not None and variant.get("dp_mode", "replicated") == "replicated"
    if replicated:  # every rank: the union of all ranks' rows, the whole global batch, the same seed
        rb = ReplicatedReplayBuffer(variant["replay_buffer_size"], obs_dim, act_dim, device, process_group,
                                    replicated_stage_rows(args, ak))
        per_rank_batch = ak["batch_size"]
    else:  # each rank samples batch_size / world rows from its own shard; the averaged gradient equals the
        # single-GPU B-row gradient in expectation
        rb = DeviceReplayBuffer(variant["replay_buffer_size"], obs_dim, act_dim, device)
        if ak["batch_size"] % world:
            raise ValueError(f"--batch_size {ak['batch_size']} must be a multiple of the {world} ranks")
        per_rank_batch = ak["batch_size"] // world
    trainer = FusedSACTrainer(env=eval_env, policy=policy, qf1=qf1, qf2=qf2, target_qf1=tq1, target_qf2=tq2,
                              batch_size=per_rank_batch, process_group=process_group, replicated=replicated,
                              backend="hip", **variant["trainer_kwargs"])
    trainer.broadcast_parameters(0)
    # the collectors sample the trainer's current policy on the matrix cores (sacf_policy_act) and replay
    # each slice pass as a HIP graph (batched_collector.py); the torch modules stay their snapshot surface
    ticks = args.slice_ticks or None
    fused = None if args.fused_collect else False
    expl_coll = BatchedPathCollector(expl_env, policy, max_path_length=ak["max_path_length"],
                                     max_ticks=ticks, device_policy=trainer.device_policy(False), fused=fused,
                                     stream_tail=None if args.stream_tail < 0 else args.stream_tail)
    eval_coll = BatchedPathCollector(eval_env, MakeDeterministic(policy), max_path_length=ak["max_path_length"],
                                     max_ticks=ticks, deterministic=True,
                                     device_policy=trainer.device_policy(True), fused=fused,
                                     stream_tail=None if args.stream_tail < 0 else args.stream_tail)
    return DeviceBatchRLAlgorithm(trainer=trainer, exploration_env=expl_env, evaluation_env=eval_env,
                                  exploration_data_collector=expl_coll, evaluation_data_collector=eval_coll,
                                  replay_buffer=rb, match_update_ratio=variant.get("match_update_ratio", True), **ak)


def main(argv=None):
    args = parse_cli_args(argv)
    from ..ast_sac.torch.utils import pytorch_util as ptu
    from ..ast_sac.launchers.launcher_utils import setup_logger
    from ..ast_sac.core.logging import logger

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise RuntimeError("the AST-SAC runner needs a HIP device (the env runs in ast_sac_amd/csrc kernels)")
    ptu.set_gpu_mode(True, local)
    torch.cuda.set_device(local)
    device = ptu.device
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)
        pg = dist.group.WORLD
    if args.seed is not None:
        torch.manual_seed(args.seed + rank)
        np.random.seed(args.seed + rank)
    variant = make_variant(args)
    if args.do_logging and rank == 0:
        setup_logger("ast-sac_maritime_logs", variant=variant, log_dir=args.log_dir)
    if rank != 0:
        logger.set_snapshot_dir(None)
    if args.n_envs <= 0:
        if world > 1:
            raise ValueError("the reference single-env graph runs on one rank; use --n_envs N for data parallel")
        algo = experiment_reference(variant, args, device)
    else:
        algo = experiment_device(variant, args, device, pg)
        algo.log_stats = rank == 0
    algo.train()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
