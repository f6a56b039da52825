"""DeviceBatchRLAlgorithm — BatchRLAlgorithm's epoch shape (batch_rl_algorithm.py:58-106) on
device-resident envs, replay buffer and a graph-captured SAC update.

Per epoch (rank-local counts; with R ranks the job does R× the decisions; the grad steps either run
replicated on every rank over the union of all ranks' transitions — a ReplicatedReplayBuffer, synced after
every collect — or average R local batches with a gradient all-reduce):
  epoch 0: collect ≥ min_num_steps_before_training exploration decisions into the buffer;
  every epoch: ≥ num_eval_steps_per_epoch decisions with the deterministic policy (eval env),
  then per train loop ≥ num_expl_steps_per_train_loop exploration decisions + grad steps, each on a
  fresh on-device uniform batch.

Update-to-data ratio. The reference collects exactly num_expl_steps_per_train_loop (256) decisions per
loop and then runs num_trains_per_train_loop (240) grad steps of batch_size (256): 240/256 grad steps
per collected decision. A sliced pass over thousands of envs overshoots 256 by a wide margin, so with
match_update_ratio (default) the loop runs round(collected_on_all_ranks × 240/256) grad steps (the
fraction carried to the next loop) — the reference's ratio of grad steps and of sampled rows (global
batch = batch_size, split over the ranks by the runner) per environment decision. With
match_update_ratio=False it runs num_trains_per_train_loop per loop, as written.
"""
import torch

from .batch_rl_algorithm import BaseRLAlgorithm


class DeviceBatchRLAlgorithm(BaseRLAlgorithm):
    def __init__(self, trainer, exploration_env, evaluation_env, exploration_data_collector,
                 evaluation_data_collector, replay_buffer, batch_size, max_path_length, num_epochs,
                 num_eval_steps_per_epoch, num_expl_steps_per_train_loop, num_trains_per_train_loop,
                 num_train_loops_per_epoch=1, min_num_steps_before_training=0, start_epoch=0,
                 match_update_ratio=True):
        super().__init__(trainer, exploration_env, evaluation_env, exploration_data_collector,
                         evaluation_data_collector, replay_buffer)
        self.batch_size = batch_size
        self.max_path_length = max_path_length
        self.num_epochs = num_epochs
        self.num_eval_steps_per_epoch = num_eval_steps_per_epoch
        self.num_trains_per_train_loop = num_trains_per_train_loop
        self.num_train_loops_per_epoch = num_train_loops_per_epoch
        self.num_expl_steps_per_train_loop = num_expl_steps_per_train_loop
        self.min_num_steps_before_training = min_num_steps_before_training
        self._start_epoch = start_epoch
        self.match_update_ratio = match_update_ratio
        self._utd_carry = 0.0
        self.num_train_steps_total = 0
        self.num_loop_expl_steps_total = 0  # rank-local decisions collected inside train loops

    def _n_grad_steps(self, collected):
        """Grad steps for `collected` rank-local decisions (same count on every rank)."""
        if not self.match_update_ratio:
            return self.num_trains_per_train_loop
        pg = getattr(self.trainer, "pg", None)
        if pg is not None and torch.distributed.get_world_size(pg) > 1:
            dev = "cuda" if torch.distributed.get_backend(pg) == "nccl" else "cpu"
            t = torch.tensor([collected], dtype=torch.int64, device=dev)
            torch.distributed.all_reduce(t, group=pg)
            collected = int(t.item())
        x = self._utd_carry + collected * self.num_trains_per_train_loop / self.num_expl_steps_per_train_loop
        k = int(x)
        self._utd_carry = x - k
        return k

    def train(self):
        for self.epoch in range(self._start_epoch, self.num_epochs):
            self._begin_epoch(self.epoch)
            self._train()
            self._end_epoch(self.epoch)

    def _train(self):
        if self.epoch == 0 and self.min_num_steps_before_training > 0:
            self.expl_data_collector.collect(self.min_num_steps_before_training, self.replay_buffer)
            self._sync_buffer()
            self.expl_data_collector.end_epoch(-1)  # (unstamped, as in the reference: counts as evaluation sampling)
        if self.num_eval_steps_per_epoch > 0:
            self.eval_data_collector.collect(self.num_eval_steps_per_epoch, None, record_paths=True)
        self.timer.stamp("evaluation sampling")
        for _ in range(self.num_train_loops_per_epoch):
            got = self.expl_data_collector.collect(self.num_expl_steps_per_train_loop, self.replay_buffer,
                                                   record_paths=True)
            self.timer.stamp("exploration sampling")
            self._sync_buffer()
            self.timer.stamp("data storing")  # the collector wrote the buffer on the device (+ the replicas' sync)
            self.training_mode(True)
            self.num_loop_expl_steps_total += got
            k = self._n_grad_steps(got)
            if k:
                self.trainer.train_from_buffer(self.replay_buffer, k)
            self.num_train_steps_total += k
            self.timer.stamp("sac training")  # the reference stamps it in SACTrainer.train_from_torch (sac.py:142)
            self.timer.stamp("training")
            self.training_mode(False)

    def _sync_buffer(self):
        """Replicated data parallel: every rank's new rows into every rank's ring (two all-gathers per collect: counts, rows)."""
        sync = getattr(self.replay_buffer, "sync", None)
        if sync is not None:
            sync()

    def to(self, device):
        for net in self.trainer.networks:
            net.to(device)

    def training_mode(self, mode):
        for net in self.trainer.networks:
            net.train(mode)
