"""DeviceBatchRLAlgorithm — BatchRLAlgorithm's epoch shape (batch_rl_algorithm.py:58-106) on
device-resident envs, replay buffer and a graph-captured SAC update.

Per epoch (rank-local counts; with R ranks the job does R× the decisions and every grad step
averages R local batches of batch_size, i.e. a global batch of R·batch_size):
  epoch 0: collect ≥ min_num_steps_before_training exploration decisions into the buffer;
  every epoch: ≥ num_eval_steps_per_epoch decisions with the deterministic policy (eval env),
  then per train loop ≥ num_expl_steps_per_train_loop exploration decisions + num_trains_per_train_loop
  grad steps, each on a fresh on-device uniform batch.
"""
from .batch_rl_algorithm import BaseRLAlgorithm


class DeviceBatchRLAlgorithm(BaseRLAlgorithm):
    def __init__(self, trainer, exploration_env, evaluation_env, exploration_data_collector,
                 evaluation_data_collector, replay_buffer, batch_size, max_path_length, num_epochs,
                 num_eval_steps_per_epoch, num_expl_steps_per_train_loop, num_trains_per_train_loop,
                 num_train_loops_per_epoch=1, min_num_steps_before_training=0, start_epoch=0):
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

    def train(self):
        for self.epoch in range(self._start_epoch, self.num_epochs):
            self._begin_epoch(self.epoch)
            self._train()
            self._end_epoch(self.epoch)

    def _train(self):
        if self.epoch == 0 and self.min_num_steps_before_training > 0:
            self.expl_data_collector.collect(self.min_num_steps_before_training, self.replay_buffer)
            self.expl_data_collector.end_epoch(-1)
            self.timer.stamp("initial exploration")
        if self.num_eval_steps_per_epoch > 0:
            self.eval_data_collector.collect(self.num_eval_steps_per_epoch, None, record_paths=True)
        self.timer.stamp("evaluation sampling")
        for _ in range(self.num_train_loops_per_epoch):
            self.expl_data_collector.collect(self.num_expl_steps_per_train_loop, self.replay_buffer,
                                             record_paths=True)
            self.timer.stamp("exploration sampling")
            self.training_mode(True)
            self.trainer.train_from_buffer(self.replay_buffer, self.num_trains_per_train_loop)
            self.timer.stamp("training")
            self.training_mode(False)

    def to(self, device):
        for net in self.trainer.networks:
            net.to(device)

    def training_mode(self, mode):
        for net in self.trainer.networks:
            net.train(mode)
