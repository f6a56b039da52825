"""BaseRLAlgorithm / BatchRLAlgorithm (ast_sac/core/rl_algorithm.py:24-150, batch_rl_algorithm.py:10-106).

Epoch shape of the reference: epoch 0 first collects `min_num_steps_before_training` exploration
steps (8192) into the buffer, then every epoch: `num_eval_steps_per_epoch` evaluation steps (180,
discard incomplete paths), and per train loop `num_expl_steps_per_train_loop` exploration steps
(256) + `num_trains_per_train_loop` (240) trainer.train(replay_buffer.random_batch(batch_size)).
"""
import abc

from . import eval_util
from .logging import logger, EpochTimer


class BaseRLAlgorithm(metaclass=abc.ABCMeta):
    def __init__(self, trainer, exploration_env, evaluation_env, exploration_data_collector,
                 evaluation_data_collector, replay_buffer):
        self.trainer = trainer
        self.expl_env = exploration_env
        self.eval_env = evaluation_env
        self.expl_data_collector = exploration_data_collector
        self.eval_data_collector = evaluation_data_collector
        self.replay_buffer = replay_buffer
        self._start_epoch = 0
        self.post_epoch_funcs = []
        self.timer = EpochTimer()
        self.log_stats = True

    def _begin_epoch(self, epoch):
        self.timer.reset_epoch()

    def _end_epoch(self, epoch):
        logger.save_itr_params(epoch, self._get_snapshot())
        self.timer.stamp("saving")
        if self.log_stats:
            self._log_stats(epoch)
        self.expl_data_collector.end_epoch(epoch)
        self.eval_data_collector.end_epoch(epoch)
        self.replay_buffer.end_epoch(epoch)
        self.trainer.end_epoch(epoch)
        for f in self.post_epoch_funcs:
            f(self, epoch)

    def _get_snapshot(self):
        snap = {}
        for src, pre in ((self.trainer, "trainer/"), (self.expl_data_collector, "exploration/"),
                         (self.eval_data_collector, "evaluation/"), (self.replay_buffer, "replay_buffer/")):
            for k, v in src.get_snapshot().items():
                snap[pre + k] = v
        return snap

    def _log_stats(self, epoch):
        logger.log(f"Epoch {epoch} finished", with_timestamp=True)
        logger.record_dict({"epoch": epoch})
        logger.record_dict(self.replay_buffer.get_diagnostics(), prefix="replay_buffer/")
        logger.record_dict(self.trainer.get_diagnostics(), prefix="trainer/")
        for coll, env, pre in ((self.expl_data_collector, self.expl_env, "expl/"),
                               (self.eval_data_collector, self.eval_env, "eval/")):
            logger.record_dict(coll.get_diagnostics(), prefix=pre)
            paths = coll.get_epoch_paths()
            if hasattr(env, "get_diagnostics"):
                logger.record_dict(env.get_diagnostics(paths), prefix=pre)
            logger.record_dict(eval_util.get_generic_path_information(paths), prefix=pre)
        self.timer.stamp("logging")
        logger.record_dict(self.timer.epoch_timings())
        logger.record_tabular("Epoch", epoch)
        logger.dump_tabular(with_prefix=False, with_timestamp=False)
        for coll, pre in ((self.expl_data_collector, "expl/"), (self.eval_data_collector, "eval/")):
            dev = getattr(coll, "device_diagnostics", None)  # build-only counters: text log, not progress.csv
            if dev is not None:
                logger.log(" ".join(f"{pre}{k}={v}" for k, v in dev().items()))

    @abc.abstractmethod
    def training_mode(self, mode):
        pass


class BatchRLAlgorithm(BaseRLAlgorithm, metaclass=abc.ABCMeta):
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
            self.offline_rl = self.epoch < 0
            self._begin_epoch(self.epoch)
            self._train()
            self._end_epoch(self.epoch)

    def _train(self):
        if self.epoch == 0 and self.min_num_steps_before_training > 0:
            init_paths = self.expl_data_collector.collect_new_paths(
                self.max_path_length, self.min_num_steps_before_training, discard_incomplete_paths=False)
            if not self.offline_rl:
                self.replay_buffer.add_paths(init_paths)
            self.expl_data_collector.end_epoch(-1)
        self.eval_data_collector.collect_new_paths(self.max_path_length, self.num_eval_steps_per_epoch,
                                                   discard_incomplete_paths=True)
        self.timer.stamp("evaluation sampling")
        for _ in range(self.num_train_loops_per_epoch):
            new_paths = self.expl_data_collector.collect_new_paths(
                self.max_path_length, self.num_expl_steps_per_train_loop, discard_incomplete_paths=False)
            self.timer.stamp("exploration sampling")
            if not self.offline_rl:
                self.replay_buffer.add_paths(new_paths)
            self.timer.stamp("data storing")
            self.training_mode(True)
            for _ in range(self.num_trains_per_train_loop):
                self.trainer.train(self.replay_buffer.random_batch(self.batch_size))
                self.timer.stamp("sac training")  # SACTrainer.train_from_torch's own stamp (sac.py:142)
            self.timer.stamp("training")
            self.training_mode(False)
