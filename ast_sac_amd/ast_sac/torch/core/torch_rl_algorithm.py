"""TorchTrainer / TorchBatchRLAlgorithm (ast_sac/torch/core/torch_rl_algorithm.py:20-53)."""
import abc
from collections import OrderedDict

import numpy as np
import torch

from ..utils import pytorch_util as ptu
from ...core.batch_rl_algorithm import BatchRLAlgorithm


def np_to_pytorch_batch(np_batch):
    """module.py:58-74: every non-object array → float32 tensor on ptu.device (bools → int first)."""
    out = {}
    for k, v in np_batch.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.float().to(ptu.device)
            continue
        v = np.asarray(v)
        if v.dtype == np.dtype("O"):
            continue
        if v.dtype == np.bool_:
            v = v.astype(int)
        out[k] = ptu.from_numpy(v)
    return out


class TorchTrainer(metaclass=abc.ABCMeta):
    def __init__(self):
        self._num_train_steps = 0

    def train(self, np_batch):
        self._num_train_steps += 1
        self.train_from_torch(np_to_pytorch_batch(np_batch))

    def get_diagnostics(self):
        return OrderedDict([("num train calls", self._num_train_steps)])

    def end_epoch(self, epoch):
        pass

    def get_snapshot(self):
        return {}

    @abc.abstractmethod
    def train_from_torch(self, batch):
        pass

    @property
    @abc.abstractmethod
    def networks(self):
        pass


class TorchBatchRLAlgorithm(BatchRLAlgorithm):
    def to(self, device):
        for net in self.trainer.networks:
            net.to(device)

    def training_mode(self, mode):
        for net in self.trainer.networks:
            net.train(mode)
