"""Stochastic-policy numpy interface and MakeDeterministic (ast_sac/torch/sac/policies/base.py:20-64)."""
import numpy as np
import torch
from torch import nn

from ...utils import pytorch_util as ptu
from ...core.distributions import Delta


def torch_ify(x):
    return ptu.from_numpy(x) if isinstance(x, np.ndarray) else x


def np_ify(x):
    return ptu.get_numpy(x) if isinstance(x, torch.Tensor) else x


def elem_or_tuple_to_numpy(x):
    return tuple(np_ify(e) for e in x) if isinstance(x, tuple) else np_ify(x)


class TorchStochasticPolicy(nn.Module):
    """get_action(obs_np) -> (action (act_dim,), {}) sampling one action (base.py:20-38)."""

    def get_action(self, obs_np):
        actions = self.get_actions(obs_np[None])
        return actions[0, :], {}

    def get_actions(self, obs_np):
        with torch.no_grad():
            dist = self._get_dist_from_np(obs_np)
            return elem_or_tuple_to_numpy(dist.sample())

    def _get_dist_from_np(self, *args, **kwargs):
        return self(*tuple(torch_ify(x) for x in args), **{k: torch_ify(v) for k, v in kwargs.items()})

    def reset(self):
        pass

    def set_num_steps_total(self, t):
        pass


class MakeDeterministic(TorchStochasticPolicy):
    """Evaluation policy: Delta(tanh(μ)) (base.py:54-64)."""

    def __init__(self, action_distribution_generator):
        super().__init__()
        self._action_distribution_generator = action_distribution_generator

    def forward(self, *args, **kwargs):
        dist = self._action_distribution_generator.forward(*args, **kwargs)
        return Delta(dist.mle_estimate())
