"""TanhGaussianPolicy (ast_sac/torch/sac/policies/gaussian_policy.py:65-118).

Mlp trunk with two heads: mean = last_fc(h) and log_std = clamp(last_fc_log_std(h), −20, 2);
both heads U(±init_w) with init_w = 1e-3 (the mean head's bias is 0, the log_std bias is U(±init_w)).
"""
import numpy as np
import torch
from torch import nn

from ...utils import pytorch_util as ptu
from ...core.distributions import TanhNormal
from ...networks.mlp import Mlp
from .base import TorchStochasticPolicy, MakeDeterministic  # noqa: F401  (re-export like the reference)

LOG_SIG_MAX = 2
LOG_SIG_MIN = -20


class TanhGaussianPolicy(Mlp, TorchStochasticPolicy):
    def __init__(self, hidden_sizes, obs_dim, action_dim, std=None, init_w=1e-3, **kwargs):
        super().__init__(hidden_sizes, input_size=obs_dim, output_size=action_dim, init_w=init_w, **kwargs)
        self.log_std = None
        self.std = std
        if std is None:
            last_hidden_size = hidden_sizes[-1] if len(hidden_sizes) > 0 else obs_dim
            self.last_fc_log_std = nn.Linear(last_hidden_size, action_dim)
            self.last_fc_log_std.weight.data.uniform_(-init_w, init_w)
            self.last_fc_log_std.bias.data.uniform_(-init_w, init_w)
        else:
            self.log_std = np.log(std)
            assert LOG_SIG_MIN <= self.log_std <= LOG_SIG_MAX

    def forward(self, obs):
        h = obs
        for fc in self.fcs:
            h = self.hidden_activation(fc(h))
        mean = self.last_fc(h)
        if self.std is None:
            log_std = torch.clamp(self.last_fc_log_std(h), LOG_SIG_MIN, LOG_SIG_MAX)
            std = torch.exp(log_std)
        else:
            std = torch.from_numpy(np.array([self.std])).float().to(obs.device)
        return TanhNormal(mean, std)

    def logprob(self, action, mean, std):
        return TanhNormal(mean, std).log_prob(action).sum(dim=1, keepdim=True)
