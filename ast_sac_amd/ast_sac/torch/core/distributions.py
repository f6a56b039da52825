"""Action distributions of the SAC actor (ast_sac/torch/core/distributions.py:20-122, :320-447).

TanhNormal: z = μ + σ·ε (ε ~ N(0, I), reparameterised), a = tanh z,
log π(a) = Σ_d N(z; μ, σ) − 2·Σ_d (log 2 − z − softplus(−2z))    (distributions.py:346-392).

`TanhNormal.noise_source` (class attribute, default None → torch.randn) lets tests inject ε so a
step can be compared against captured reference fixtures; it is the only hook added.
"""
import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

from ...core.eval_util import create_stats_ordered_dict
from ..utils import pytorch_util as ptu

_LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))
_LOG2 = math.log(2.0)


class Distribution:
    def sample_and_logprob(self):
        s = self.sample()
        return s, self.log_prob(s)

    def rsample_and_logprob(self):
        s = self.rsample()
        return s, self.log_prob(s)

    def mle_estimate(self):
        return self.mean

    def get_diagnostics(self):
        return {}


class Delta(Distribution):
    """Deterministic distribution (distributions.py:98-121)."""

    def __init__(self, value):
        self.value = value

    def sample(self):
        return self.value.detach()

    def rsample(self):
        return self.value

    @property
    def mean(self):
        return self.value

    @property
    def variance(self):
        return 0

    @property
    def entropy(self):
        return 0


def diag_normal_log_prob(x, mean, std):
    """Independent(Normal(mean, std), 1).log_prob(x), torch's evaluation order."""
    var = std ** 2
    return (-((x - mean) ** 2) / (2 * var) - torch.log(std) - _LOG_SQRT_2PI).sum(-1)


class MultivariateDiagonalNormal(Distribution):
    def __init__(self, loc, scale_diag):
        self.loc = loc
        self.scale = scale_diag

    @property
    def mean(self):
        return self.loc

    @property
    def stddev(self):
        return self.scale

    def sample(self):
        with torch.no_grad():
            return torch.normal(self.loc.expand_as(self.scale), self.scale)

    def rsample(self):
        return self.loc + self.scale * torch.randn_like(self.scale)

    def log_prob(self, value):
        return diag_normal_log_prob(value, self.loc, self.scale)


class TanhNormal(Distribution):
    noise_source = None  # callable(shape, device, dtype) -> ε, or None for torch.randn

    def __init__(self, normal_mean, normal_std, epsilon=1e-6):
        self.normal_mean = normal_mean
        self.normal_std = normal_std
        self.normal = MultivariateDiagonalNormal(normal_mean, normal_std)
        self.epsilon = epsilon

    def _eps(self):
        shape = self.normal_mean.shape
        src = TanhNormal.noise_source
        if src is not None:
            return src(shape, self.normal_mean.device, self.normal_mean.dtype)
        return torch.randn(shape, device=self.normal_mean.device, dtype=self.normal_mean.dtype)

    def _log_prob_from_pre_tanh(self, pre_tanh_value):
        log_prob = self.normal.log_prob(pre_tanh_value)
        correction = -2.0 * (_LOG2 - pre_tanh_value - F.softplus(-2.0 * pre_tanh_value)).sum(dim=1)
        return log_prob + correction

    def log_prob(self, value, pre_tanh_value=None):
        if pre_tanh_value is None:
            value = torch.clamp(value, -0.999999, 0.999999)
            pre_tanh_value = torch.log(1 + value) / 2 - torch.log(1 - value) / 2
        return self._log_prob_from_pre_tanh(pre_tanh_value)

    def rsample_with_pretanh(self):
        z = self.normal_mean + self.normal_std * self._eps()
        return torch.tanh(z), z

    def sample(self):
        value, _ = self.rsample_with_pretanh()
        return value.detach()

    def rsample(self):
        value, _ = self.rsample_with_pretanh()
        return value

    def sample_and_logprob(self):
        value, pre = self.rsample_with_pretanh()
        value, pre = value.detach(), pre.detach()
        return value, self.log_prob(value, pre)

    def rsample_and_logprob(self):
        value, pre = self.rsample_with_pretanh()
        return value, self.log_prob(value, pre)

    def rsample_logprob_and_pretanh(self):
        value, pre = self.rsample_with_pretanh()
        return value, self.log_prob(value, pre), pre

    @property
    def mean(self):
        return torch.tanh(self.normal_mean)

    @property
    def stddev(self):
        return self.normal_std

    def get_diagnostics(self):
        stats = OrderedDict()
        stats.update(create_stats_ordered_dict("mean", ptu.get_numpy(self.mean)))
        stats.update(create_stats_ordered_dict("normal/std", ptu.get_numpy(self.normal_std)))
        stats.update(create_stats_ordered_dict("normal/log_std", ptu.get_numpy(torch.log(self.normal_std))))
        return stats
