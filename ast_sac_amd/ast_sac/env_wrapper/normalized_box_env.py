"""Action-normalising wrappers (ast_sac/env_wrapper/proxy_env.py:3-49, normalized_box_env.py:6-64).

`NormalizedBoxEnv` — reference semantics over a single env: a ∈ [-1, 1] →
lb + (a + 1)·0.5·(ub − lb), clipped to [lb, ub] in the box dtype (float32), reward × reward_scale.
`BatchedNormalizedBoxEnv` — the same mapping on (N, 1) device tensors in float32 (the box dtype),
so the scoping angle handed to the kernels equals the reference's float32 value bit for bit.
"""
import numpy as np
import torch

from ...spaces import Box


class ProxyEnv:
    def __init__(self, wrapped_env):
        self._wrapped_env = wrapped_env
        self.action_space = self._wrapped_env.action_space
        self.observation_space = self._wrapped_env.observation_space

    @property
    def wrapped_env(self):
        return self._wrapped_env

    def reset(self, **kwargs):
        return self._wrapped_env.reset(**kwargs)

    def step(self, action):
        return self._wrapped_env.step(action)

    def render(self, *args, **kwargs):
        return self._wrapped_env.render(*args, **kwargs)

    @property
    def horizon(self):
        return self._wrapped_env.horizon

    def terminate(self):
        if hasattr(self.wrapped_env, "terminate"):
            self.wrapped_env.terminate()

    def __getattr__(self, attr):
        if attr == "_wrapped_env":
            raise AttributeError()
        return getattr(self._wrapped_env, attr)

    def __getstate__(self):
        return self.__dict__

    def __setstate__(self, state):
        self.__dict__.update(state)

    def __str__(self):
        return f"{type(self).__name__}({self.wrapped_env})"


class NormalizedBoxEnv(ProxyEnv):
    def __init__(self, env, reward_scale=1.0, obs_mean=None, obs_std=None):
        ProxyEnv.__init__(self, env)
        self._should_normalize = not (obs_mean is None and obs_std is None)
        if self._should_normalize:
            obs_mean = np.zeros_like(env.observation_space.low) if obs_mean is None else np.array(obs_mean)
            obs_std = np.ones_like(env.observation_space.low) if obs_std is None else np.array(obs_std)
        self._reward_scale = reward_scale
        self._obs_mean = obs_mean
        self._obs_std = obs_std
        ub = np.ones(self._wrapped_env.action_space.shape, dtype=np.float32)
        self.action_space = Box(-1 * ub, ub, dtype=np.float32)

    def estimate_obs_stats(self, obs_batch, override_values=False):
        if self._obs_mean is not None and not override_values:
            raise Exception("Observation mean and std already set. To override, set override_values to True.")
        self._obs_mean = np.mean(obs_batch, axis=0)
        self._obs_std = np.std(obs_batch, axis=0)

    def _apply_normalize_obs(self, obs):
        return (obs - self._obs_mean) / (self._obs_std + 1e-8)

    def step(self, action):
        lb = self._wrapped_env.action_space.low
        ub = self._wrapped_env.action_space.high
        scaled_action = lb + (action + 1.0) * 0.5 * (ub - lb)
        scaled_action = np.clip(scaled_action, lb, ub)
        next_obs, reward, done, info = self._wrapped_env.step(scaled_action)
        if self._should_normalize:
            next_obs = self._apply_normalize_obs(next_obs)
        return next_obs, reward * self._reward_scale, done, info

    def reset(self):
        return self._wrapped_env.reset()

    def __str__(self):
        return f"Normalized: {self._wrapped_env}"


def denormalize_action(a, low, high):
    """float32 lb + (a + 1)·0.5·(ub − lb), clipped — normalized_box_env.py:48-51 on tensors. low / high:
    numbers, or float32 tensors already on a's device (no host copy: graph-capturable)."""
    lb = low if torch.is_tensor(low) else torch.as_tensor(np.float32(low), dtype=torch.float32, device=a.device)
    ub = high if torch.is_tensor(high) else torch.as_tensor(np.float32(high), dtype=torch.float32, device=a.device)
    a = a.to(torch.float32)
    return torch.minimum(torch.maximum(lb + (a + 1.0) * 0.5 * (ub - lb), lb), ub)


class BatchedNormalizedBoxEnv:
    """NormalizedBoxEnv over a BatchedMultiShipRLEnv: (N, 1) device actions in [-1, 1]."""

    def __init__(self, env, reward_scale=1.0):
        self._wrapped_env = env
        self._reward_scale = reward_scale
        self.observation_space = env.observation_space
        ub = np.ones(env.action_space.shape, dtype=np.float32)
        self.action_space = Box(-1 * ub, ub, dtype=np.float32)
        self._lb = float(env.action_space.low.reshape(-1)[0])
        self._ub = float(env.action_space.high.reshape(-1)[0])

    @property
    def wrapped_env(self):
        return self._wrapped_env

    @property
    def n_envs(self):
        return self._wrapped_env.n_envs

    def scale_action(self, a):
        key = a.device
        if getattr(self, "_bounds_dev", None) != key:  # the bounds as device scalars, made once per device
            self._bounds = (torch.tensor(np.float32(self._lb), device=key), torch.tensor(np.float32(self._ub), device=key))
            self._bounds_dev = key
        return denormalize_action(a, *self._bounds)

    def reset(self, mask=None, obs_out=None):
        return self._wrapped_env.reset(mask, obs_out=obs_out)

    def step(self, action, active=None):
        obs, r, done, info = self._wrapped_env.step(self.scale_action(action), active=active)
        return obs, r * self._reward_scale, done, info

    def step_async(self, action, max_ticks=64, active=None, out=None):
        out = self._wrapped_env.step_async(self.scale_action(action), max_ticks=max_ticks, active=active, out=out)
        return out

    def __getattr__(self, attr):
        if attr == "_wrapped_env":
            raise AttributeError()
        return getattr(self._wrapped_env, attr)
