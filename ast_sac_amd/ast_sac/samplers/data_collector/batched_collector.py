"""BatchedPathCollector — MdpPathCollector + ast_sac_rollout for N device-resident envs.

Per env the semantics of ast_sac_rollout (rollout_functions.py:74-181) hold: an episode starts
with reset(), the policy picks an action from the current observation whenever the env waits for
a decision, the env runs that decision, the transition (o, a, r·reward_scale, o', terminal =
env_info['terminal']) is recorded, and the episode ends on done or after max_path_length
decisions. Unlike the reference, thousands of envs advance together: one sliced
`step_async(max_ticks)` call advances every env by ≤ max_ticks ticks, envs that complete a
decision emit their transition straight into a DeviceReplayBuffer, and finished envs are reset
in the same pass (masked reset). Nothing crosses to the host inside `collect`.
"""
from collections import OrderedDict, deque

import numpy as np
import torch

from ...core.eval_util import create_stats_ordered_dict


class BatchedPathCollector:
    def __init__(self, env, policy, max_path_length=9, max_ticks=64, deterministic=False,
                 max_num_epoch_paths_saved=None):
        self._env = env                       # BatchedNormalizedBoxEnv
        self._policy = policy
        self.max_path_length = int(max_path_length)
        self.max_ticks = int(max_ticks)
        self.deterministic = deterministic
        N = env.n_envs
        dev = env.device
        self.N, self.device = N, dev
        self._obs = env.reset().clone()                           # (N, 8) obs at the pending decision
        self._act = torch.zeros((N, 1), dtype=torch.float32, device=dev)
        self._awaiting = torch.ones(N, dtype=torch.bool, device=dev)
        self._path_len = torch.zeros(N, dtype=torch.int32, device=dev)
        self._ret = torch.zeros(N, dtype=torch.float64, device=dev)
        f = lambda dt: torch.empty(N, dtype=dt, device=dev)
        self._out = dict(obs=torch.empty((N, 8), dtype=torch.float32, device=dev), reward=f(torch.float64),
                         done=f(torch.uint8), events=f(torch.int32), ticks=f(torch.int32), ready=f(torch.uint8))
        self._obs_reset = torch.empty((N, 8), dtype=torch.float32, device=dev)
        # device-side counters (read by get_diagnostics only)
        self._steps_total = torch.zeros((), dtype=torch.int64, device=dev)
        self._paths_total = torch.zeros((), dtype=torch.int64, device=dev)
        self._ticks_total = torch.zeros((), dtype=torch.int64, device=dev)
        self._epoch_returns = []
        self._epoch_lens = []
        self._max_saved = max_num_epoch_paths_saved

    @torch.no_grad()
    def _actions(self, obs):
        dist = self._policy(obs)
        if self.deterministic or not hasattr(dist, "rsample_with_pretanh"):
            return dist.mle_estimate() if hasattr(dist, "mle_estimate") else dist.sample()
        return dist.sample()

    @torch.no_grad()
    def step(self, replay_buffer=None):
        """One sliced pass over all envs. Returns (ready mask, #transitions) as device tensors."""
        new_a = self._actions(self._obs)
        self._act = torch.where(self._awaiting.unsqueeze(1), new_a.to(torch.float32), self._act)
        out = self._env.step_async(self._act, max_ticks=self.max_ticks, out=self._out)
        ready = out["ready"].bool()
        done = out["done"].bool()
        rew = out["reward"] * self._env._reward_scale
        terminal = (out["events"] & (1 << 16)) != 0
        if replay_buffer is not None:
            replay_buffer.add_batch(self._obs, self._act, rew.to(torch.float32).unsqueeze(1), out["obs"],
                                    terminal.to(torch.float32).unsqueeze(1), mask=ready)
        self._path_len += ready.to(torch.int32)
        self._ret += torch.where(ready, rew, torch.zeros_like(rew))
        end = ready & (done | (self._path_len >= self.max_path_length))
        self._obs = torch.where(ready.unsqueeze(1), out["obs"], self._obs)
        self._awaiting = ready.clone()
        n_ready = ready.sum()
        self._steps_total += n_ready
        self._paths_total += end.sum()
        self._ticks_total += out["ticks"].sum()
        self._last_end = end
        self._last_end_ret = torch.where(end, self._ret, torch.zeros_like(self._ret))
        self._last_end_len = torch.where(end, self._path_len, torch.zeros_like(self._path_len))
        # masked auto-reset of finished episodes
        self._env.reset(mask=end.to(torch.uint8), obs_out=self._obs_reset)
        self._obs = torch.where(end.unsqueeze(1), self._obs_reset, self._obs)
        self._path_len.masked_fill_(end, 0)
        self._ret.masked_fill_(end, 0.0)
        return ready, n_ready

    def collect(self, num_steps, replay_buffer=None, record_paths=False):
        """Advance until ≥ num_steps transitions were produced (host sync once per pass)."""
        got = 0
        while got < num_steps:
            _, n = self.step(replay_buffer)
            got += int(n.item())
            if record_paths:
                e = self._last_end
                self._epoch_returns.append(self._last_end_ret[e].cpu().numpy())
                self._epoch_lens.append(self._last_end_len[e].cpu().numpy())
        return got

    # reference collector surface -------------------------------------------------------------
    def get_epoch_paths(self):
        return []

    def end_epoch(self, epoch):
        self._epoch_returns, self._epoch_lens = [], []

    def get_diagnostics(self):
        st = OrderedDict([("num steps total", int(self._steps_total.item())),
                          ("num paths total", int(self._paths_total.item())),
                          ("num env ticks total", int(self._ticks_total.item()))])
        if self._epoch_lens:
            lens = np.concatenate(self._epoch_lens)
            rets = np.concatenate(self._epoch_returns)
            if lens.size:
                st.update(create_stats_ordered_dict("path length", lens, always_show_all_stats=True))
                st.update(create_stats_ordered_dict("Returns", rets, always_show_all_stats=True))
        return st

    def get_snapshot(self):
        return dict(policy=self._policy)
