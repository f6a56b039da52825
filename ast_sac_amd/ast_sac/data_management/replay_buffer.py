"""Replay buffers.

* `SimpleReplayBuffer` / `EnvReplayBuffer` — the reference host ring buffer (numpy fp64, uint8
  terminals; uniform sampling with replacement via np.random.choice)
  (data_management/simple_replay_buffer.py:8-103, env_replay_buffer.py:8-50, replay_buffer.py:34-77).
* `DeviceReplayBuffer` — the same ring + uniform-with-replacement sampler resident in HBM
  (fp32 obs/actions/next_obs, fp32 rewards, fp32 terminals), filled straight from the batched
  device env and sampled on-device (torch.randint + gather), so the SAC update never touches the
  host. The batch it returns is what SACTrainer.compute_loss consumes after
  np_to_pytorch_batch (everything float32), so the arithmetic downstream is unchanged.
"""
import abc
import warnings
from collections import OrderedDict

import numpy as np
import torch

from ..env_wrapper.env_utils import get_dim


class ReplayBuffer(metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def add_sample(self, observation, action, reward, next_observation, terminal, **kwargs):
        pass

    @abc.abstractmethod
    def terminate_episode(self):
        pass

    @abc.abstractmethod
    def num_steps_can_sample(self, **kwargs):
        pass

    def add_path(self, path):
        for obs, action, reward, next_obs, terminal, agent_info, env_info in zip(
                path["observations"], path["actions"], path["rewards"], path["next_observations"],
                path["terminals"], path["agent_infos"], path["env_infos"]):
            self.add_sample(observation=obs, action=action, reward=reward, next_observation=next_obs,
                            terminal=terminal, agent_info=agent_info, env_info=env_info)
        self.terminate_episode()

    def add_paths(self, paths):
        for path in paths:
            self.add_path(path)

    @abc.abstractmethod
    def random_batch(self, batch_size):
        pass

    def get_diagnostics(self):
        return {}

    def get_snapshot(self):
        return {}

    def end_epoch(self, epoch):
        return


class SimpleReplayBuffer(ReplayBuffer):
    def __init__(self, max_replay_buffer_size, observation_dim, action_dim, env_info_sizes, replace=True):
        self._observation_dim = observation_dim
        self._action_dim = action_dim
        self._max_replay_buffer_size = max_replay_buffer_size
        self._observations = np.zeros((max_replay_buffer_size, observation_dim))
        self._next_obs = np.zeros((max_replay_buffer_size, observation_dim))
        self._actions = np.zeros((max_replay_buffer_size, action_dim))
        self._rewards = np.zeros((max_replay_buffer_size, 1))
        self._terminals = np.zeros((max_replay_buffer_size, 1), dtype="uint8")
        self._env_infos = {k: np.zeros((max_replay_buffer_size, s)) for k, s in env_info_sizes.items()}
        self._env_info_keys = list(env_info_sizes.keys())
        self._replace = replace
        self._top = 0
        self._size = 0

    def add_sample(self, observation, action, reward, next_observation, terminal, env_info=None, **kwargs):
        t = self._top
        self._observations[t] = observation
        self._actions[t] = action
        self._rewards[t] = reward
        self._terminals[t] = terminal
        self._next_obs[t] = next_observation
        for key in self._env_info_keys:
            self._env_infos[key][t] = env_info[key]
        self._advance()

    def terminate_episode(self):
        pass

    def clear(self):
        self._top = 0
        self._size = 0

    def _advance(self):
        self._top = (self._top + 1) % self._max_replay_buffer_size
        if self._size < self._max_replay_buffer_size:
            self._size += 1

    def random_batch(self, batch_size):
        indices = np.random.choice(self._size, size=batch_size, replace=self._replace or self._size < batch_size)
        if not self._replace and self._size < batch_size:
            warnings.warn("Replace was set to false, but is temporarily set to true because batch size is larger "
                          "than current size of replay.")
        batch = dict(observations=self._observations[indices], actions=self._actions[indices],
                     rewards=self._rewards[indices], terminals=self._terminals[indices],
                     next_observations=self._next_obs[indices])
        for key in self._env_info_keys:
            batch[key] = self._env_infos[key][indices]
        return batch

    def num_steps_can_sample(self):
        return self._size

    def get_diagnostics(self):
        return OrderedDict([("size", self._size)])


class EnvReplayBuffer(SimpleReplayBuffer):
    def __init__(self, max_replay_buffer_size, env, env_info_sizes=None):
        self.env = env
        self._ob_space = env.observation_space
        self._action_space = env.action_space
        if env_info_sizes is None:
            env_info_sizes = getattr(env, "info_sizes", dict())
        super().__init__(max_replay_buffer_size=max_replay_buffer_size, observation_dim=get_dim(self._ob_space),
                         action_dim=get_dim(self._action_space), env_info_sizes=env_info_sizes)

    def add_sample(self, observation, action, reward, terminal, next_observation, **kwargs):
        if hasattr(self._action_space, "n"):
            new_action = np.zeros(self._action_dim)
            new_action[action] = 1
        else:
            new_action = action
        return super().add_sample(observation=observation, action=new_action, reward=reward,
                                  next_observation=next_observation, terminal=terminal, **kwargs)


class DeviceReplayBuffer(ReplayBuffer):
    """Ring buffer in device memory; uniform sampling with replacement (simple_replay_buffer.py:72-76).

    One (obs, action, reward, next_obs, terminal) row = (8 + 1 + 1 + 8 + 1) · 4 B = 76 B; the
    runner's 300,000 rows are 22.8 MB per GPU. `add_batch` appends a masked set of rows (the
    envs whose decision completed) with one prefix-sum scatter and no host sync.
    """

    def __init__(self, max_replay_buffer_size, observation_dim, action_dim, device, generator=None):
        self._max = int(max_replay_buffer_size)
        self.device = torch.device(device)
        f = dict(dtype=torch.float32, device=self.device)
        # one spare row at the end absorbs the scatter of rows a masked add does not keep
        self._store = dict(observations=torch.zeros((self._max + 1, observation_dim), **f),
                           next_observations=torch.zeros((self._max + 1, observation_dim), **f),
                           actions=torch.zeros((self._max + 1, action_dim), **f),
                           rewards=torch.zeros((self._max + 1, 1), **f),
                           terminals=torch.zeros((self._max + 1, 1), **f))
        self._observations = self._store["observations"][:self._max]
        self._next_obs = self._store["next_observations"][:self._max]
        self._actions = self._store["actions"][:self._max]
        self._rewards = self._store["rewards"][:self._max]
        self._terminals = self._store["terminals"][:self._max]
        # device-side top/size so add_batch and random_batch never sync with the host
        self._top_t = torch.zeros((), dtype=torch.int64, device=self.device)
        self._size_t = torch.zeros((), dtype=torch.int64, device=self.device)
        self.generator = generator

    # -- reference-compatible per-sample path --
    def add_sample(self, observation, action, reward, next_observation, terminal, **kwargs):
        one = torch.ones(1, dtype=torch.bool, device=self.device)
        t = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32), device=self.device).reshape(1, -1)
        self.add_batch(t(observation), t(action), t(reward), t(next_observation), t(terminal), one)

    def terminate_episode(self):
        pass

    def add_batch(self, obs, action, reward, next_obs, terminal, mask=None):
        """Append rows where mask is True (all rows if None), in row order."""
        n = obs.shape[0]
        if n > self._max:
            raise ValueError(f"add_batch of {n} rows exceeds the buffer size {self._max}")
        if mask is None:
            mask = torch.ones(n, dtype=torch.bool, device=self.device)
        mask = mask.reshape(-1).bool()
        m64 = mask.to(torch.int64)
        pos = (torch.cumsum(m64, 0) - m64 + self._top_t) % self._max
        idx = torch.where(mask, pos, torch.full_like(pos, self._max))
        for k, val in (("observations", obs), ("next_observations", next_obs), ("actions", action),
                       ("rewards", reward), ("terminals", terminal)):
            buf = self._store[k]
            buf.index_copy_(0, idx, val.reshape(n, -1).to(buf.dtype))
        cnt = m64.sum()
        self._top_t.copy_((self._top_t + cnt) % self._max)
        self._size_t.copy_(torch.clamp(self._size_t + cnt, max=self._max))

    def add_capacity(self):
        """Rows one add_batch can take."""
        return self._max

    def random_batch(self, batch_size, out=None):
        """Uniform with replacement over the filled rows; returns device tensors (float32)."""
        size = self._size_t.clamp(min=1)
        u = torch.rand(batch_size, device=self.device, generator=self.generator, dtype=torch.float64)
        idx = torch.clamp((u * size).to(torch.int64), max=self._max - 1)
        if out is None:
            return dict(observations=self._observations[idx], actions=self._actions[idx],
                        rewards=self._rewards[idx], terminals=self._terminals[idx],
                        next_observations=self._next_obs[idx])
        for k, buf in (("observations", self._observations), ("actions", self._actions),
                       ("rewards", self._rewards), ("terminals", self._terminals),
                       ("next_observations", self._next_obs)):
            torch.index_select(buf, 0, idx, out=out[k])
        return out

    def num_steps_can_sample(self):
        return int(self._size_t.item())

    def get_diagnostics(self):
        return OrderedDict([("size", self.num_steps_can_sample())])


class ReplicatedReplayBuffer(DeviceReplayBuffer):
    """The union of every rank's transitions, held identically by every rank of `process_group` — the
    replicated-trainer data-parallel shape. `add_batch` (the collector's, graph-capturable)
    stages this rank's rows; `sync()` all-gathers every rank's staged rows — once per train loop (a count, then the rows),
    76 B per row, instead of one gradient all-reduce per grad step — and appends them in rank order, so
    every rank's ring holds the same rows in the same slots. Every rank then runs the same SAC step on the
    same global batch (the reference's uniform sample over all collected transitions, replay_buffer.py /
    simple_replay_buffer.py:72-76) with the same seed, and the replicas stay bitwise equal without any
    per-step exchange. A sync is two all-gathers: the ranks' staged-row counts (one int64 each), then the rows
    (the largest count of rows from every rank)."""

    def __init__(self, max_replay_buffer_size, observation_dim, action_dim, device, process_group, stage_size,
                 generator=None):
        super().__init__(max_replay_buffer_size, observation_dim, action_dim, device, generator)
        self.pg = process_group
        self._stage = DeviceReplayBuffer(int(stage_size), observation_dim, action_dim, device)
        self._staged_t = torch.zeros((), dtype=torch.int64, device=self.device)  # rows added since the last sync
        self._dims = (observation_dim, action_dim)

    def add_batch(self, obs, action, reward, next_obs, terminal, mask=None):
        n = obs.shape[0]
        self._stage.add_batch(obs, action, reward, next_obs, terminal, mask)
        self._staged_t += n if mask is None else mask.reshape(-1).to(torch.int64).sum()

    def add_capacity(self):
        """Rows one add_batch can take: the staging ring's."""
        return self._stage._max

    def staging_room(self):
        """Rows that can still be staged before the next sync (a host read of the device count)."""
        return self._stage._max - int(self._staged_t.item())

    def sync(self):
        """Append every rank's staged rows (rank order) to the shared ring; returns the rows appended."""
        import torch.distributed as dist
        od, ad = self._dims
        world = dist.get_world_size(self.pg)
        comm_dev = self.device if dist.get_backend(self.pg) == "nccl" else torch.device("cpu")
        cnt = self._staged_t.reshape(1).to(comm_dev)
        counts = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(counts, cnt, group=self.pg)
        counts = [int(c.item()) for c in counts]
        if max(counts) > self._stage._max:
            raise RuntimeError(f"ReplicatedReplayBuffer: a rank staged {max(counts)} rows between syncs, more than "
                               f"the staging ring's {self._stage._max}; sync after every collect or enlarge stage_size")
        m = max(counts)
        if m:
            st = self._stage._store
            rows = torch.cat([st["observations"][:m], st["actions"][:m], st["rewards"][:m], st["next_observations"][:m],
                              st["terminals"][:m]], 1).to(comm_dev).contiguous()
            got = [torch.empty_like(rows) for _ in range(world)]
            dist.all_gather(got, rows, group=self.pg)
            for r, c in enumerate(counts):
                if not c:
                    continue
                x = got[r][:c].to(self.device)
                DeviceReplayBuffer.add_batch(self, x[:, :od], x[:, od:od + ad], x[:, od + ad:od + ad + 1],
                                             x[:, od + ad + 1:2 * od + ad + 1], x[:, 2 * od + ad + 1:])
        self._stage._top_t.zero_()
        self._stage._size_t.zero_()
        self._staged_t.zero_()
        return sum(counts)
