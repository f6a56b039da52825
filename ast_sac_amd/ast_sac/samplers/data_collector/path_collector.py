"""MdpPathCollector (ast_sac/samplers/data_collector/path_collector.py:9-99)."""
from collections import deque, OrderedDict

from ...core.eval_util import create_stats_ordered_dict
from .rollout_functions import ast_sac_rollout


class MdpPathCollector:
    def __init__(self, env, policy, max_num_epoch_paths_saved=None, render=False, render_kwargs=None,
                 rollout_fn=ast_sac_rollout, save_env_in_snapshot=True):
        self._env = env
        self._policy = policy
        self._max_num_epoch_paths_saved = max_num_epoch_paths_saved
        self._epoch_paths = deque(maxlen=max_num_epoch_paths_saved)
        self._render = render
        self._render_kwargs = render_kwargs or {}
        self._rollout_fn = rollout_fn
        self._num_steps_total = 0
        self._num_paths_total = 0
        self._save_env_in_snapshot = save_env_in_snapshot

    def collect_new_paths(self, max_path_length, num_steps, discard_incomplete_paths):
        """Whole episodes until num_steps decisions; the last one is cut to the remaining budget and
        dropped when incomplete and discard_incomplete_paths (path_collector.py:36-75)."""
        paths = []
        collected = 0
        while collected < num_steps:
            mpl = min(max_path_length, num_steps - collected)
            path = self._rollout_fn(self._env, self._policy, max_path_length=mpl, render=self._render,
                                    render_kwargs=self._render_kwargs)
            path_len = len(path["actions"])
            if path_len != max_path_length and not path["dones"][-1] and discard_incomplete_paths:
                break
            collected += path_len
            paths.append(path)
        self._num_paths_total += len(paths)
        self._num_steps_total += collected
        self._epoch_paths.extend(paths)
        return paths

    def get_epoch_paths(self):
        return self._epoch_paths

    def end_epoch(self, epoch):
        self._epoch_paths = deque(maxlen=self._max_num_epoch_paths_saved)

    def get_diagnostics(self):
        lens = [len(p["actions"]) for p in self._epoch_paths]
        stats = OrderedDict([("num steps total", self._num_steps_total), ("num paths total", self._num_paths_total)])
        stats.update(create_stats_ordered_dict("path length", lens, always_show_all_stats=True))
        return stats

    def get_snapshot(self):
        snap = dict(policy=self._policy)
        if self._save_env_in_snapshot:
            snap["env"] = self._env
        return snap
