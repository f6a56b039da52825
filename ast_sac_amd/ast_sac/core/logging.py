"""Tabular/text logger and snapshot writer (subset of ast_sac/core/logging.py used by the runner).

progress.csv keeps the reference rule: the column set is fixed by the first dump (sorted keys),
later rows write those columns only (logging.py:274-315). Snapshots: torch.save of the snapshot
dict, modes all / last / gap / gap_and_last / none (logging.py:316-338).
"""
import csv
import datetime
import json
import os
import os.path as osp
import time
from collections import OrderedDict
from contextlib import contextmanager

import numpy as np
import torch


class _Encoder(json.JSONEncoder):
    def default(self, o):
        if isinstance(o, type):
            return {"$class": o.__module__ + "." + o.__name__}
        if callable(o):
            return {"$function": getattr(o, "__module__", "?") + "." + getattr(o, "__name__", repr(o))}
        if isinstance(o, (np.integer,)):
            return int(o)
        if isinstance(o, (np.floating,)):
            return float(o)
        if isinstance(o, np.ndarray):
            return o.tolist()
        return repr(o)


class Logger:
    def __init__(self):
        self._prefixes = []
        self._prefix_str = ""
        self._tabular_prefixes = []
        self._tabular_prefix_str = ""
        self._tabular = []
        self._text_fds = {}
        self._tabular_fds = {}
        self._tabular_keys = {}
        self._tabular_header_written = set()
        self._snapshot_dir = None
        self._snapshot_mode = "all"
        self._snapshot_gap = 1
        self._log_tabular_only = False
        self.quiet = False

    def reset(self):
        self.__init__()

    def add_text_output(self, file_name):
        os.makedirs(osp.dirname(file_name) or ".", exist_ok=True)
        if file_name not in self._text_fds:
            self._text_fds[file_name] = open(file_name, "a")

    def add_tabular_output(self, file_name, mode="w"):
        os.makedirs(osp.dirname(file_name) or ".", exist_ok=True)
        if file_name not in self._tabular_fds:
            self._tabular_fds[file_name] = open(file_name, mode)

    def remove_tabular_output(self, file_name):
        fd = self._tabular_fds.pop(file_name, None)
        if fd is not None:
            self._tabular_header_written.discard(fd)
            self._tabular_keys.pop(file_name, None)
            fd.close()

    def set_snapshot_dir(self, d):
        self._snapshot_dir = d

    def get_snapshot_dir(self):
        return self._snapshot_dir

    def set_snapshot_mode(self, mode):
        self._snapshot_mode = mode

    def set_snapshot_gap(self, gap):
        self._snapshot_gap = gap

    def set_log_tabular_only(self, v):
        self._log_tabular_only = v

    def push_prefix(self, prefix):
        self._prefixes.append(prefix)
        self._prefix_str = "".join(self._prefixes)

    def pop_prefix(self):
        del self._prefixes[-1]
        self._prefix_str = "".join(self._prefixes)

    def push_tabular_prefix(self, key):
        self._tabular_prefixes.append(key)
        self._tabular_prefix_str = "".join(self._tabular_prefixes)

    def pop_tabular_prefix(self):
        del self._tabular_prefixes[-1]
        self._tabular_prefix_str = "".join(self._tabular_prefixes)

    @contextmanager
    def tabular_prefix(self, key):
        self.push_tabular_prefix(key)
        yield
        self.pop_tabular_prefix()

    def log(self, s, with_prefix=True, with_timestamp=True):
        out = s
        if with_prefix:
            out = self._prefix_str + out
        if with_timestamp:
            out = datetime.datetime.now().strftime("%Y-%m-%d %H:%M:%S.%f %Z") + " | " + out
        if not self._log_tabular_only and not self.quiet:
            print(out)
        for fd in self._text_fds.values():
            fd.write(out + "\n")
            fd.flush()

    def record_tabular(self, key, val):
        self._tabular.append((self._tabular_prefix_str + str(key), str(val)))

    def record_dict(self, d, prefix=None):
        if prefix is not None:
            self.push_tabular_prefix(prefix)
        for k, v in d.items():
            self.record_tabular(k, v)
        if prefix is not None:
            self.pop_tabular_prefix()

    def get_table_dict(self):
        return dict(self._tabular)

    def log_variant(self, log_file, variant_data):
        os.makedirs(osp.dirname(log_file) or ".", exist_ok=True)
        with open(log_file, "w") as f:
            json.dump(variant_data, f, indent=2, sort_keys=True, cls=_Encoder)

    def dump_tabular(self, *args, **kwargs):
        wh = kwargs.pop("write_header", None)
        if not self._tabular:
            return
        if not self._log_tabular_only:
            width = max(len(k) for k, _ in self._tabular)
            for k, v in self._tabular:
                self.log(f"{k:<{width}}  {v}", *args, **kwargs)
        row = dict(self._tabular)
        for filename, fd in list(self._tabular_fds.items()):
            keys = self._tabular_keys.get(filename)
            if keys is None:
                keys = sorted(row.keys())
                self._tabular_keys[filename] = keys
            w = csv.DictWriter(fd, fieldnames=keys, extrasaction="ignore")
            if wh or (wh is None and fd not in self._tabular_header_written):
                w.writeheader()
                self._tabular_header_written.add(fd)
            w.writerow(row)
            fd.flush()
        del self._tabular[:]

    def save_itr_params(self, itr, params):
        if not self._snapshot_dir:
            return
        mode = self._snapshot_mode
        if mode == "all" or (mode in ("gap", "gap_and_last") and itr % self._snapshot_gap == 0):
            torch.save(params, osp.join(self._snapshot_dir, f"itr_{itr}.pkl"))
        if mode in ("last", "gap_and_last"):
            torch.save(params, osp.join(self._snapshot_dir, "params.pkl"))
        elif mode not in ("all", "gap", "none"):
            raise NotImplementedError(mode)


logger = Logger()


class EpochTimer:
    """Replaces the gtimer stamps the reference logs as `time/<stamp> (s)` (rl_algorithm.py:11-21)."""

    def __init__(self):
        self.t_start = time.perf_counter()
        self.reset_epoch()

    def reset_epoch(self):
        self._last = time.perf_counter()
        self.stamps = OrderedDict()

    def stamp(self, name):
        now = time.perf_counter()
        self.stamps[name] = self.stamps.get(name, 0.0) + now - self._last
        self._last = now

    def epoch_timings(self):
        times = OrderedDict()
        total = 0.0
        for k in sorted(self.stamps):
            times[f"time/{k} (s)"] = self.stamps[k]
            total += self.stamps[k]
        times["time/epoch (s)"] = total
        times["time/total (s)"] = time.perf_counter() - self.t_start
        return times
