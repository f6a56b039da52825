"""Path statistics for progress.csv (ast_sac/core/eval_util.py:10-117)."""
from collections import OrderedDict
from numbers import Number

import numpy as np


def list_of_dicts__to__dict_of_lists(lst):
    if len(lst) == 0:
        return {}
    keys = lst[0].keys()
    return {k: [d[k] for d in lst] for k in keys}


def get_generic_path_information(paths, stat_prefix=""):
    statistics = OrderedDict()
    if len(paths) == 0:
        return statistics
    returns = [sum(path["rewards"]) for path in paths]
    rewards = np.vstack([path["rewards"] for path in paths])
    statistics.update(create_stats_ordered_dict("Rewards", rewards, stat_prefix=stat_prefix))
    statistics.update(create_stats_ordered_dict("Returns", returns, stat_prefix=stat_prefix))
    actions = [path["actions"] for path in paths]
    if len(actions[0].shape) == 1:
        actions = np.hstack(actions)
    else:
        actions = np.vstack(actions)
    statistics.update(create_stats_ordered_dict("Actions", actions, stat_prefix=stat_prefix))
    statistics["Num Paths"] = len(paths)
    statistics[stat_prefix + "Average Returns"] = get_average_returns(paths)
    for info_key in ["env_infos", "agent_infos"]:
        if info_key in paths[0]:
            all_infos = [list_of_dicts__to__dict_of_lists(p[info_key]) for p in paths]
            if not all_infos[0]:
                continue
            for k in all_infos[0].keys():
                sample = all_infos[0][k][0]
                if not np.issubdtype(np.array(sample).dtype, np.number):
                    continue
                final_ks = np.array([info[k][-1] for info in all_infos])
                first_ks = np.array([info[k][0] for info in all_infos])
                all_ks = np.concatenate([np.atleast_1d(info[k]) for info in all_infos])
                statistics.update(create_stats_ordered_dict(stat_prefix + k, final_ks,
                                                            stat_prefix=f"{info_key}/final/"))
                statistics.update(create_stats_ordered_dict(stat_prefix + k, first_ks,
                                                            stat_prefix=f"{info_key}/initial/"))
                statistics.update(create_stats_ordered_dict(stat_prefix + k, all_ks, stat_prefix=f"{info_key}/"))
    return statistics


def get_average_returns(paths):
    return np.mean([sum(path["rewards"]) for path in paths])


def create_stats_ordered_dict(name, data, stat_prefix=None, always_show_all_stats=True, exclude_max_min=False):
    if stat_prefix is not None:
        name = f"{stat_prefix}{name}"
    if isinstance(data, Number):
        return OrderedDict({name: data})
    if len(data) == 0:
        return OrderedDict()
    if isinstance(data, tuple):
        od = OrderedDict()
        for number, d in enumerate(data):
            od.update(create_stats_ordered_dict(f"{name}_{number}", d))
        return od
    if isinstance(data, list):
        try:
            iter(data[0])
        except TypeError:
            pass
        else:
            data = np.concatenate(data)
    if isinstance(data, np.ndarray) and data.size == 1 and not always_show_all_stats:
        return OrderedDict({name: float(data)})
    stats = OrderedDict([(name + " Mean", np.mean(data)), (name + " Std", np.std(data))])
    if not exclude_max_min:
        stats[name + " Max"] = np.max(data)
        stats[name + " Min"] = np.min(data)
    return stats
