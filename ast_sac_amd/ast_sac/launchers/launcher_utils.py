"""setup_logger (ast_sac/launchers/launcher_utils.py:197-330), without git-info capture."""
import datetime
import json
import os
import os.path as osp

from ..core.logging import logger

LOCAL_LOG_DIR = osp.join(os.getcwd(), "data")


def create_exp_name(exp_prefix, exp_id=0, seed=0):
    now = datetime.datetime.now()
    return "%s_%s_%04d--s-%d" % (exp_prefix, now.strftime("%Y_%m_%d_%H_%M_%S"), exp_id, seed)


def create_log_dir(exp_prefix, exp_id=0, seed=0, base_log_dir=None, include_exp_prefix_sub_dir=True):
    exp_name = create_exp_name(exp_prefix, exp_id=exp_id, seed=seed)
    base_log_dir = base_log_dir or LOCAL_LOG_DIR
    log_dir = (osp.join(base_log_dir, exp_prefix.replace("_", "-"), exp_name) if include_exp_prefix_sub_dir
               else osp.join(base_log_dir, exp_name))
    os.makedirs(log_dir, exist_ok=True)
    return log_dir


def setup_logger(exp_prefix="default", variant=None, text_log_file="debug.log", variant_log_file="variant.json",
                 tabular_log_file="progress.csv", snapshot_mode="last", snapshot_gap=1, log_tabular_only=False,
                 log_dir=None, git_infos=None, script_name=None, **create_log_dir_kwargs):
    first_time = log_dir is None
    if first_time:
        log_dir = create_log_dir(exp_prefix, **create_log_dir_kwargs)
    os.makedirs(log_dir, exist_ok=True)
    if variant is not None:
        logger.log("Variant:")
        logger.log(json.dumps(variant, indent=2, default=repr))
        logger.log_variant(osp.join(log_dir, variant_log_file), variant)
    logger.add_text_output(osp.join(log_dir, text_log_file))
    logger.add_tabular_output(osp.join(log_dir, tabular_log_file), mode="w" if first_time else "a")
    logger.set_snapshot_dir(log_dir)
    logger.set_snapshot_mode(snapshot_mode)
    logger.set_snapshot_gap(snapshot_gap)
    logger.set_log_tabular_only(log_tabular_only)
    logger.push_prefix("[%s] " % log_dir.rstrip("/").split("/")[-1])
    if script_name is not None:
        with open(osp.join(log_dir, "script_name.txt"), "w") as f:
            f.write(script_name)
    return log_dir
