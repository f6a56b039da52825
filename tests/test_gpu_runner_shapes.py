"""The reference runner's argument space on the hip backend (run/ast-sac_runner.py:51,55,
121-153 take any --layer_size / --batch_size): the device experiment trains with 2x512 networks and a batch of
100 (not a multiple of 32) — libsacfused's two-chunk K slices and padded row tiles — for one epoch, the
collector's policy inside the env launch at both widths (the in-kernel fc1 in two 256-unit slices at 512). Needs an MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layer,batch", [(512, 100), (256, 100)])
def test_runner_trains_on_hip_backend(layer, batch):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ast_sac_amd.run.ast_sac_runner import parse_cli_args, make_variant, experiment_device
    args = parse_cli_args(["--n_envs", "1024", "--layer_size", str(layer), "--batch_size", str(batch),
                           "--num_epochs", "1", "--min_num_steps_before_training", "1024",
                           "--num_expl_steps_per_train_loop", "1024", "--num_eval_steps_per_epoch", "64",
                           "--do_logging", "false", "--seed", "3"])
    torch.manual_seed(3)
    np.random.seed(3)
    algo = experiment_device(make_variant(args), args, torch.device("cuda", 0))
    tr = algo.trainer
    assert tr.backend == "hip" and tr.batch_size == batch
    assert tr.policy.fcs[1].weight.shape == (layer, layer)
    assert algo.expl_data_collector.fused
    before = tr.flat_param.clone()
    algo.log_stats = False
    algo.train()
    torch.cuda.synchronize()
    assert algo.num_train_steps_total > 0
    # the reference's update ratio: num_trains_per_train_loop (240) per num_expl_steps_per_train_loop (1024 here)
    assert abs(algo.num_train_steps_total - algo.num_loop_expl_steps_total * 240 / 1024) < 1 + 1e-9
    assert torch.isfinite(tr.flat_param).all() and torch.isfinite(tr.flat_target).all()
    assert not torch.equal(before, tr.flat_param)
    d = tr.get_diagnostics()
    assert np.isfinite(d["QF1 Loss"]) and np.isfinite(d["Policy Loss"]) and np.isfinite(d["Alpha"])
    assert int(tr._step_t.item()) == algo.num_train_steps_total
