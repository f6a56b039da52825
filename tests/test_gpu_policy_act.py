"""The collector's policy on the matrix cores (libsacfused sacf_policy_act, FusedSACTrainer.device_policy)
against the same TanhGaussianPolicy in PyTorch fp32 ops (gaussian_policy.py:105-118, distributions.py:
394-425; MakeDeterministic policies/base.py:54-64), and the graph-replayed collector pass against the
eager one. Needs an MI355X."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Env:
    class action_space:
        shape = (1,)


def _trainer(H=256, seed=3):
    from ast_sac_amd.ast_sac.torch.networks.mlp import ConcatMlp
    from ast_sac_amd.ast_sac.torch.sac.policies.gaussian_policy import TanhGaussianPolicy
    from ast_sac_amd.ast_sac.torch.sac.sac_fused import FusedSACTrainer
    torch.manual_seed(seed)
    dev = torch.device("cuda", 0)
    pol = TanhGaussianPolicy(obs_dim=8, action_dim=1, hidden_sizes=[H, H]).to(dev)
    with torch.no_grad():  # raw AST observations are O(1e4): scale the first layer so tanh is not saturated
        pol.fcs[0].weight.mul_(1e-3)
        pol.last_fc_log_std.bias.fill_(-0.5)
    qs = [ConcatMlp(input_size=9, output_size=1, hidden_sizes=[H, H]).to(dev) for _ in range(4)]
    tr = FusedSACTrainer(env=_Env, policy=pol, qf1=qs[0], qf2=qs[1], target_qf1=qs[2], target_qf2=qs[3],
                         discount=0.965, reward_scale=0.75, policy_lr=8e-5, qf_lr=8e-5, soft_target_tau=1e-3,
                         action_reg_coeff=0.01, clip_val=100.0, batch_size=256, backend="hip")
    return tr, pol


def _obs(n, seed=1):
    g = torch.Generator().manual_seed(seed)
    o = torch.rand(n, 8, generator=g) * torch.tensor([10000, 20000, 3000, 10000, 20000, 6, 5, 500]) - \
        torch.tensor([0, 0, 1500, 0, 0, 3, 0, 250])
    return o.cuda()


@pytest.mark.parametrize("H,n", [(256, 8192), (256, 1000), (64, 77)])
def test_device_policy_matches_torch_policy(H, n):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    tr, pol = _trainer(H)
    obs = _obs(n)
    with torch.no_grad():
        dist = pol(obs)
        mean, std = dist.normal_mean, dist.normal_std
    # deterministic: tanh(mean)
    dp = tr.device_policy(deterministic=True)
    dp.reserve(n)
    act = torch.full((n, 1), 7.0, device="cuda")
    dp.act(obs, None, act)
    torch.cuda.synchronize()
    ref = torch.tanh(mean)
    err = (act - ref).abs().max().item()
    assert err < 5e-6, err
    # stochastic: tanh(mean + std * eps) with the kernel's eps, which is N(0, 1)
    sp = tr.device_policy(deterministic=False, seed=123)
    sp.reserve(n)
    eps = torch.zeros(n, device="cuda")
    act2 = torch.zeros((n, 1), device="cuda")
    sp.act(obs, None, act2, eps_out=eps)
    torch.cuda.synchronize()
    ref2 = torch.tanh(mean + std * eps[:, None])
    assert (act2 - ref2).abs().max().item() < 5e-6
    if n >= 4096:
        e = eps.double()
        assert abs(e.mean().item()) < 0.05 and abs(e.std().item() - 1) < 0.05
    # the counter advanced: a second call draws fresh noise; the mask keeps the unmasked rows
    eps_b = torch.zeros(n, device="cuda")
    mask = (torch.arange(n, device="cuda") % 3 == 0).to(torch.uint8)
    act3 = act2.clone()
    sp.act(obs, mask, act3, eps_out=eps_b)
    torch.cuda.synchronize()
    assert not torch.equal(eps, eps_b)
    keep = mask == 0
    assert torch.equal(act3[keep], act2[keep])
    ref3 = torch.tanh(mean + std * eps_b[:, None])
    assert (act3[~keep] - ref3[~keep]).abs().max().item() < 5e-6


def test_graph_replayed_collector_equals_eager_collector():
    """A deterministic device-policy collector: the HIP-graph pass and the eager pass produce the same
    transitions in the same replay rows and the same epoch paths."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ast_sac_amd.rl_env.ship_in_transit.env import BatchedMultiShipRLEnv, default_args
    from ast_sac_amd.ast_sac.env_wrapper.normalized_box_env import BatchedNormalizedBoxEnv
    from ast_sac_amd.ast_sac.samplers.data_collector.batched_collector import BatchedPathCollector
    from ast_sac_amd.ast_sac.data_management.replay_buffer import DeviceReplayBuffer
    tr, pol = _trainer(64)
    res = []
    for use_graph in (True, False):
        env = BatchedNormalizedBoxEnv(BatchedMultiShipRLEnv(default_args(collav_mode="sbmpc"), 512), 0.75)
        coll = BatchedPathCollector(env, pol, max_path_length=9, max_ticks=128, deterministic=True,
                                    device_policy=tr.device_policy(True), use_graph=use_graph)
        rb = DeviceReplayBuffer(40000, 8, 1, "cuda")
        got = coll.collect(6500, rb, record_paths=True)  # ~15 passes of 128 ticks: episodes end
        torch.cuda.synchronize()
        n = rb.num_steps_can_sample()
        res.append((got, n, {k: v[:n].cpu() for k, v in rb._store.items()},
                    [(p["rewards"].copy(), p["actions"].copy()) for p in coll.get_epoch_paths()],
                    int(coll._ticks_total.item())))
    (g1, n1, s1, p1, t1), (g2, n2, s2, p2, t2) = res
    assert g1 == g2 and n1 == n2 and t1 == t2 and n1 >= 6500
    for k in s1:
        assert torch.equal(s1[k], s2[k]), k
    assert len(p1) == len(p2) > 0
    for (r1, a1), (r2, a2) in zip(p1, p2):
        np.testing.assert_array_equal(r1, r2)
        np.testing.assert_array_equal(a1, a2)
