"""The algebra of libsacfused's three-pass grad step (csrc/sac_kernels.hip), restated in float64
torch and checked against autograd of the reference losses (sac.py:156-270) — no GPU involved:

* ∂Q/∂ã as the forward-mode tangent of Q along the 1-d action: v = ([g1 > 0] ⊙ W1[:, a]) W2ᵀ,
  ∂Q/∂ã = Σ w3 ⊙ [g2 > 0] ⊙ v (computed beside Q(obs, ã) on the same W2 operand, P2);
* the input gradients as per-row scalings of backward factors formed from forward masks only:
  dh1 = dmean·U_m + dls·U_s with U_h = ((h_w ⊙ [h2 > 0]) W2) ⊙ [h1 > 0] (actor), dg1 = dq·U_q (critics);
* every weight gradient from those per-row scalars (P3).
"""
import numpy as np
import torch

LOG2 = float(np.log(2.0))


def _nets(H, O, g):
    def lin(o, i):
        return torch.randn(o, i, generator=g) / np.sqrt(i), torch.randn(o, generator=g) * 0.1
    pol = dict(zip(("w1", "b1"), lin(H, O))) | dict(zip(("w2", "b2"), lin(H, H))) | \
        dict(zip(("wm", "bm"), lin(1, H))) | dict(zip(("ws", "bs"), lin(1, H)))
    qs = []
    for _ in range(4):
        qs.append(dict(zip(("w1", "b1"), lin(H, O + 1))) | dict(zip(("w2", "b2"), lin(H, H))) |
                  dict(zip(("w3", "b3"), lin(1, H))))
    return pol, qs


def _q(q, x):
    g1 = torch.relu(x @ q["w1"].T + q["b1"])
    g2 = torch.relu(g1 @ q["w2"].T + q["b2"])
    return (g2 @ q["w3"].T + q["b3"])[:, 0], g1, g2


def _losses(pol, qs, log_alpha, b, eps, hp):
    obs, act, rew, term, nobs = b
    B = obs.shape[0]
    h1 = torch.relu(torch.cat([obs, nobs]) @ pol["w1"].T + pol["b1"])
    h2 = torch.relu(h1 @ pol["w2"].T + pol["b2"])
    mean = (h2 @ pol["wm"].T + pol["bm"])[:, 0]
    ls = torch.clamp((h2 @ pol["ws"].T + pol["bs"])[:, 0], -20, 2)
    std = torch.exp(ls)
    z = mean + std * eps
    a = torch.tanh(z)
    logp = -((z - mean) ** 2) / (2 * std ** 2) - torch.log(std) - 0.5 * np.log(2 * np.pi) \
        - 2.0 * (LOG2 - z - torch.nn.functional.softplus(-2.0 * z))
    alpha = torch.exp(log_alpha).detach()
    q1a = _q(qs[0], torch.cat([obs, a[:B, None]], 1))[0]
    q2a = _q(qs[1], torch.cat([obs, a[:B, None]], 1))[0]
    pl = (alpha * logp[:B] - torch.min(q1a, q2a)).mean() + hp["areg"] * (a[:B] ** 2).mean()
    with torch.no_grad():
        t1 = _q(qs[2], torch.cat([nobs, a[B:, None]], 1))[0]
        t2 = _q(qs[3], torch.cat([nobs, a[B:, None]], 1))[0]
        y = torch.clamp(hp["rs"] * rew + (1 - term) * hp["gamma"] * (torch.min(t1, t2) - alpha * logp[B:]),
                        -hp["clip"], hp["clip"])
    q1 = _q(qs[0], torch.cat([obs, act[:, None]], 1))[0]
    q2 = _q(qs[1], torch.cat([obs, act[:, None]], 1))[0]
    return pl, ((q1 - y) ** 2).mean(), ((q2 - y) ** 2).mean()


def _three_pass(pol, qs, log_alpha, b, eps, hp):
    """What the kernels compute, in their order (float64 here)."""
    obs, act, rew, term, nobs = b
    B = obs.shape[0]
    alpha = float(torch.exp(log_alpha))
    invB = 1.0 / B
    # P1: actor forward (obs rows), critics on the data rows
    h1 = torch.relu(obs @ pol["w1"].T + pol["b1"])
    h2 = torch.relu(h1 @ pol["w2"].T + pol["b2"])
    mean = (h2 @ pol["wm"].T + pol["bm"])[:, 0]
    ls_raw = (h2 @ pol["ws"].T + pol["bs"])[:, 0]
    h1n = torch.relu(nobs @ pol["w1"].T + pol["b1"])
    h2n = torch.relu(h1n @ pol["w2"].T + pol["b2"])
    mean_n = (h2n @ pol["wm"].T + pol["bm"])[:, 0]
    ls_n = (h2n @ pol["ws"].T + pol["bs"])[:, 0]
    xd = torch.cat([obs, act[:, None]], 1)
    qd, gd1, gd2 = zip(*[_q(qs[k], xd) for k in range(2)])

    def head(m, l, e):
        std = torch.exp(torch.clamp(l, -20, 2))
        z = m + std * e
        a = torch.tanh(z)
        lp = -((z - m) ** 2) / (2 * std ** 2) - torch.log(std) - 0.5 * np.log(2 * np.pi) \
            - 2.0 * (LOG2 - z - torch.nn.functional.softplus(-2.0 * z))
        return std, z, a, lp
    std, z, a, logp = head(mean, ls_raw, eps[:B])
    _, _, an, logpn = head(mean_n, ls_n, eps[B:])
    # P2: Q on (obs, ã) with the action tangent; targets; backward factors
    qa, D = [], []
    for k in range(2):
        q = qs[k]
        x = torch.cat([obs, a[:, None]], 1)
        g1 = torch.relu(x @ q["w1"].T + q["b1"])
        t1 = (g1 > 0) * q["w1"][:, -1]                   # [g1 > 0] ⊙ W1[:, a]
        g2 = torch.relu(g1 @ q["w2"].T + q["b2"])
        v = t1 @ q["w2"].T                               # the tangent through layer 2 (pre-activation)
        qa.append((g2 @ q["w3"].T + q["b3"])[:, 0])
        D.append(((g2 > 0) * q["w3"][0] * v).sum(1))     # ∂Q/∂ã
    tq = [_q(qs[2 + k], torch.cat([nobs, an[:, None]], 1))[0] for k in range(2)]
    um = ((pol["wm"][0] * (h2 > 0)) @ pol["w2"]) * (h1 > 0)
    us = ((pol["ws"][0] * (h2 > 0)) @ pol["w2"]) * (h1 > 0)
    uq = [((qs[k]["w3"][0] * (gd2[k] > 0)) @ qs[k]["w2"]) * (gd1[k] > 0) for k in range(2)]
    # P3: per-row scalars, then every gradient
    y = torch.clamp(hp["rs"] * rew + (1 - term) * hp["gamma"] * (torch.min(tq[0], tq[1]) - alpha * logpn),
                    -hp["clip"], hp["clip"])
    dq = [2 * invB * (qd[k] - y) for k in range(2)]
    w1 = torch.where(qa[0] < qa[1], 1.0, torch.where(qa[0] == qa[1], 0.5, 0.0))
    dA = -w1 * invB * D[0] - (1 - w1) * invB * D[1] + hp["areg"] * invB * 2 * a
    ainv = alpha * invB
    d, var = z - mean, std * std
    sig = 1 / (1 + torch.exp(2 * z))
    gz = dA * (1 - a * a) + ainv * (-(d / var) + (2 - 4 * sig))
    dmean = gz + ainv * (d / var)
    dstd = gz * eps[:B] + ainv * (d * d / (var * std) - 1 / std)
    dls = torch.where((ls_raw >= -20) & (ls_raw <= 2), dstd * std, 0.0)
    dh1 = dmean[:, None] * um + dls[:, None] * us
    dh2 = (h2 > 0) * (dmean[:, None] * pol["wm"][0] + dls[:, None] * pol["ws"][0])
    g = dict(p_w1=dh1.T @ obs, p_b1=dh1.sum(0), p_w2=dh2.T @ h1, p_b2=dh2.sum(0), p_wm=(dmean[:, None] * h2).sum(0),
             p_bm=dmean.sum(), p_ws=(dls[:, None] * h2).sum(0), p_bs=dls.sum())
    for k in range(2):
        dg1 = dq[k][:, None] * uq[k]
        dg2 = (gd2[k] > 0) * (dq[k][:, None] * qs[k]["w3"][0])
        g |= {f"q{k}_w1": dg1.T @ xd, f"q{k}_b1": dg1.sum(0), f"q{k}_w2": dg2.T @ gd1[k], f"q{k}_b2": dg2.sum(0),
              f"q{k}_w3": (dq[k][:, None] * gd2[k]).sum(0), f"q{k}_b3": dq[k].sum()}
    return g


def test_three_pass_gradients_equal_autograd():
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)  # (restored below: other tests build float32 buffers)
    try:
        _check_three_pass()
    finally:
        torch.set_default_dtype(prev)


def _check_three_pass():
    gen = torch.Generator().manual_seed(4)
    H, O, B = 48, 8, 37
    pol, qs = _nets(H, O, gen)
    b = (torch.randn(B, O, generator=gen) * 3, torch.rand(B, generator=gen) * 2 - 1, torch.randn(B, generator=gen),
         (torch.rand(B, generator=gen) < 0.2).double(), torch.randn(B, O, generator=gen) * 3)
    eps = torch.randn(2 * B, generator=gen)
    hp = dict(areg=0.01, rs=0.75, gamma=0.965, clip=100.0)
    log_alpha = torch.tensor(-0.3)
    for d in [pol] + qs[:2]:
        for v in d.values():
            v.requires_grad_(True)
    pl, l1, l2 = _losses(pol, qs, log_alpha, b, eps, hp)
    gp = torch.autograd.grad(pl, list(pol.values()))
    gq = torch.autograd.grad(l1 + l2, list(qs[0].values()) + list(qs[1].values()))
    with torch.no_grad():
        g = _three_pass(pol, qs, log_alpha, b, eps, hp)
    ref = dict(zip(("p_w1", "p_b1", "p_w2", "p_b2", "p_wm", "p_bm", "p_ws", "p_bs"), gp))
    for k in range(2):
        ref |= dict(zip([f"q{k}_{n}" for n in ("w1", "b1", "w2", "b2", "w3", "b3")], gq[6 * k:6 * k + 6]))
    for name, r in ref.items():
        np.testing.assert_allclose(g[name].reshape(r.shape).numpy(), r.numpy(), rtol=1e-10, atol=1e-12, err_msg=name)
