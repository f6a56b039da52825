"""FusedSACTrainer — the SAC update (sac.py:102-300) restructured for MI355X.

The reference update is ~20 tiny GEMMs (B = 256, H = 256) plus ~150 elementwise kernels,
four optimizer steps and a soft update — launch-bound on any GPU. Restructuring, all exact
rewrites of the same math:

* every loss is built from the pre-step parameters and each optimizer reads only its own
  parameters' gradients, so the α → π → Q1 → Q2 step sequence equals one combined step:
  grads of (α-loss + π-loss) w.r.t. (log α, π) and of (Q1-loss + Q2-loss) w.r.t. (Q1, Q2) are
  taken from ONE forward graph (two autograd.grad calls; the π-loss gradient that the reference
  lets flow into Q1/Q2 is zeroed by their zero_grad before their own backward, so it is never
  computed here), then one fused Adam over two param groups (policy_lr / qf_lr);
* the actor runs once on [obs; next_obs] (2B rows); twin critics run as one batched GEMM per
  layer (torch.baddbmm over the stacked [Q1, Q2] weights) on [(obs, ã); (obs, a)] (2B rows);
  twin targets likewise on (next_obs, ã');
* the whole step — on-device batch sampling from DeviceReplayBuffer, forward, both grads,
  Adam, soft target update — is captured once in a HIP graph and replayed (capturable Adam).
  For data-parallel training the gradients are flattened into one bucket and averaged with a
  single RCCL all-reduce between two graph halves (one ≈550 KB bucket, xGMI
  latency-bound; α + π and Q1 + Q2 in one bucket because each optimizer reads only its own).

Two backends run this restructured step. backend="hip" (the default on a GPU; the runner's) calls
libsacfused (include/sac_fused.h, csrc/sac_kernels.hip): the forward / backward passes and the
H x H weight gradients as batched fp32 GEMMs on the matrix cores (v_mfma_f32_32x32x2_f32), with
Adam, the soft target update and the transposed-weight refresh fused into the weight-gradient
kernel when there is no all-reduce — three launches per step inside the HIP graph (the critics'
action gradient is a forward-mode tangent and the backward factors of layer 2 are formed beside the
forward pass, so no separate backward pass is launched). It raises ValueError for networks it does
not cover (two equal hidden layers of a width libsacfused compiles — every multiple of 32 up to 256,
and 320 / 384 / 448 / 512 —, act_dim 1, obs_dim <= 15, per-rank batch 1..8192). backend="torch" runs
the same step with PyTorch ops (any shape).

Numerics: fp32 like the reference; results equal SACTrainer's up to GEMM accumulation order
(tests/test_sac.py checks both against the captured reference step, tests/golden/sac_step.npz,
and the hip gradients against torch autograd).
"""
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

from ..utils import pytorch_util as ptu
from ..core.torch_rl_algorithm import TorchTrainer
from ..core.distributions import diag_normal_log_prob
from ..sac.policies.gaussian_policy import LOG_SIG_MIN, LOG_SIG_MAX
from ...core.eval_util import create_stats_ordered_dict
from .sac import SACLosses

_LOG2 = float(np.log(2.0))
_BATCH_KEYS = ("observations", "actions", "rewards", "terminals", "next_observations")


def _layers(mlp):
    return list(mlp.fcs) + [mlp.last_fc]


class FusedSACTrainer(TorchTrainer):
    def __init__(self, env, policy, qf1, qf2, target_qf1, target_qf2, discount=0.99, reward_scale=1.0,
                 policy_lr=1e-3, qf_lr=1e-3, optimizer_class=None, soft_target_tau=1e-2, target_update_period=1,
                 plotter=None, render_eval_paths=False, use_automatic_entropy_tuning=True, target_entropy=None,
                 action_reg_coeff=None, clip_val=np.inf, batch_size=256, use_graph=None, process_group=None,
                 backend=None, split_update=None, replicated=False, capture_collective=None):
        super().__init__()
        if target_update_period != 1:
            raise NotImplementedError("FusedSACTrainer soft-updates every step (runner: target_update_period=1)")
        self.env = env
        self.policy, self.qf1, self.qf2 = policy, qf1, qf2
        self.target_qf1, self.target_qf2 = target_qf1, target_qf2
        self.discount = float(discount)
        self.reward_scale = float(reward_scale)
        self.soft_target_tau = float(soft_target_tau)
        self.target_update_period = 1
        self.use_automatic_entropy_tuning = use_automatic_entropy_tuning
        self.action_reg_coeff = action_reg_coeff
        self.clip_val = float(clip_val)
        self.batch_size = int(batch_size)
        self.device = next(policy.parameters()).device
        dev = self.device
        if use_automatic_entropy_tuning:
            self.target_entropy = (-np.prod(env.action_space.shape).item() if target_entropy is None
                                   else target_entropy)
        else:
            self.target_entropy = 0.0
        self.log_alpha = torch.zeros(1, requires_grad=use_automatic_entropy_tuning, device=dev)
        self.pg = process_group
        # data-parallel shapes. replicated: every rank of process_group runs this same step on the
        # same global batch from a ReplicatedReplayBuffer (the union of all ranks' transitions) with the same seed,
        # so the replicas stay equal with no per-step exchange (parameters and the sampling seed are broadcast
        # once). Otherwise (gradient all-reduce): each rank takes its batch_size rows from its own buffer and the
        # flat gradient is all-reduced every step.
        self.replicated = bool(replicated) and process_group is not None
        self.world = (torch.distributed.get_world_size(process_group)
                      if process_group is not None and not self.replicated else 1)
        # the all-reduce step shape: grads | all-reduce over process_group | update. Default: whenever world > 1;
        # split_update=True forces it on one rank too (the all-reduce then runs over a world-size-1 group: the
        # same code path as N ranks, an identity on the values)
        self.split = (self.world > 1) if split_update is None else bool(split_update)
        if self.replicated and (self.split or capture_collective):
            # (every replica runs the whole global batch: an all-reduce would sum R identical gradients, and
            # Adam would apply them R times over)
            raise ValueError("replicated=True runs no gradient collective: split_update / capture_collective "
                             "belong to the all-reduce shape (replicated=False)")
        # the all-reduce inside the one captured HIP graph of the step (RCCL kernels are capturable) instead of
        # an eager call between two graph halves; default with an RCCL ("nccl") group
        nccl = process_group is not None and torch.distributed.get_backend(process_group) == "nccl"
        self.capture_collective = (self.split and nccl) if capture_collective is None else bool(capture_collective)

        self.pi_params = ([self.log_alpha] if use_automatic_entropy_tuning else []) + list(policy.parameters())
        self.q_params = list(qf1.parameters()) + list(qf2.parameters())
        self.t_params = list(target_qf1.parameters()) + list(target_qf2.parameters())
        fused = dev.type == "cuda"
        self.use_graph = fused if use_graph is None else bool(use_graph)
        self.optimizer = torch.optim.Adam([dict(params=self.pi_params, lr=policy_lr),
                                           dict(params=self.q_params, lr=qf_lr)],
                                          fused=fused, capturable=self.use_graph)
        # one flat gradient bucket; p.grad are persistent views into it
        params = self.pi_params + self.q_params
        self._numel = [p.numel() for p in params]
        self.flat_grad = torch.zeros(sum(self._numel), device=dev)
        self._grad_views = []
        off = 0
        for p, n in zip(params, self._numel):
            v = self.flat_grad[off:off + n].view_as(p)
            self._grad_views.append(v)
            p.grad = v
            off += n
        self.noise_fn = None  # callable(shape) -> ε for [obs; next_obs] rows; None = torch.randn
        self._static = None
        self._graphs = None
        # backend "hip": the fused kernels of libsacfused.so (csrc/sac_kernels.hip), the product path
        # on a HIP device; "torch": the PyTorch-op formulation above, chosen only explicitly (or on a
        # CPU device, where it is the test/reference path). No silent switch: networks the hip kernels
        # do not cover raise here instead of falling back.
        if backend is None:
            backend = "hip" if dev.type == "cuda" else "torch"
        if backend not in ("hip", "torch"):
            raise ValueError(f"backend must be 'hip' or 'torch', got {backend!r}")
        self.backend = backend
        if backend == "hip":
            if not self._hip_shapes_ok():
                raise ValueError("FusedSACTrainer hip backend: needs 2 equal hidden layers of a compiled width (multiples "
                                 "of 32 up to 256, 320, 384, 448, 512), act_dim 1, obs_dim <= 15 and a per-rank batch_size "
                                 "of 1..8192; pass backend='torch' to run these networks with PyTorch ops")
            self._init_hip(policy_lr, qf_lr)
        self._n_train_steps_total = 0
        self._need_to_update_eval_statistics = True
        self.eval_statistics = OrderedDict()

    # ---------------------------------------------------------------- hip backend
    def _hip_shapes_ok(self):
        from ....sacfused import hidden_supported
        pol, nets = self.policy, (self.qf1, self.qf2, self.target_qf1, self.target_qf2)
        try:
            H = pol.fcs[0].weight.shape[0]
            obs = pol.fcs[0].weight.shape[1]
            ok = (len(pol.fcs) == 2 and pol.fcs[1].weight.shape == (H, H) and pol.last_fc.weight.shape == (1, H)
                  and getattr(pol, "last_fc_log_std", None) is not None and hidden_supported(H)
                  and obs <= 15 and 1 <= self.batch_size <= 8192)
            for n in nets:
                ok = ok and len(n.fcs) == 2 and n.fcs[0].weight.shape == (H, obs + 1) \
                    and n.fcs[1].weight.shape == (H, H) and n.last_fc.weight.shape == (1, H)
            return bool(ok)
        except (AttributeError, IndexError):
            return False

    def _init_hip(self, policy_lr, qf_lr):
        from ....sacfused import SacFused
        dev = self.device
        H = self.policy.fcs[0].weight.shape[0]
        obs_dim = self.policy.fcs[0].weight.shape[1]
        pol_params = list(self.policy.parameters())
        with torch.no_grad():
            flat = torch.cat([self.log_alpha.detach().reshape(-1)] +
                             [p.detach().reshape(-1) for p in pol_params + self.q_params]).contiguous()
            tflat = torch.cat([p.detach().reshape(-1) for p in self.t_params]).contiguous()
        # the modules' parameters become views of the flat buffers the kernels update in place
        off = 1
        for p in pol_params + self.q_params:
            p.data = flat[off:off + p.numel()].view_as(p)
            p.grad = None
            off += p.numel()
        off = 0
        for p in self.t_params:
            p.data = tflat[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.log_alpha = flat[0:1]
        if self.use_automatic_entropy_tuning:
            self.pi_params = [self.log_alpha] + pol_params
        self.flat_param, self.flat_target = flat, tflat
        self.flat_grad = torch.zeros_like(flat)
        self._adam_m = torch.zeros_like(flat)
        self._adam_v = torch.zeros_like(flat)
        self._step_t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.optimizer = None
        self._sf = SacFused(obs_dim, H, self.batch_size, dev, self.discount, self.reward_scale, self.soft_target_tau,
                            self.action_reg_coeff, self.clip_val, float(self.target_entropy), policy_lr, qf_lr,
                            auto_entropy=self.use_automatic_entropy_tuning, world_size=self.world,
                            split_update=self.split)
        if self._sf.n_params != flat.numel() or self._sf.n_targets != tflat.numel():
            raise RuntimeError("hip backend: flat layout mismatch")
        self._stats_t = torch.zeros(self._sf.n_stats, device=dev)
        self._sf.bind(flat, tflat, self.flat_grad, self._adam_m, self._adam_v, self._step_t, self._stats_t)
        self._seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self._collective_warm = False
        self._eps_static = None
        self._replay_key = None

    def _hip_launch(self, replay_buffer, part, chain=0):
        sf = self._sf
        if part in ("a", "ab"):
            eps = self._eps_static if self.noise_fn is not None else None
            if chain:
                sf.grads_chain(chain, eps)
            else:
                sf.grads(None if replay_buffer is not None else self._static, eps)
        if part == "ab":
            sf.apply()
        elif part == "b":
            sf.apply()

    def _hip_step_prepare(self, replay_buffer):
        if replay_buffer is not None and self._replay_key != id(replay_buffer):
            st = replay_buffer._store
            self._sf.set_replay(st["observations"], st["actions"], st["rewards"], st["terminals"],
                                st["next_observations"], replay_buffer._size_t, replay_buffer._max, self._seed)
            self._replay_key = id(replay_buffer)
            self._graphs = None
            self._mgraph = None

    def _hip_step(self, replay_buffer):
        sf = self._sf
        self._hip_step_prepare(replay_buffer)
        if self.noise_fn is not None:
            eps = self.noise_fn((2 * self.batch_size, 1)).reshape(-1)
            if self._eps_static is None:
                self._eps_static = torch.empty(2 * self.batch_size, device=self.device)
                self._graphs = None
            self._eps_static.copy_(eps)
        key = (id(replay_buffer) if replay_buffer is not None else None, self.noise_fn is not None)
        if not self.use_graph:
            sf.set_stream()
            self._hip_launch(replay_buffer, "a")
            self._allreduce()
            self._hip_launch(replay_buffer, "b")
            return
        if self._graphs is None or self._graphs[0] != key:
            torch.cuda.synchronize(self.device)
            graphs = []
            if self.split and self.capture_collective:  # grads | all-reduce | update in one graph
                self._warm_collective()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    sf.set_stream()
                    self._hip_launch(replay_buffer, "a")
                    torch.distributed.all_reduce(self.flat_grad, group=self.pg)
                    self._hip_launch(replay_buffer, "b")
                graphs.append(g)
            else:
                for part in (("a", "b") if self.split else ("ab",)):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        sf.set_stream()
                        self._hip_launch(replay_buffer, part)
                    graphs.append(g)
            sf.set_stream()
            self._graphs = (key, graphs)
        graphs = self._graphs[1]
        graphs[0].replay()
        if len(graphs) > 1:
            self._allreduce()
            graphs[1].replay()

    def _warm_collective(self):
        if not self._collective_warm:  # the communicator's first collective runs eagerly (set-up)
            torch.distributed.all_reduce(torch.zeros(1, device=self.device), group=self.pg)
            torch.cuda.synchronize(self.device)
            self._collective_warm = True

    # grad steps per captured multi-step graph (hip backend, replay sampling on the device): consecutive steps
    # inside one graph are separated by a kernel boundary instead of a graph launch from the host
    GRAPH_STEPS = 8

    def _multi_ok(self, replay_buffer):
        return (self.backend == "hip" and self.use_graph and replay_buffer is not None and self.noise_fn is None
                and (not self.split or self.capture_collective))

    def _multi_graph(self, replay_buffer):
        """The GRAPH_STEPS-step graph for this buffer: each step's kernels read the device step counter (the
        Philox counter of the batch draw, Adam's bias corrections), so the steps are the same as one graph each.
        The steps form a chain (sacf_grads_chain): each but the last stages the next step's batch in its
        weight-gradient pass, and each but the first starts from that staged batch (nothing writes the replay
        ring inside the graph, so it is the batch its own gather would draw). With the update in the same launch,
        each but the last leaves the flat gradient unwritten (nothing reads it in between: p.grad after the run is
        the last step's gradient, as with one graph per step)."""
        self._hip_step_prepare(replay_buffer)
        key = (id(replay_buffer), self.GRAPH_STEPS)
        if getattr(self, "_mgraph", None) is None or self._mgraph[0] != key:
            from .... import sacfused as sfb
            sf = self._sf
            torch.cuda.synchronize(self.device)
            if self.split:
                self._warm_collective()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                sf.set_stream()
                for k in range(self.GRAPH_STEPS):
                    last = k == self.GRAPH_STEPS - 1
                    chain = ((sfb.CHAIN_FROM_STAGED if k > 0 else 0) | (0 if last else sfb.CHAIN_STAGE_NEXT) |
                             (0 if last or self.split else sfb.CHAIN_NO_GRADS))
                    self._hip_launch(replay_buffer, "a" if self.split else "ab", chain)
                    if self.split:
                        torch.distributed.all_reduce(self.flat_grad, group=self.pg)
                        self._hip_launch(replay_buffer, "b")
            sf.set_stream()
            self._mgraph = (key, g)
        return self._mgraph[1]

    # ---------------------------------------------------------------- math
    def _actor(self, x):
        h = x
        for fc in self.policy.fcs:
            h = F.relu(F.linear(h, fc.weight, fc.bias))
        w = torch.cat([self.policy.last_fc.weight, self.policy.last_fc_log_std.weight], 0)
        b = torch.cat([self.policy.last_fc.bias, self.policy.last_fc_log_std.bias], 0)
        out = torch.addmm(b, h, w.t())
        a_dim = self.policy.last_fc.weight.shape[0]
        mean, log_std = out[:, :a_dim], out[:, a_dim:]
        std = torch.exp(torch.clamp(log_std, LOG_SIG_MIN, LOG_SIG_MAX))
        return mean, std

    @staticmethod
    def _twin(nets, x):
        """x: (R, in) shared by both nets → (2, R, out) via one baddbmm per layer."""
        layers = [_layers(n) for n in nets]
        h = x.unsqueeze(0).expand(len(nets), -1, -1)
        n_l = len(layers[0])
        for i in range(n_l):
            w = torch.stack([ls[i].weight for ls in layers])          # (2, out, in)
            b = torch.stack([ls[i].bias for ls in layers]).unsqueeze(1)  # (2, 1, out)
            h = torch.baddbmm(b, h, w.transpose(1, 2))
            if i < n_l - 1:
                h = F.relu(h)
        return h

    def _eps(self, shape):
        if self.noise_fn is not None:
            return self.noise_fn(shape)
        return torch.randn(shape, device=self.device)

    def _forward_and_grads(self, b):
        """Losses and gradients for one batch; grads land in self.flat_grad."""
        obs, act, rew, term, nobs = (b[k] for k in _BATCH_KEYS)
        B = obs.shape[0]
        mean, std = self._actor(torch.cat([obs, nobs], 0))
        z = mean + std * self._eps(mean.shape)
        a = torch.tanh(z)
        logp = diag_normal_log_prob(z, mean, std) + (-2.0 * (_LOG2 - z - F.softplus(-2.0 * z)).sum(dim=1))
        new_a, log_pi = a[:B], logp[:B].unsqueeze(-1)
        nn_a, nlog_pi = a[B:], logp[B:].unsqueeze(-1)
        if self.use_automatic_entropy_tuning:
            alpha_loss = -(self.log_alpha * (log_pi + self.target_entropy).detach()).mean()
            alpha = self.log_alpha.exp().detach()
        else:
            alpha_loss = torch.zeros((), device=self.device)
            alpha = torch.ones(1, device=self.device)
        q = self._twin((self.qf1, self.qf2), torch.cat([torch.cat([obs, new_a], 1), torch.cat([obs, act], 1)], 0))
        q_new = torch.min(q[0, :B], q[1, :B])
        policy_loss = (alpha * log_pi - q_new).mean()
        if self.action_reg_coeff:
            policy_loss = policy_loss + self.action_reg_coeff * (new_a ** 2).mean()
        q1_pred, q2_pred = q[0, B:], q[1, B:]
        with torch.no_grad():
            tq = self._twin((self.target_qf1, self.target_qf2), torch.cat([nobs, nn_a], 1))
            target_q = torch.min(tq[0], tq[1]) - alpha * nlog_pi
            q_target = self.reward_scale * rew + (1.0 - term) * self.discount * target_q
            q_target = torch.clamp(q_target, min=-self.clip_val, max=self.clip_val)
        qf1_loss = ((q1_pred - q_target) ** 2).mean()
        qf2_loss = ((q2_pred - q_target) ** 2).mean()
        g_pi = torch.autograd.grad(policy_loss + alpha_loss, self.pi_params, retain_graph=True)
        g_q = torch.autograd.grad(qf1_loss + qf2_loss, self.q_params)
        torch._foreach_copy_(self._grad_views, list(g_pi) + list(g_q))
        return dict(policy_loss=policy_loss.detach(), qf1_loss=qf1_loss.detach(), qf2_loss=qf2_loss.detach(),
                    alpha_loss=alpha_loss.detach(), q1_pred=q1_pred.detach(), q2_pred=q2_pred.detach(),
                    q_target=q_target, log_pi=log_pi.detach(), alpha=alpha.detach(),
                    pi_mean=torch.tanh(mean[:B]).detach(), pi_std=std[:B].detach())

    def _apply(self):
        if self.split:
            self.flat_grad.mul_(1.0 / self.world)
        self.optimizer.step()
        with torch.no_grad():
            tau = self.soft_target_tau
            torch._foreach_mul_(self.t_params, 1.0 - tau)
            torch._foreach_add_(self.t_params, self.q_params, alpha=tau)

    def _allreduce(self):
        if self.split and self.pg is not None:
            torch.distributed.all_reduce(self.flat_grad, group=self.pg)

    # ---------------------------------------------------------------- graph
    def _alloc_static(self, obs_dim, act_dim):
        B, dev = self.batch_size, self.device
        self._static = dict(observations=torch.zeros(B, obs_dim, device=dev), actions=torch.zeros(B, act_dim, device=dev),
                            rewards=torch.zeros(B, 1, device=dev), terminals=torch.zeros(B, 1, device=dev),
                            next_observations=torch.zeros(B, obs_dim, device=dev))

    def _snapshot_state(self):
        params = {id(p): p.detach().clone() for p in self.pi_params + self.q_params + self.t_params}
        st = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in s.items()}
              for p, s in self.optimizer.state.items()}
        return params, st

    def _restore_state(self, snap):
        params, st = snap
        with torch.no_grad():
            for p in self.pi_params + self.q_params + self.t_params:
                p.copy_(params[id(p)])
            for p, s in self.optimizer.state.items():
                old = st.get(id(p))
                for k, v in s.items():
                    if torch.is_tensor(v):
                        v.copy_(old[k]) if old is not None else v.zero_()

    def _body_a(self, replay_buffer):
        if replay_buffer is not None:
            replay_buffer.random_batch(self.batch_size, out=self._static)
        self._out = self._forward_and_grads(self._static)

    def _build_graphs(self, replay_buffer):
        snap = self._snapshot_state()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(3):
                self._body_a(replay_buffer)
                self._allreduce()
                self._apply()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._restore_state(snap)
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        pool = torch.cuda.graph_pool_handle()
        if self.split:
            with torch.cuda.graph(ga, pool=pool):
                self._body_a(replay_buffer)
            with torch.cuda.graph(gb, pool=pool):
                self._apply()
        else:
            with torch.cuda.graph(ga, pool=pool):
                self._body_a(replay_buffer)
                self._apply()
            gb = None
        torch.cuda.synchronize(self.device)
        return ga, gb

    def _run_step(self, replay_buffer):
        if self.backend == "hip":
            if replay_buffer is None and self._static is None:
                raise RuntimeError("no batch")
            return self._hip_step(replay_buffer)
        key = id(replay_buffer) if replay_buffer is not None else None
        if self._static is None:
            obs_dim = self.policy.input_size
            act_dim = self.policy.last_fc.weight.shape[0]
            self._alloc_static(obs_dim, act_dim)
        if not self.use_graph:
            self._body_a(replay_buffer)
            self._allreduce()
            self._apply()
            return
        if self._graphs is None or self._graphs[0] != key:
            self._graphs = (key,) + self._build_graphs(replay_buffer)
        _, ga, gb = self._graphs
        ga.replay()
        if gb is not None:
            self._allreduce()
            gb.replay()

    # ---------------------------------------------------------------- API
    def train_from_torch(self, batch):
        """One update on an explicit batch (copied into the static batch buffers)."""
        if self._static is None:
            self._alloc_static(batch["observations"].shape[1], batch["actions"].shape[1])
        if batch["observations"].shape[0] != self.batch_size:
            raise ValueError(f"batch has {batch['observations'].shape[0]} rows, trainer batch_size={self.batch_size}")
        for k in _BATCH_KEYS:
            self._static[k].copy_(batch[k].reshape(self._static[k].shape))
        self._run_step(None)
        self._after_step()

    def train_from_buffer(self, replay_buffer, n_steps=1):
        """n_steps updates, each on a fresh uniform batch drawn on-device from a DeviceReplayBuffer (hip backend:
        runs of GRAPH_STEPS steps replay one multi-step graph; the steps and their results are the same)."""
        done = 0
        G = self.GRAPH_STEPS
        if self._multi_ok(replay_buffer) and n_steps >= G:
            if self._need_to_update_eval_statistics:  # the epoch's statistics are its first step's (sac.py:102-154)
                self._num_train_steps += 1
                self._run_step(replay_buffer)
                self._after_step()
                done = 1
            while n_steps - done >= G:
                self._multi_graph(replay_buffer).replay()
                self._num_train_steps += G
                self._n_train_steps_total += G
                done += G
        for _ in range(n_steps - done):
            self._num_train_steps += 1
            self._run_step(replay_buffer)
            self._after_step()

    def _after_step(self):
        self._n_train_steps_total += 1
        if self._need_to_update_eval_statistics:
            self.eval_statistics = self._stats()
            self._need_to_update_eval_statistics = False

    def last_losses(self):
        if self.backend == "hip":
            st = self._stats_t
            return SACLosses(policy_loss=st[0], qf1_loss=st[1], qf2_loss=st[2], alpha_loss=st[3])
        o = self._out
        return SACLosses(policy_loss=o["policy_loss"], qf1_loss=o["qf1_loss"], qf2_loss=o["qf2_loss"],
                         alpha_loss=o["alpha_loss"])

    def _stats(self):
        if self.backend == "hip":
            st = ptu.get_numpy(self._stats_t)
            B = self.batch_size
            rows = st[8:].reshape(6, B)
            o = dict(qf1_loss=st[1], qf2_loss=st[2], policy_loss=st[0], alpha_loss=st[3], alpha=st[4:5],
                     q1_pred=rows[0][:, None], q2_pred=rows[1][:, None], q_target=rows[2][:, None],
                     log_pi=rows[3][:, None], pi_mean=rows[4][:, None], pi_std=rows[5][:, None])
        else:
            o = {k: ptu.get_numpy(v) for k, v in self._out.items()}
        st = OrderedDict()
        st["QF1 Loss"] = float(np.mean(o["qf1_loss"]))
        st["QF2 Loss"] = float(np.mean(o["qf2_loss"]))
        st["Policy Loss"] = float(np.mean(o["policy_loss"]))
        st.update(create_stats_ordered_dict("Q1 Predictions", o["q1_pred"]))
        st.update(create_stats_ordered_dict("Q2 Predictions", o["q2_pred"]))
        st.update(create_stats_ordered_dict("Q Targets", o["q_target"]))
        st.update(create_stats_ordered_dict("Log Pis", o["log_pi"]))
        st.update(create_stats_ordered_dict("policy/mean", o["pi_mean"]))
        st.update(create_stats_ordered_dict("policy/normal/std", o["pi_std"]))
        st.update(create_stats_ordered_dict("policy/normal/log_std", np.log(o["pi_std"])))
        if self.use_automatic_entropy_tuning:
            st["Alpha"] = float(o["alpha"].reshape(-1)[0])
            st["Alpha Loss"] = float(o["alpha_loss"])
        return st

    def broadcast_parameters(self, src=0):
        """Make every rank start from rank `src`'s networks; replicated: also its batch-
        sampling / noise seed, so every rank draws the same batches."""
        if self.pg is None or torch.distributed.get_world_size(self.pg) == 1:
            return
        with torch.no_grad():
            if self.backend == "hip":
                torch.distributed.broadcast(self.flat_param, src, group=self.pg)
                torch.distributed.broadcast(self.flat_target, src, group=self.pg)
                self._sf.sync_params()
                if self.replicated:
                    dev = self.device if torch.distributed.get_backend(self.pg) == "nccl" else "cpu"
                    t = torch.tensor([self._seed], dtype=torch.int64, device=dev)
                    torch.distributed.broadcast(t, src, group=self.pg)
                    self._seed = int(t.item())
                    self._replay_key = None  # (re-bind the replay ring with the common seed)
                return
            for p in self.pi_params + self.q_params + self.t_params:
                torch.distributed.broadcast(p.data, src, group=self.pg)

    def device_policy(self, deterministic=False, seed=None):
        """The collector's policy on the matrix cores (hip backend): DevicePolicy.act(obs, mask, out) writes
        TanhGaussianPolicy samples (or MakeDeterministic's tanh(mean)) of the trainer's CURRENT parameters
        for every row whose mask is set, with no host sync (graph-capturable). Same math as
        `policy(obs)` + sample(), fp32 with the kernels' accumulation order."""
        if self.backend != "hip":
            raise ValueError("device_policy needs the hip backend")
        s = int(torch.randint(0, 2 ** 62, (1,)).item()) if seed is None else int(seed)
        return DevicePolicy(self._sf, deterministic, s, self.device)

    def get_diagnostics(self):
        stats = super().get_diagnostics()
        stats.update(self.eval_statistics)
        return stats

    def end_epoch(self, epoch):
        self._need_to_update_eval_statistics = True

    @property
    def networks(self):
        return [self.policy, self.qf1, self.qf2, self.target_qf1, self.target_qf2]

    @property
    def optimizers(self):
        return [self.optimizer] if self.optimizer is not None else []

    def get_snapshot(self):
        return dict(policy=self.policy, qf1=self.qf1, qf2=self.qf2, target_qf1=self.target_qf1,
                    target_qf2=self.target_qf2)


class DevicePolicy:
    """Policy actions through libsacfused's sacf_policy_act (see FusedSACTrainer.device_policy)."""

    def __init__(self, sf, deterministic, seed, device):
        self._sf, self.deterministic, self.seed = sf, bool(deterministic), seed
        self.counter = torch.zeros(1, dtype=torch.int64, device=device)  # Philox counter, advanced per call
        self._n = 0

    def reserve(self, n):
        if n > self._n:
            self._sf.policy_reserve(n)
            self._n = n

    def act(self, obs, mask, out, eps_out=None):
        """out[i] = action of obs[i] where mask[i] (uint8 / bool tensor or None), on the current stream."""
        if obs.shape[0] > self._n:
            raise RuntimeError("DevicePolicy.reserve(n) first (outside any graph capture)")
        m = None if mask is None else (mask if mask.dtype == torch.uint8 else mask.view(torch.uint8))
        self._sf.set_stream()
        self._sf.policy_act(obs, out, mask=m, deterministic=self.deterministic, seed=self.seed,
                            counter=self.counter, eps_out=eps_out)
        if not self.deterministic:
            self.counter.add_(1)

    def weights(self):
        """(params_ptr, w2t_ptr, obs_dim, hidden) of the trainer's live policy: what ShipSim.run_policy
        (the decision stream with this policy in the loop) reads; stable for the trainer's lifetime."""
        return self._sf.policy_weights()
