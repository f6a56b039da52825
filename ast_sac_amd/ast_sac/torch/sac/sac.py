"""SACTrainer with the reference's update semantics (ast_sac/torch/sac/sac.py:21-335).

One `train_from_torch(batch)`:
  π, log π ← policy(obs)  (rsample);  α = exp(log α)
  α-loss  = −mean(log α · (log π + H̄).detach())
  π-loss  = mean(α log π − min(Q1, Q2)(obs, ã)) + c_reg · mean(ã²)
  target  = clamp(r_s·r + (1 − d)·γ·(min(Q̄1, Q̄2)(s', ã') − α log π'), ±clip)
  Q-loss  = MSE(Qi(obs, a), target.detach())
then Adam steps in the order α → π → Q1 → Q2 and a soft target update every
`target_update_period` steps. Every loss is built from the pre-step parameters, so the four
optimizer steps are independent; `FusedSACTrainer` (sac_fused.py) exploits that.
"""
from collections import OrderedDict, namedtuple

import numpy as np
import torch
import torch.optim as optim
from torch import nn

from ..utils import pytorch_util as ptu
from ..core.torch_rl_algorithm import TorchTrainer
from ...core.eval_util import create_stats_ordered_dict

SACLosses = namedtuple("SACLosses", "policy_loss qf1_loss qf2_loss alpha_loss")


def add_prefix(d, prefix):
    return OrderedDict((prefix + k, v) for k, v in d.items())


class SACTrainer(TorchTrainer):
    def __init__(self, env, policy, qf1, qf2, target_qf1, target_qf2, discount=0.99, reward_scale=1.0,
                 policy_lr=1e-3, qf_lr=1e-3, optimizer_class=optim.Adam, soft_target_tau=1e-2,
                 target_update_period=1, plotter=None, render_eval_paths=False,
                 use_automatic_entropy_tuning=True, target_entropy=None, action_reg_coeff=None, clip_val=np.inf):
        super().__init__()
        self.env = env
        self.policy = policy
        self.qf1 = qf1
        self.qf2 = qf2
        self.target_qf1 = target_qf1
        self.target_qf2 = target_qf2
        self.soft_target_tau = soft_target_tau
        self.target_update_period = target_update_period
        self.use_automatic_entropy_tuning = use_automatic_entropy_tuning
        dev = next(policy.parameters()).device
        if use_automatic_entropy_tuning:
            self.target_entropy = (-np.prod(env.action_space.shape).item() if target_entropy is None
                                   else target_entropy)
            self.log_alpha = torch.zeros(1, requires_grad=True, device=dev)
            self.alpha_optimizer = optimizer_class([self.log_alpha], lr=policy_lr)
        self.plotter = plotter
        self.render_eval_paths = render_eval_paths
        self.qf_criterion = nn.MSELoss()
        self.vf_criterion = nn.MSELoss()
        self.policy_optimizer = optimizer_class(self.policy.parameters(), lr=policy_lr)
        self.qf1_optimizer = optimizer_class(self.qf1.parameters(), lr=qf_lr)
        self.qf2_optimizer = optimizer_class(self.qf2.parameters(), lr=qf_lr)
        self.discount = discount
        self.reward_scale = reward_scale
        self._n_train_steps_total = 0
        self._need_to_update_eval_statistics = True
        self.eval_statistics = OrderedDict()
        self.action_reg_coeff = action_reg_coeff
        self.clip_val = clip_val

    def train_from_torch(self, batch):
        losses, stats = self.compute_loss(batch, skip_statistics=not self._need_to_update_eval_statistics)
        if self.use_automatic_entropy_tuning:
            self.alpha_optimizer.zero_grad()
            losses.alpha_loss.backward()
            self.alpha_optimizer.step()
        self.policy_optimizer.zero_grad()
        losses.policy_loss.backward()
        self.policy_optimizer.step()
        self.qf1_optimizer.zero_grad()
        losses.qf1_loss.backward()
        self.qf1_optimizer.step()
        self.qf2_optimizer.zero_grad()
        losses.qf2_loss.backward()
        self.qf2_optimizer.step()
        self._n_train_steps_total += 1
        self.try_update_target_networks()
        if self._need_to_update_eval_statistics:
            self.eval_statistics = stats
            self._need_to_update_eval_statistics = False

    def try_update_target_networks(self):
        if self._n_train_steps_total % self.target_update_period == 0:
            self.update_target_networks()

    def update_target_networks(self):
        ptu.soft_update_from_to(self.qf1, self.target_qf1, self.soft_target_tau)
        ptu.soft_update_from_to(self.qf2, self.target_qf2, self.soft_target_tau)

    def compute_loss(self, batch, skip_statistics=False, debug=False):
        rewards = batch["rewards"]
        terminals = batch["terminals"]
        obs = batch["observations"]
        actions = batch["actions"]
        next_obs = batch["next_observations"]

        dist = self.policy(obs)
        new_obs_actions, log_pi = dist.rsample_and_logprob()
        log_pi = log_pi.unsqueeze(-1)
        if self.use_automatic_entropy_tuning:
            alpha_loss = -(self.log_alpha * (log_pi + self.target_entropy).detach()).mean()
            alpha = self.log_alpha.exp()
        else:
            alpha_loss = 0
            alpha = 1
        q_new_actions = torch.min(self.qf1(obs, new_obs_actions), self.qf2(obs, new_obs_actions))
        policy_loss = (alpha * log_pi - q_new_actions).mean()
        if self.action_reg_coeff:
            policy_loss = policy_loss + self.action_reg_coeff * (new_obs_actions ** 2).mean()

        q1_pred = self.qf1(obs, actions)
        q2_pred = self.qf2(obs, actions)
        next_dist = self.policy(next_obs)
        new_next_actions, new_log_pi = next_dist.rsample_and_logprob()
        new_log_pi = new_log_pi.unsqueeze(-1)
        target_q_values = torch.min(self.target_qf1(next_obs, new_next_actions),
                                    self.target_qf2(next_obs, new_next_actions)) - alpha * new_log_pi
        q_target = self.reward_scale * rewards + (1.0 - terminals) * self.discount * target_q_values
        q_target = torch.clamp(q_target, min=-self.clip_val, max=self.clip_val)
        qf1_loss = self.qf_criterion(q1_pred, q_target.detach())
        qf2_loss = self.qf_criterion(q2_pred, q_target.detach())

        stats = OrderedDict()
        if not skip_statistics:
            stats["QF1 Loss"] = np.mean(ptu.get_numpy(qf1_loss))
            stats["QF2 Loss"] = np.mean(ptu.get_numpy(qf2_loss))
            stats["Policy Loss"] = np.mean(ptu.get_numpy(policy_loss))
            stats.update(create_stats_ordered_dict("Q1 Predictions", ptu.get_numpy(q1_pred)))
            stats.update(create_stats_ordered_dict("Q2 Predictions", ptu.get_numpy(q2_pred)))
            stats.update(create_stats_ordered_dict("Q Targets", ptu.get_numpy(q_target)))
            stats.update(create_stats_ordered_dict("Log Pis", ptu.get_numpy(log_pi)))
            stats.update(add_prefix(dist.get_diagnostics(), "policy/"))
            if self.use_automatic_entropy_tuning:
                stats["Alpha"] = alpha.item()
                stats["Alpha Loss"] = alpha_loss.item()
        return SACLosses(policy_loss=policy_loss, qf1_loss=qf1_loss, qf2_loss=qf2_loss, alpha_loss=alpha_loss), stats

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
        return [self.alpha_optimizer, self.qf1_optimizer, self.qf2_optimizer, self.policy_optimizer]

    def get_snapshot(self):
        return dict(policy=self.policy, qf1=self.qf1, qf2=self.qf2, target_qf1=self.target_qf1,
                    target_qf2=self.target_qf2)
