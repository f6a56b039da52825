"""ReLU MLPs of the SAC critics and actor (ast_sac/torch/networks/mlp.py:13-70, :125-136).

Parameter names (fc0, fc1, ..., last_fc) and init rules match the reference so state dicts
and snapshots interchange: hidden weights fanin_init (U(±1/sqrt(out_features)), rlkit quirk),
hidden biases b_init_value, last layer weight U(±init_w), bias 0.
"""
import torch
from torch import nn
from torch.nn import functional as F

from ..utils import pytorch_util as ptu


class Mlp(nn.Module):
    def __init__(self, hidden_sizes, output_size, input_size, init_w=3e-3, hidden_activation=F.relu,
                 output_activation=ptu.identity, hidden_init=ptu.fanin_init, b_init_value=0.0,
                 layer_norm=False, layer_norm_kwargs=None):
        super().__init__()
        if layer_norm:
            raise NotImplementedError("layer_norm is not used by the AST-SAC runner")
        self.input_size = input_size
        self.output_size = output_size
        self.hidden_sizes = list(hidden_sizes)
        self.hidden_activation = hidden_activation
        self.output_activation = output_activation
        self.layer_norm = False
        self.fcs = []
        in_size = input_size
        for i, next_size in enumerate(hidden_sizes):
            fc = nn.Linear(in_size, next_size)
            in_size = next_size
            hidden_init(fc.weight)
            fc.bias.data.fill_(b_init_value)
            self.__setattr__(f"fc{i}", fc)
            self.fcs.append(fc)
        self.last_fc = nn.Linear(in_size, output_size)
        self.last_fc.weight.data.uniform_(-init_w, init_w)
        self.last_fc.bias.data.fill_(0)

    def forward(self, input, return_preactivations=False):
        h = input
        for fc in self.fcs:
            h = self.hidden_activation(fc(h))
        pre = self.last_fc(h)
        out = self.output_activation(pre)
        return (out, pre) if return_preactivations else out


class ConcatMlp(Mlp):
    """Concatenate inputs along `dim`, then the MLP (mlp.py:125-136)."""

    def __init__(self, *args, dim=1, **kwargs):
        super().__init__(*args, **kwargs)
        self.dim = dim

    def forward(self, *inputs, **kwargs):
        return super().forward(torch.cat(inputs, dim=self.dim), **kwargs)
