"""Device plumbing and small tensor helpers (ast_sac/torch/utils/pytorch_util.py).

Same module-level state as the reference (`device`, `set_gpu_mode`, `from_numpy`, ...); on
ROCm `cuda:N` is the HIP device N.
"""
import numpy as np
import torch

_use_gpu = False
_gpu_id = 0
device = torch.device("cpu")


def set_gpu_mode(mode, gpu_id=0):
    """pytorch_util.py:216-222"""
    global _use_gpu, device, _gpu_id
    _gpu_id = gpu_id
    _use_gpu = bool(mode)
    device = torch.device(f"cuda:{gpu_id}" if _use_gpu else "cpu")


def gpu_enabled():
    return _use_gpu


def set_device(gpu_id):
    torch.cuda.set_device(gpu_id)


def soft_update_from_to(source, target, tau):
    """θ' ← θ'·(1−τ) + θ·τ, same evaluation order as pytorch_util.py:21-25."""
    for tp, p in zip(target.parameters(), source.parameters()):
        tp.data.copy_(tp.data * (1.0 - tau) + p.data * tau)


def copy_model_params_from_to(source, target):
    for tp, p in zip(target.parameters(), source.parameters()):
        tp.data.copy_(p.data)


def fanin_init(tensor):
    """U(±1/sqrt(size[0])) — for nn.Linear weights size[0] is out_features (pytorch_util.py:132-141)."""
    size = tensor.size()
    if len(size) == 2:
        fan_in = size[0]
    elif len(size) > 2:
        fan_in = np.prod(size[1:])
    else:
        raise Exception("Shape must be have dimension at least 2.")
    bound = 1.0 / np.sqrt(fan_in)
    return tensor.data.uniform_(-bound, bound)


def identity(x):
    return x


def from_numpy(*args, **kwargs):
    return torch.from_numpy(*args, **kwargs).float().to(device)


def get_numpy(tensor):
    return tensor.to("cpu").detach().numpy()


def _dev(torch_device):
    return device if torch_device is None else torch_device


def zeros(*sizes, torch_device=None, **kwargs):
    return torch.zeros(*sizes, **kwargs, device=_dev(torch_device))


def ones(*sizes, torch_device=None, **kwargs):
    return torch.ones(*sizes, **kwargs, device=_dev(torch_device))


def zeros_like(*args, torch_device=None, **kwargs):
    return torch.zeros_like(*args, **kwargs, device=_dev(torch_device))


def ones_like(*args, torch_device=None, **kwargs):
    return torch.ones_like(*args, **kwargs, device=_dev(torch_device))


def randn(*args, torch_device=None, **kwargs):
    return torch.randn(*args, **kwargs, device=_dev(torch_device))


def randint(*sizes, torch_device=None, **kwargs):
    return torch.randint(*sizes, **kwargs, device=_dev(torch_device))


def tensor(*args, torch_device=None, **kwargs):
    return torch.tensor(*args, **kwargs, device=_dev(torch_device))


def normal(*args, **kwargs):
    return torch.normal(*args, **kwargs).to(device)
