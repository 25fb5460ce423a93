"""legged_gym/utils/math.py equivalents (reference math.py:8-25)."""
import numpy as np
import torch
from isaacgym.torch_utils import normalize, quat_apply

__all__ = ["quat_apply_yaw", "wrap_to_pi", "torch_rand_sqrt_float"]


def quat_apply_yaw(quat, vec):
    q = quat.clone().view(-1, 4)
    q[:, :2] = 0.0
    return quat_apply(normalize(q), vec)


def wrap_to_pi(angles):
    """In place, like the reference: angles mod 2pi, then shifted into (-pi, pi]."""
    angles %= 2 * np.pi
    angles -= 2 * np.pi * (angles > np.pi)
    return angles


def torch_rand_sqrt_float(lower, upper, shape, device):
    r = 2 * torch.rand(*shape, device=device) - 1
    r = torch.where(r < 0.0, -torch.sqrt(-r), torch.sqrt(r))
    return (upper - lower) * (r + 1.0) / 2.0 + lower
