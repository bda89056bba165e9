"""Quaternion helpers (xyzw) used by host-side torch code (drop initialisation).

Same conventions and formulas as the reference's isaacgymenvs/utils/torch_jit_utils.py:41-123,215-218
and multi_object_manipulation.py:12-15 (randomize_rotation); written for device tensors.
"""
import math

import torch


def quat_mul(a, b):
    x1, y1, z1, w1 = a.unbind(-1)
    x2, y2, z2, w2 = b.unbind(-1)
    ww = (z1 + x1) * (x2 + y2)
    yy = (w1 - y1) * (w2 + z2)
    zz = (w1 + y1) * (w2 - z2)
    xx = ww + yy + zz
    qq = 0.5 * (xx + (z1 - x1) * (x2 - y2))
    w = qq - ww + (z1 - y1) * (y2 - z2)
    x = qq - xx + (x1 + w1) * (x2 + w2)
    y = qq - yy + (w1 - x1) * (y2 + z2)
    z = qq - zz + (z1 + y1) * (w2 - x2)
    return torch.stack([x, y, z, w], -1)


def normalize(x, eps=1e-9):
    return x / x.norm(p=2, dim=-1).clamp(min=eps).unsqueeze(-1)


def quat_from_angle_axis(angle, axis):
    theta = (angle / 2).unsqueeze(-1)
    xyz = normalize(axis) * theta.sin()
    return normalize(torch.cat([xyz, theta.cos()], -1))


def randomize_rotation(rand0, rand1):
    n = rand0.shape[0]
    xu = torch.tensor([1.0, 0.0, 0.0], device=rand0.device).repeat(n, 1)
    yu = torch.tensor([0.0, 1.0, 0.0], device=rand0.device).repeat(n, 1)
    return quat_mul(quat_from_angle_axis(rand0 * math.pi, xu), quat_from_angle_axis(rand1 * math.pi, yu))


def torch_rand_float(lower, upper, shape, device, generator=None):
    return (upper - lower) * torch.rand(*shape, device=device, generator=generator) + lower
