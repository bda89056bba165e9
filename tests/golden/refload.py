"""Load the REFERENCE hand_arm task code in this (GPU-less, Isaac-Gym-less) container.

Used ONLY by ``tests/golden/make_goldens.py`` to generate committed golden vectors; nothing under
``tests/`` imports this at test time and the reference never leaves this container.

Mechanism: a meta-path finder that
  * loads ``isaacgymenvs.*`` modules straight from ``/root/reference/isaacgymenvs/**.py`` without
    executing package ``__init__`` files (they import every task in the fork);
  * maps ``isaacgym.torch_utils`` onto the reference's own ``utils/torch_jit_utils.py`` (SURVEY.md §8c:
    the hand_arm files import the same-named functions from the binary package);
  * replaces absent third-party packages (Isaac Gym binary, ROS, hydra/omegaconf, cv2, trimesh,
    urdfpy, openai gym) by inert mock modules - none of them is on the task-math path;
  * provides ``torchcubicspline`` as a restatement of its published natural-cubic-spline algorithm
    (package absent; version unpinned - see ``oracle/task_oracle.py`` ``NaturalCubicSpline``).
"""
import importlib.abc
import importlib.machinery
import importlib.util
import os
import sys
import types
from unittest import mock

import torch

REF_ROOT = "/root/reference"
MOCKED = ("isaacgym", "rospy", "sensor_msgs", "std_msgs", "trajectory_msgs", "actionlib", "control_msgs",
          "tf", "hydra", "omegaconf", "cv2", "trimesh", "urdfpy", "gym", "wandb", "rl_games")


def _tridiagonal_solve(b, A_upper, A_diagonal, A_lower):
    """Thomas algorithm, as in torchcubicspline.misc.tridiagonal_solve."""
    A_upper, _ = torch.broadcast_tensors(A_upper, b[..., :-1])
    A_lower, _ = torch.broadcast_tensors(A_lower, b[..., :-1])
    A_diagonal, b = torch.broadcast_tensors(A_diagonal, b)
    channels = b.size(-1)
    new_b = torch.empty(channels, *b.shape[:-1], dtype=b.dtype, device=b.device)
    new_A_diagonal = torch.empty(channels, *b.shape[:-1], dtype=b.dtype, device=b.device)
    outs = torch.empty(channels, *b.shape[:-1], dtype=b.dtype, device=b.device)
    new_b[0] = b[..., 0]
    new_A_diagonal[0] = A_diagonal[..., 0]
    for i in range(1, channels):
        w = A_lower[..., i - 1] / new_A_diagonal[i - 1]
        new_A_diagonal[i] = A_diagonal[..., i] - w * A_upper[..., i - 1]
        new_b[i] = b[..., i] - w * new_b[i - 1]
    outs[channels - 1] = new_b[channels - 1] / new_A_diagonal[channels - 1]
    for i in range(channels - 2, -1, -1):
        outs[i] = (new_b[i] - A_upper[..., i] * outs[i + 1]) / new_A_diagonal[i]
    return outs.permute(*range(1, outs.ndimension()), 0)


def _make_torchcubicspline():
    m = types.ModuleType("torchcubicspline")

    def natural_cubic_spline_coeffs(t, x):
        path = x.transpose(-1, -2)  # (..., channels, length)
        length = path.size(-1)
        if length == 2:
            a = path[..., :1]
            b = (path[..., 1:] - path[..., :1]) / (t[..., 1:] - t[..., :1])
            two_c = torch.zeros_like(b)
            three_d = torch.zeros_like(b)
        else:
            time_diffs = t[1:] - t[:-1]
            time_diffs_reciprocal = time_diffs.reciprocal()
            time_diffs_reciprocal_squared = time_diffs_reciprocal ** 2
            three_path_diffs = 3 * (path[..., 1:] - path[..., :-1])
            six_path_diffs = 2 * three_path_diffs
            path_diffs_scaled = three_path_diffs * time_diffs_reciprocal_squared
            system_diagonal = torch.empty(length, dtype=path.dtype, device=path.device)
            system_diagonal[:-1] = time_diffs_reciprocal
            system_diagonal[-1] = 0
            system_diagonal[1:] += time_diffs_reciprocal
            system_diagonal *= 2
            system_rhs = torch.empty_like(path)
            system_rhs[..., :-1] = path_diffs_scaled
            system_rhs[..., -1] = 0
            system_rhs[..., 1:] += path_diffs_scaled
            knot_derivatives = _tridiagonal_solve(system_rhs, time_diffs_reciprocal, system_diagonal,
                                                  time_diffs_reciprocal)
            a = path[..., :-1]
            b = knot_derivatives[..., :-1]
            two_c = (six_path_diffs * time_diffs_reciprocal - 4 * knot_derivatives[..., :-1]
                     - 2 * knot_derivatives[..., 1:]) * time_diffs_reciprocal
            three_d = (-six_path_diffs * time_diffs_reciprocal
                       + 3 * (knot_derivatives[..., :-1] + knot_derivatives[..., 1:])) * time_diffs_reciprocal_squared
        return (t, a.transpose(-1, -2), b.transpose(-1, -2), two_c.transpose(-1, -2), three_d.transpose(-1, -2))

    class NaturalCubicSpline:
        def __init__(self, coeffs):
            t, a, b, two_c, three_d = coeffs
            self._t, self._a, self._b, self._two_c, self._three_d = t, a, b, two_c, three_d

        def _interpret_t(self, t):
            maxlen = self._b.size(-2) - 1
            index = torch.bucketize(t.detach(), self._t) - 1
            index = index.clamp(0, maxlen)
            fractional_part = t - self._t[index]
            return fractional_part, index

        def evaluate(self, t):
            fractional_part, index = self._interpret_t(t)
            fractional_part = fractional_part.unsqueeze(-1)
            inner = 0.5 * self._two_c[..., index, :] + self._three_d[..., index, :] * fractional_part / 3
            inner = self._b[..., index, :] + inner * fractional_part
            return self._a[..., index, :] + inner * fractional_part

    m.natural_cubic_spline_coeffs = natural_cubic_spline_coeffs
    m.NaturalCubicSpline = NaturalCubicSpline
    return m


class _RefFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, name, path=None, target=None):
        top = name.split(".")[0]
        if name == "torchcubicspline":
            return importlib.machinery.ModuleSpec(name, self, is_package=False)
        if name == "isaacgym.torch_utils":
            fn = os.path.join(REF_ROOT, "isaacgymenvs", "utils", "torch_jit_utils.py")
            return importlib.util.spec_from_file_location(name, fn)
        if top in MOCKED:
            return importlib.machinery.ModuleSpec(name, self, is_package=True)
        if top == "isaacgymenvs":
            rel = name.split(".")
            d = os.path.join(REF_ROOT, *rel)
            if os.path.isdir(d):
                return importlib.machinery.ModuleSpec(name, self, is_package=True)
            fn = d + ".py"
            if os.path.exists(fn):
                return importlib.util.spec_from_file_location(name, fn)
        return None

    def create_module(self, spec):
        if spec.name == "torchcubicspline":
            return _make_torchcubicspline()
        if spec.name.split(".")[0] == "isaacgymenvs":
            m = types.ModuleType(spec.name)
            m.__path__ = [os.path.join(REF_ROOT, *spec.name.split("."))]
            return m
        m = mock.MagicMock(name=spec.name)
        m.__path__ = []
        m.__spec__ = spec
        m.__all__ = []
        if spec.name == "isaacgym.gymtorch":
            m.wrap_tensor = lambda t: t
            m.unwrap_tensor = lambda t: t
        return m

    def exec_module(self, module):
        pass


def install():
    if not any(isinstance(f, _RefFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _RefFinder())


def load(name):
    install()
    return importlib.import_module(name)
