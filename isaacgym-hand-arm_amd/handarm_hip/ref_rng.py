"""Seed-faithful random draws: the reference's RNG stream, in the reference's order (cfg "reference_rng").

The reference draws its reset randomness from torch's GLOBAL generator of the sim device. On the path the
north_star names (sim_device=cpu, seeded by utils/utils.py:94 set_seed: random.seed, np.random.seed,
torch.manual_seed) that is the CPU generator. By default the fused kernels draw from a counter hash instead
(ha_task.h uniform01), which is fast and needs no host sync but matches nothing in the reference. With
``reference_rng`` on, the VecTask classes draw every reset value here, on the host, from that same global CPU
generator with the reference's calls (same functions, shapes and order), upload the values into
``ha_state_t.reset_draws`` and launch with HA_FLAG_REPLAY_DRAWS. A user who seeds like the reference then gets
the reference's reset indexing (target object, object configuration, goal, cube/hand resets).

The price is one device->host read of the reset flags per step (the reference reads them too, with
``nonzero()``) and one small upload.

Each function cites the reference lines whose draws it reproduces; the kernel-side slot layouts are documented
in csrc/ha_task.h (Ur5Sih), csrc/ak_task.h (AllegroKuka) and csrc/ah_task.h (AllegroHand).
"""
import math
import random

import numpy as np
import torch

from . import model as HM


def set_seed(seed, torch_deterministic=False):
    """utils/utils.py:88-110 set_seed: the seeding the reference's train.py does before building the task."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    return seed


def torch_rand_float(lower, upper, shape):
    """torch_jit_utils.py:216-218 on the CPU global generator."""
    return (upper - lower) * torch.rand(*shape, device="cpu") + lower


# --------------------------------------------------------------------------- HandArm (Ur5Sih)
def ur5sih_reset_draws(n, num_initial_poses, num_objects):
    """reset_idx of all envs (multi_object_manipulation.py:62-91,193-230): _reset_objects'
    torch.randint(num_initial_poses, (n,)), _reset_target_object's torch.randint(num_objects, (n,)), then
    _reset_goal -> _get_random_object_pos(..., 'goal')'s torch.rand((n, 3)).
    Returns (n, 5) float32 in the ha_task.h replay slots: [cfg index, target index, goal rand x3]."""
    cfg = torch.randint(num_initial_poses, (n,), dtype=torch.int64, device="cpu")
    tgt = torch.randint(num_objects, (n,), dtype=torch.int64, device="cpu")
    goal = torch.rand((n, 3), dtype=torch.float32, device="cpu")
    return torch.cat([cfg.float()[:, None], tgt.float()[:, None], goal], 1)


def ur5sih_drop_pose(n, pos, noise):
    """One drop of n objects (multi_object_manipulation.py:107-110): _get_random_object_pos(env_ids, 'drop')
    (:175-184: torch.rand((n, 3)), noise @ diag) then _get_random_quat (:186-191: torch_rand_float(-1, 1, (n, 2)),
    randomize_rotation). Returns CPU (pos (n, 3), quat (n, 4))."""
    from .torch_utils import randomize_rotation
    p = torch.tensor(pos, dtype=torch.float32).unsqueeze(0).repeat(n, 1)
    r = 2 * (torch.rand((n, 3), dtype=torch.float32, device="cpu") - 0.5)
    p = p + r @ torch.diag(torch.tensor(noise, dtype=torch.float32))
    rf = torch_rand_float(-1.0, 1.0, (n, 2))
    return p, randomize_rotation(rf[:, 0], rf[:, 1])


# --------------------------------------------------------------------------- AllegroKuka
def kuka_force_prob(n, prob_range):
    """random_force_prob (allegro_kuka_base.py:323-327 at __init__, :1262-1266 in reset_idx): one torch.rand(n).
    Returns (draw, prob) in float32 with the reference's arithmetic on the CPU."""
    r = torch.tensor(prob_range, dtype=torch.float32)
    u = torch.rand(n, device="cpu")
    return u, torch.exp((torch.log(r[0]) - torch.log(r[1])) * u + torch.log(r[1]))


class KukaDraws:
    """The draws of one AllegroKuka pre_physics_step (allegro_kuka_base.py:1355-1414), slot layout of ak_task.h.

    The per-step force selection ``torch.rand(N) < random_force_prob`` is made here, with the reference's CPU
    arithmetic and the host copy of random_force_prob; the kernel gets the decision as draw 0 (selected) or 1
    (not selected) in slot 71 (2 G + 53), which its ``u < prob`` test reproduces for every prob in (0, 1)."""

    def __init__(self, num_envs, subtask, prob_range, force_scale):
        self.n = num_envs
        self.subtask = subtask
        self.regrasping = subtask == "regrasping"
        self.G = 10 if subtask == "throw" else 9        # draws of one reset_target_pose (ak_task.h ak_goal_draws)
        self.prob_range = prob_range
        self.force_scale = force_scale
        _, self.prob = kuka_force_prob(num_envs, prob_range)          # __init__ draw (:323-327)

    def _target(self, D, ids, base):
        """reset_target_pose -> _reset_target (regrasping.py:76-98 / reorientation.py:104-128 / throw.py:85-103)."""
        k = len(ids)
        if self.subtask == "throw":
            D[ids, base:base + 1] = torch_rand_float(-1.0, 1.0, (k, 1))     # left / right of the table
            D[ids, base + 1:base + 2] = torch_rand_float(0, 0.4, (k, 1))
            D[ids, base + 2:base + 3] = torch_rand_float(-1.0, 0.7, (k, 1))
            D[ids, base + 3:base + 4] = torch_rand_float(0.0, 1.0, (k, 1))
            self._object(D, ids, base + 4)
            return
        D[ids, base:base + 3] = torch_rand_float(0.0, 1.0, (k, 3))
        if self.regrasping:
            self._object(D, ids, base + 3)                              # reset_object_pose (:1196-1220)
        else:
            D[ids, base + 3:base + 6] = torch_rand_float(0, 1.0, (k, 3))    # get_random_quat (:1178-1189)

    @staticmethod
    def _object(D, ids, base):
        k = len(ids)
        D[ids, base:base + 3] = torch_rand_float(-1.0, 1.0, (k, 3))
        D[ids, base + 3:base + 6] = torch_rand_float(0, 1.0, (k, 3))

    def step(self, reset, reset_goal, forces=True):
        """reset / reset_goal: host bool/int (N,) flags; forces=False for a bare reset_idx call (no
        pre_physics_step force draw). Returns (draws (N, HA_DRAW_STRIDE) float32, raw dict)."""
        N = self.n
        D = torch.zeros((N, HM.DRAW_STRIDE), dtype=torch.float32)
        goal_ids = torch.as_tensor(reset_goal).nonzero(as_tuple=False).squeeze(-1)
        env_ids = torch.as_tensor(reset).nonzero(as_tuple=False).squeeze(-1)
        self._target(D, goal_ids, 0)                                    # reset_target_pose(reset_goal_env_ids)
        G = self.G
        if len(env_ids) > 0:                                            # reset_idx(reset_env_ids), :1246-1353
            self._target(D, env_ids, G)
            self._object(D, env_ids, 2 * G)
            u, p = kuka_force_prob(len(env_ids), self.prob_range)
            D[env_ids, 2 * G + 6] = u
            self.prob[env_ids] = p
            D[env_ids, 2 * G + 7:2 * G + 30] = torch_rand_float(0.0, 1.0, (len(env_ids), 23))
            D[env_ids, 2 * G + 30:2 * G + 53] = torch_rand_float(-1.0, 1.0, (len(env_ids), 23))
        raw = {"force_u": None}
        if forces and self.force_scale > 0.0:                           # :1399-1410
            u = torch.rand(N, device="cpu")
            sel = (u < self.prob).nonzero()
            g = torch.randn((len(sel), 1, 3), device="cpu")
            D[:, 2 * G + 53] = 1.0
            D[sel[:, 0], 2 * G + 53] = 0.0
            D[sel[:, 0], 2 * G + 54:2 * G + 57] = g.reshape(len(sel), 3)
            raw["force_u"] = u
        return D, raw


# --------------------------------------------------------------------------- AllegroHand
class AllegroDraws:
    """The draws of one AllegroHand pre_physics_step (allegro_hand.py:586-599), slot layout of ah_task.h."""

    def __init__(self, num_envs, num_dofs=16, force_scale=0.0, force_prob_range=(0.001, 0.1)):
        self.n = num_envs
        self.nd = num_dofs
        self.force_scale = float(force_scale)
        self.lo, self.hi = torch.tensor(force_prob_range, dtype=torch.float32)
        self.prob = self._prob(torch.rand(num_envs, device="cpu"))     # random_force_prob at __init__ (:191-194)

    def _prob(self, u):
        return torch.exp((torch.log(self.lo) - torch.log(self.hi)) * u + torch.log(self.hi))

    def step(self, reset, reset_goal):
        N = self.n
        D = torch.zeros((N, HM.DRAW_STRIDE), dtype=torch.float32)
        env_ids = torch.as_tensor(reset).nonzero(as_tuple=False).squeeze(-1)
        goal_ids = torch.as_tensor(reset_goal).nonzero(as_tuple=False).squeeze(-1)
        if len(goal_ids) > 0:                                           # reset_target_pose (:506-521)
            D[goal_ids, 0:4] = torch_rand_float(-1.0, 1.0, (len(goal_ids), 4))
        if len(env_ids) > 0:                                            # reset_idx (:524-584)
            R = len(env_ids)
            D[env_ids, 4:4 + 2 * self.nd + 5] = torch_rand_float(-1.0, 1.0, (R, 2 * self.nd + 5))
            D[env_ids, 41:45] = torch_rand_float(-1.0, 1.0, (R, 4))   # reset_target_pose(env_ids)
            u = torch.rand(R, device="cpu")                             # random_force_prob (:557-560)
            D[env_ids, 45] = u
            self.prob[env_ids] = self._prob(u)
        if self.force_scale > 0.0:                                      # random forces (:617-623)
            u = torch.rand(N, device="cpu")
            D[:, 46] = u
            idx = (u < self.prob).nonzero(as_tuple=False)              # force_indices, (k, 1)
            g = torch.randn((len(idx), 1, 3), device="cpu")
            D[idx[:, 0], 47:50] = g[:, 0, :]
            D[idx[:, 0], 50] = 1.0                                      # the selection (ah_task.h AH_DRAW_FORCE_SEL)
        return D


_ = math
