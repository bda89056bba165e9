"""Reference-side binding of the lower surface: the Isaac Gym calls the hand_arm task code makes, with
Isaac Gym's own signatures (`gym.<fn>(sim, ...)`, `gymtorch.wrap_tensor/unwrap_tensor`), routed to
libhandarm_hip.so through ``HandArmSim``.

Call sites this serves (under /root/reference/isaacgymenvs):
  gym.simulate / fetch_results                    tasks/base/vec_task.py:412-416
  gym.acquire_*_tensor + gymtorch.wrap_tensor     tasks/hand_arm/base/observable_vec_task.py:123-155
  gym.refresh_*_tensor                            observable_vec_task.py:173-177
  gym.set_dof_position_target_tensor              tasks/hand_arm/base/actionable_vec_task.py:39-40
  gym.set_actor_root_state_tensor_indexed         tasks/hand_arm/task/multi_object_manipulation.py:89,118,167,228
  gym.set_dof_state_tensor_indexed                tasks/hand_arm/base/ur5sih.py:630
  gym.set_dof_position_target_tensor_indexed      ur5sih.py:626
  gym.apply_rigid_body_force_tensors              tasks/allegro_kuka/allegro_kuka_base.py:1412-1414
  gym.acquire_dof_force_tensor / refresh          tasks/allegro_hand.py:151-152,409
Isaac Gym returns bool from the set_* calls; so does this (a failing ABI call raises HandArmError
instead of being silently ignored).
"""
import types

import torch

from .sim import HandArmSim


class _Unwrapped:
    """gymtorch.unwrap_tensor result: keeps the tensor (the ABI needs its device pointer and dtype)."""
    __slots__ = ("tensor",)

    def __init__(self, t):
        self.tensor = t


gymtorch = types.SimpleNamespace(
    unwrap_tensor=lambda t: _Unwrapped(t),
    wrap_tensor=lambda t: t,                 # acquire_* already returns the live torch tensor
)
# gymapi.CoordinateSpace values used by apply_rigid_body_force_tensors
gymapi = types.SimpleNamespace(ENV_SPACE=0, LOCAL_SPACE=1, GLOBAL_SPACE=2)


def _quat_rotate(q, v):
    """Rotate v (..., 3) by unit quaternions q (..., 4) xyzw."""
    qv, w = q[..., :3], q[..., 3:4]
    t = 2.0 * torch.cross(qv, v, dim=-1)
    return v + w * t + torch.cross(qv, t, dim=-1)


def _t(x):
    return x.tensor if isinstance(x, _Unwrapped) else x


class Gym:
    """The subset of isaacgym.gymapi.Gym the hand-arm task calls. ``create_sim`` returns the sim handle."""

    def create_sim(self, num_envs, device="cuda:0", **kw):
        return HandArmSim(num_envs, device, **kw)

    def prepare_sim(self, sim):
        return True

    def simulate(self, sim):
        sim.simulate(1)

    def fetch_results(self, sim, wait):
        sim.fetch_results(wait)

    def acquire_actor_root_state_tensor(self, sim):
        return sim.acquire_actor_root_state_tensor()

    def acquire_rigid_body_state_tensor(self, sim):
        return sim.acquire_rigid_body_state_tensor()

    def acquire_dof_state_tensor(self, sim):
        return sim.acquire_dof_state_tensor()

    def acquire_net_contact_force_tensor(self, sim):
        return sim.acquire_net_contact_force_tensor()

    def acquire_dof_force_tensor(self, sim):
        return sim.t["dof_force"]

    def refresh_actor_root_state_tensor(self, sim):
        sim.refresh_actor_root_state_tensor()

    refresh_rigid_body_state_tensor = refresh_dof_state_tensor = refresh_net_contact_force_tensor = \
        refresh_dof_force_tensor = refresh_actor_root_state_tensor

    def apply_rigid_body_force_tensors(self, sim, force_tensor=None, torque_tensor=None, space=gymapi.ENV_SPACE):
        """Forces (N*B or N, B, 3) at the COM of the free objects for the next simulate call. LOCAL_SPACE
        forces are rotated by the object's current orientation. Forces on robot links and torques are not
        supported by the simulator (the reference applies neither on the hot path)."""
        if torque_tensor is not None:
            raise NotImplementedError("rigid-body torques are not supported")
        if force_tensor is None:
            return True
        f = _t(force_tensor).view(sim.num_envs, sim.num_bodies, 3)
        o0, no = sim.model.body_object0, sim.n_obj
        fo = f[:, o0:o0 + no, :]
        if space == gymapi.LOCAL_SPACE:
            a0 = sim.model.actor_object0
            q = sim.t["root_state"].view(sim.num_envs, sim.num_actors, 13)[:, a0:a0 + no, 3:7]
            fo = _quat_rotate(q, fo)
        sim.t["object_force"].view(sim.num_envs, no, 3).copy_(fo)
        return True

    def set_dof_position_target_tensor(self, sim, targets):
        sim.set_dof_position_target_tensor(_t(targets))
        return True

    def set_actor_root_state_tensor_indexed(self, sim, root_state, actor_indices, n):
        sim.set_actor_root_state_tensor_indexed(_t(root_state), _t(actor_indices)[:n])
        return True

    def set_dof_state_tensor_indexed(self, sim, dof_state, actor_indices, n):
        sim.set_dof_state_tensor_indexed(_t(dof_state), _t(actor_indices)[:n])
        return True

    def set_dof_position_target_tensor_indexed(self, sim, targets, actor_indices, n):
        sim.set_dof_position_target_tensor_indexed(_t(targets), _t(actor_indices)[:n])
        return True


def acquire_gym():
    """gymapi.acquire_gym() analogue."""
    return Gym()
