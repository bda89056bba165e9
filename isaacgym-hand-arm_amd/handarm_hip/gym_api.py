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
Isaac Gym returns bool from the set_* calls; so does this (a failing ABI call raises HandArmError
instead of being silently ignored).
"""
import types

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

    def refresh_actor_root_state_tensor(self, sim):
        sim.refresh_actor_root_state_tensor()

    refresh_rigid_body_state_tensor = refresh_dof_state_tensor = refresh_net_contact_force_tensor = \
        refresh_actor_root_state_tensor

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
