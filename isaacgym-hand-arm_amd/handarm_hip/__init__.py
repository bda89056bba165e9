"""handarm_hip - MI355X-native hand-arm manipulation environment (HIP kernels for gfx950).

Drop-in for the Ur5SihMultiObjectManipulation hot path of maltemosbach/isaacgym-hand-arm:
VecTask step()/reset() on top, the Isaac Gym tensor API (libhandarm_hip.so, include/handarm_abi.h)
below.  See DESIGN.md.
"""
from . import model  # noqa: F401

__all__ = ["model", "make"]


def make(task="Ur5SihMultiObjectManipulation", num_envs=8192, sim_device="cuda:0", rl_device=None, cfg=None):
    """isaacgymenvs.make() analogue (isaacgymenvs/__init__.py:16-57) for the hand-arm task."""
    from .tasks import isaacgym_task_map
    cfg = dict(cfg or {})
    cfg.setdefault("env", {})["numEnvs"] = num_envs
    return isaacgym_task_map[task](cfg, rl_device or sim_device, sim_device)
