"""Self-collision drive scenes (shared by tests/test_self_collision.py on the C oracle and tests/test_gpu_self_collision.py
on the GPU): joint targets that push robot links into each other, and the deepest link-link interpenetration of a
state, measured with the oracle's contact generation."""
import numpy as np

from handarm_hip import model as HM

F = np.float32


def allegro_drives(lo, up):
    """AllegroHand DOF targets (index 0-3, middle 4-7, ring 8-11, thumb 12-15):
    'fingers': index and middle curled (joints 1-3 at 1.2 rad) with their base twists turned toward each other
               (-0.55 / +0.55): index link 2-3 and middle link 2-3 cross;
    'thumb':   every thumb joint at its upper limit: the thumb tip presses into the palm."""
    f = np.zeros(16, F)
    f[0], f[4] = -0.55, 0.55
    f[1:4] = 1.2
    f[5:8] = 1.2
    t = np.zeros(16, F)
    t[12:16] = up[12:16]
    return {"fingers": f, "thumb": t}


def kuka_drives(lo, up, reset_pose):
    """AllegroKuka (arm 0-6 at its reset pose, hand 7-22 in the AllegroHand order): the same two drives."""
    arm = np.asarray(reset_pose[:7], F)
    out = {}
    for k, v in allegro_drives(lo[7:], up[7:]).items():
        out[k] = np.concatenate([arm, v]).astype(F)
    return out


def without_self_collision(scene):
    s = dict(scene)
    s.pop("self_collision", None)
    return s


def min_self_separation(probe, st, env):
    """deepest link-link contact separation of env's state (probe: an oracle whose model has the self pairs); 0 with
    no self contact"""
    cs = probe.contacts(st, env)
    return min([float(r[6]) for r in cs if r[7] >= 100 and r[8] >= 100], default=0.0)


def drive_state(st, m, targets, n, object_away=True):
    """Every env at the zero pose (clipped into the limits), at rest, driven to targets[e]; objects parked far away."""
    D = m.n_dofs
    lo = np.array(m.dof_lower[:D], F)
    up = np.array(m.dof_upper[:D], F)
    ds = st["dof_state"].reshape(n, D, 2)
    ds[..., 0] = np.clip(0.0, lo, up)
    if D == 23:
        ds[:, :7, 0] = targets[:, :7]
    ds[..., 1] = 0
    st["sim_targets"][:] = targets
    rs = st["root_state"].reshape(n, m.n_actors, 13)
    rs[..., 6] = 1
    if object_away:
        rs[:, m.actor_object0, 0:3] = [5.0, 5.0, 5.0]
    if m.actor_table >= 0:
        rs[:, m.actor_table, 0:3] = list(m.table_pos)
    st["collision_enabled"][:] = 1
    if "object_scale" in st.arrays:
        st["object_scale"][:] = 1.0
    return st
