"""Self-collision of the Allegro actors on the C oracle (CPU). Both Allegro tasks create the hand with collision
filter -1 (allegro_hand.py:334-335, allegro_kuka_base.py:664), so PhysX collides every link pair except parent and
child; the build restates that as ha_model_t v12 self pairs with an oriented-box mid-phase (include/ha_obb.h).
Drives that push two fingers into each other, and the thumb into the palm, end within contact_slop after 120 calls
(2 s) with it, and interpenetrate by centimetres without it."""
import numpy as np
import pytest

from handarm_hip import model as HM
from oracle.oracle_lib import HostState, Oracle
from tests import self_collision_scenes as SC


def _setup(task):
    asset = HM.ALLEGRO_ASSET if task == HM.TASK_ALLEGRO_HAND else HM.KUKA_ASSET
    scene = HM.load_scene(asset)
    p, _ = HM.build_params(task=task)
    m_on, m_off = HM.build_model(scene), HM.build_model(SC.without_self_collision(scene))
    D = m_on.n_dofs
    lo, up = np.array(m_on.dof_lower[:D], np.float32), np.array(m_on.dof_upper[:D], np.float32)
    drives = SC.allegro_drives(lo, up) if task == HM.TASK_ALLEGRO_HAND else SC.kuka_drives(lo, up, list(p.reset_pose))
    return scene, p, m_on, m_off, drives


def test_self_pairs_in_the_model():
    for task, npairs in ((HM.TASK_ALLEGRO_HAND, 202), (HM.TASK_ALLEGRO_KUKA, 289)):
        scene, p, m_on, m_off, _ = _setup(task)
        assert m_on.n_self_pairs == npairs and m_off.n_self_pairs == 0
        L = [m_on.link_parent[i] for i in range(m_on.n_links)]
        for k in range(m_on.n_self_pairs):
            a, b = m_on.self_pair[k] & 255, m_on.self_pair[k] >> 8
            la, lb = m_on.hull_link[a], m_on.hull_link[b]
            assert la != lb and L[la] != lb and L[lb] != la
    m = HM.build_model(HM.load_scene(HM.ASSET))
    assert m.n_self_pairs == 0                  # Ur5Sih: robot filter 0b1, no self-collision (ur5sih.py:123-125)


def test_hull_boxes_contain_their_hulls():
    scene = HM.load_scene(HM.ALLEGRO_ASSET)
    m = HM.build_model(scene)
    for k, h in enumerate(scene["link_hulls"]):
        ob = np.array(list(m.hull_obb[k]), np.float64)
        x, y, z, w = ob[6:10]
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        loc = (np.asarray(h["verts"]) - ob[0:3]) @ R
        assert (np.abs(loc) <= ob[3:6] + 1e-7).all()


@pytest.mark.parametrize("task", [HM.TASK_ALLEGRO_HAND, HM.TASK_ALLEGRO_KUKA])
def test_fingers_and_thumb_stop_at_the_contact_slop(task):
    scene, p, m_on, m_off, drives = _setup(task)
    names = list(drives)
    n = len(names)
    targets = np.stack([drives[k] for k in names])
    probe = Oracle(m_on, p, n)
    seps = {}
    for tag, m in (("on", m_on), ("off", m_off)):
        st = SC.drive_state(HostState(n, model=m, params=p), m, targets, n)
        Oracle(m, p, n).simulate(st, 120)
        seps[tag] = [SC.min_self_separation(probe, st, e) for e in range(n)]
        assert np.isfinite(st["dof_state"]).all()
    print(task, dict(zip(names, seps["on"])), dict(zip(names, seps["off"])))
    for e, k in enumerate(names):
        assert seps["on"][e] >= -(p.contact_slop + 5e-4), (k, seps["on"][e])
        assert seps["off"][e] < -0.01, (k, "the drive must push the links into each other", seps["off"][e])


def test_no_self_contacts_at_the_reset_poses():
    """the self pairs are every non-adjacent link pair (no exclude list). At each task's reset pose - AllegroHand
    zero DOF positions clamped to the limits (allegro_hand.py:252-273), AllegroKuka the arm's desired pose with the
    fingers at 0 (allegro_kuka_base.py:316-319) - at zero velocity, no pair of cooked hulls is within the contact offset,
    so no standing self contact pushes against the PD drives at rest."""
    for task in (HM.TASK_ALLEGRO_HAND, HM.TASK_ALLEGRO_KUKA):
        scene, p, m, _, _ = _setup(task)
        D = m.n_dofs
        lo, up = np.array(m.dof_lower[:D], np.float32), np.array(m.dof_upper[:D], np.float32)
        pose = np.array(list(p.reset_pose)[:D], np.float32) if task == HM.TASK_ALLEGRO_KUKA else np.zeros(D, np.float32)
        st = HostState(1, model=m, params=p)
        st["dof_state"].reshape(1, D, 2)[0, :, 0] = np.clip(pose, lo, up)
        rs = st["root_state"].reshape(1, m.n_actors, 13)
        rs[..., 6] = 1.0
        rs[0, m.actor_object0, 0:3] = [5.0, 5.0, 5.0]         # the object out of reach
        if task == HM.TASK_ALLEGRO_KUKA:
            st["object_scale"][:] = 1.0
        cs = Oracle(m, p, 1).contacts(st, 0)
        assert not [r for r in cs if r[7] >= 100 and r[8] >= 100], (task, cs)
        # and the oracle's simulate agrees: one call offers no self-collision contact
        st["sim_targets"][0] = np.clip(pose, lo, up)
        Oracle(m, p, 1).simulate(st, 1)
        assert st["contact_stats"][0, 4] == 0
