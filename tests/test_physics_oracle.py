"""CPU checks of the C oracle: controller vs reference goldens, and physical sanity of the simulator
(physics parity vs PhysX is unpinned; these are the domain properties it must satisfy)."""
import os

import numpy as np
import pytest

from handarm_hip import model as HM
from oracle.oracle_lib import HostState, Oracle
from tests import scenes

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def mp():
    m = HM.build_model(HM.load_scene())
    p, cfg = HM.build_params()
    return m, p, cfg


def test_c_controller_against_reference_goldens(mp):
    m, p, _ = mp
    d = np.load(os.path.join(G, "ur5sih_controller.npz"))
    steps, n = d["actions"].shape[:2]
    orc = Oracle(m, p, n)
    st = HostState(n)
    st["ur5_target"][:] = d["init_ur5_target"]
    st["servo"][:] = d["init_servo"]
    for s in range(steps):
        st["dof_state"].reshape(n, 17, 2)[..., 0] = d["dof_pos"][s]
        st["actions"][:] = d["actions"][s]
        orc.controller(st)
        np.testing.assert_array_equal(st["ur5_target"], d["ur5_target"][s])
        np.testing.assert_array_equal(st["smoothed"], d["smoothed"][s])
        np.testing.assert_array_equal(st["servo"], d["servo"][s])
        np.testing.assert_allclose(st["dof_position_targets"], d["targets"][s], rtol=1e-6, atol=1e-6)


def _scene(mp, n, seed=0, collide=True):
    m, p, _ = mp
    orc = Oracle(m, p, n)
    st = HostState(n)
    scenes.fill_scene(st, n, seed=seed)
    if not collide:
        st["collision_enabled"][:] = 0
    return orc, st


def test_saturating_drives_stay_stable(mp):
    orc, st = _scene(mp, 4, collide=False)
    st["sim_targets"][:, 6:] = np.where(np.arange(6, 17) == 14, 0.0, -1.5)   # drive fingers hard into flexion
    st["sim_targets"][:, 15:] = 1.5
    for _ in range(30):
        orc.simulate(st, 1)
    ds = st["dof_state"].reshape(4, 17, 2)
    assert np.isfinite(ds).all()
    assert np.abs(ds[..., 1]).max() < 20.0
    # the PD drives pull the fingers toward their (limit-clamped) targets
    assert (ds[:, 6:14, 0] < -1.0).all()


def test_arm_tracks_target(mp):
    orc, st = _scene(mp, 2, collide=False)
    ds = st["dof_state"].reshape(2, 17, 2)
    ds[..., 1] = 0
    tgt = ds[..., 0].copy()
    tgt[:, 0] += 0.1
    st["sim_targets"][:] = tgt
    for _ in range(120):        # 2 s
        orc.simulate(st, 1)
    np.testing.assert_allclose(ds[:, 0, 0], tgt[:, 0], atol=5e-3)


def test_free_fall_is_symplectic_euler(mp):
    m, p, cfg = mp
    orc, st = _scene(mp, 1)
    rs = st["root_state"].reshape(1, 6, 13)
    rs[0, 3:, 0] = [0.1, 0.3, 0.5]
    rs[0, 3:, 1] = 0.55
    rs[0, 3:, 2] = 1.5
    rs[0, 3:, 3:7] = [0, 0, 0, 1]
    rs[0, 3:, 7:13] = 0
    z0 = rs[0, 3:, 2].copy()
    orc.simulate(st, 5)                          # 10 substeps, nothing to hit
    h = np.float32(cfg["dt"] / 2)
    k = 10
    z = z0 - 9.81 * h * h * k * (k + 1) / 2
    np.testing.assert_allclose(rs[0, 3:, 2], z, atol=2e-5)
    np.testing.assert_allclose(rs[0, 3:, 9], -9.81 * h * k, rtol=1e-5)


def test_objects_settle_on_table(mp):
    orc, st = _scene(mp, 8, seed=3)
    for _ in range(60):
        orc.simulate(st, 1)
    rs = st["root_state"].reshape(8, 6, 13)
    assert np.isfinite(rs).all()
    assert (rs[:, 3:, 2] > 0.5).all() and (rs[:, 3:, 2] < 0.7).all()
    assert np.median(np.abs(rs[:, 3:, 7:10])) < 0.05


def test_bin_scene_layout():
    """tools/build_model.py --bin: the table with a hole and the tote as static boxes (multi_object.py:535-540,
    497-507), gym layout goal / robot / table / bin / 8 objects, fixed bodies for the table links and the bin."""
    scene = HM.load_scene(HM.BIN_ASSET)
    m = HM.build_model(scene)
    assert (m.n_actors, m.actor_object0, m.n_bodies, m.body_object0) == (12, 4, 44, 36)
    assert m.n_static == 9 and m.table_hull == -1 and m.n_fixed_bodies == 6 and m.body_fixed0 == 30
    lo, hi = np.array(scene["bin_extent"][0]), np.array(scene["bin_extent"][1])
    np.testing.assert_allclose(lo, [0.10, 0.2325, 0.31], atol=1e-9)   # bin_info.yaml extent + bin.pos + table
    np.testing.assert_allclose(hi, [0.46, 0.8275, 0.565], atol=1e-9)
    # the four table walls leave exactly the hole open at the table top
    for k in range(4):
        c, h = np.array(m.static_pos[k][:]), np.array(m.static_half[k][:])
        assert c[2] + h[2] == pytest.approx(0.5, abs=1e-6)
        inter = (np.minimum(c[:2] + h[:2], hi[:2]) - np.maximum(c[:2] - h[:2], lo[:2])).clip(0)
        assert inter.prod() < 1e-6, "a table wall covers the hole"
    # tote floor: top face at the inner floor (mesh z 0.005 - 0.19 + table height)
    assert m.static_pos[4][2] + m.static_half[4][2] == pytest.approx(0.315, abs=1e-6)


def test_bin_objects_settle_in_tote():
    """C oracle, 8 objects per env dropped into the tote: they stay inside the bin extent, rest on the floor
    or on each other, and each object's net contact force carries its weight."""
    scene = HM.load_scene(HM.BIN_ASSET)
    m = HM.build_model(scene)
    p, _ = HM.build_params({"n_objects": 8})
    n = 8
    st = HostState(n, model=m, params=p)
    scenes.fill_bin_scene(st, n, scene, seed=0)
    orc = Oracle(m, p, n)
    for _ in range(60):
        orc.simulate(st, 1)
    rs = st["root_state"].reshape(n, 12, 13)
    assert np.isfinite(rs).all()
    lo, hi = np.array(scene["bin_extent"][0]), np.array(scene["bin_extent"][1])
    pos = rs[:, 4:, 0:3]
    assert ((pos >= lo) & (pos <= hi)).all()
    assert pos[..., 2].min() > 0.315
    assert np.median(np.abs(rs[:, 4:, 7:10])) < 0.02
    f = st["net_contact_force"].reshape(n, 44, 3)[:, 36:44]
    mass = np.array([m.pool_mass[i] for i in range(16)])[st["object_indices"]]
    np.testing.assert_allclose(np.median(f[..., 2] / (9.81 * mass)), 1.0, rtol=0.1)
    # fixed bodies: model poses, zero velocity
    body = st["rigid_body_state"].reshape(n, 44, 13)
    np.testing.assert_array_equal(body[:, 30:36, 0:7], np.broadcast_to(
        np.array([list(m.body_fixed_pose[k]) for k in range(6)], np.float32), (n, 6, 7)))
