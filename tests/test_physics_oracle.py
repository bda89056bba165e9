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
