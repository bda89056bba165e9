"""AllegroKuka scene on the C physics oracle (CPU): per-env cuboid dimensions (scaled pool hull, mass and
inertia), the table, the 23-DOF arm+hand, and the object force channel (apply_rigid_body_force_tensors).
Parity vs PhysX is unpinned; the GPU is compared with this oracle in test_gpu_kuka.py."""
import numpy as np

from handarm_hip import model as HM
from oracle.oracle_lib import HostState, Oracle
from tests import scenes


def setup(n, seed=0, force=0.0):
    scene = HM.load_scene(HM.KUKA_ASSET)
    model = HM.build_model(scene)
    params, cfg = HM.build_params(task=HM.TASK_ALLEGRO_KUKA)
    lo, up = np.array(model.dof_lower[:23], np.float32), np.array(model.dof_upper[:23], np.float32)
    scales, _ = HM.kuka_env_tables(n, scene, cfg)
    st = HostState(n, model=model, params=params)
    scenes.fill_kuka_scene(st, n, lo, up, list(params.reset_pose), scales, list(model.table_pos), seed=seed,
                           object_force=force)
    return scene, model, params, st, scales, lo, up


def test_cuboids_settle_on_the_table_with_their_own_weight():
    n = 12
    scene, model, params, st, scales, lo, up = setup(n)
    root = st["root_state"].reshape(n, 4, 13)
    root[:, 1, 7:13] = 0
    root[:, 1, 3:7] = [0, 0, 0, 1]                               # upright: rests on its z face
    root[:, 1, 0:2] = [0.12, -0.09]    # table front half, clear of the hand; the 20 cm cuboids (scale 4) end inside the
                                       # table edges (x 0.2375, y -0.2): vertex contacts do not clip an overhanging face
    root[:, 1, 2] = 0.53 + 0.025 * scales[:, 0, 2] + 0.002
    orc = Oracle(model, params, n)
    for _ in range(90):
        st["dof_state"].reshape(n, 23, 2)[..., 1] = 0             # keep the hand still, away from the table
        orc.simulate(st, 1)
    z = root[:, 1, 2]
    np.testing.assert_allclose(z, 0.53 + 0.025 * scales[:, 0, 2], atol=2e-3)
    mass = 400.0 * 0.05 ** 3 * scales[:, 0].prod(-1)
    fz = st["net_contact_force"].reshape(n, 27, 3)[:, 24, 2]
    np.testing.assert_allclose(fz, 9.81 * mass, rtol=0.05)


def test_object_force_accelerates_a_free_cuboid():
    """object_force is consumed by one simulate call and adds F/m to the free-fall velocity."""
    n = 4
    scene, model, params, st, scales, lo, up = setup(n)
    root = st["root_state"].reshape(n, 4, 13)
    root[:, 1, 0:3] = [0.0, -0.6, 1.5]                          # clear of table and hand
    root[:, 1, 7:13] = 0
    f = np.array([[0.3, -0.2, 0.5]], np.float32) * (np.arange(n)[:, None] + 1)
    st["object_force"][:] = f[:, None, :]
    orc = Oracle(model, params, n)
    orc.simulate(st, 1)
    mass = 400.0 * 0.05 ** 3 * scales[:, 0].prod(-1)
    v = root[:, 1, 7:10].copy()
    exp = f / mass[:, None] * params.dt + np.array([0, 0, -9.81]) * params.dt
    np.testing.assert_allclose(v, exp, rtol=2e-3, atol=1e-5)
    assert np.all(st["object_force"] == 0)                      # consumed
    orc.simulate(st, 1)
    np.testing.assert_allclose(root[:, 1, 7:10] - v, np.tile([0, 0, -9.81 * params.dt], (n, 1)), atol=1e-5)


def test_arm_and_hand_stay_stable_under_random_targets_and_forces():
    n = 16
    scene, model, params, st, scales, lo, up = setup(n, seed=3, force=1.0)
    orc = Oracle(model, params, n)
    for _ in range(60):
        orc.simulate(st, 1)
    dof = st["dof_state"].reshape(n, 23, 2)
    root = st["root_state"].reshape(n, 4, 13)
    assert np.isfinite(dof).all() and np.isfinite(root).all()
    assert (dof[..., 0] >= lo - 0.05).all() and (dof[..., 0] <= up + 0.05).all()
    # PD drives (kp 40, kd 5) track the targets unless a contact or an effort limit holds a joint back
    assert np.median(np.abs(dof[..., 0] - st["sim_targets"])) < 0.05
    assert (root[:, 1, 2] > 0.0).all() and (root[:, 1, 2] < 1.5).all()
