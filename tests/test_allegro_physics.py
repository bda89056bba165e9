"""AllegroHand scene on the C physics oracle (CPU): the restated physics is stable for the Allegro model
(17 bodies, 16 DOF with armature, one free cube, no table) and behaves physically. Parity vs PhysX is
unpinned; the GPU is compared with this oracle in test_gpu_allegro.py."""
import numpy as np

from handarm_hip import model as HM
from oracle.oracle_lib import HostState, Oracle
from tests import scenes


def setup(n, seed=0, in_hand=1.0):
    model = HM.build_model(HM.load_scene(HM.ALLEGRO_ASSET))
    params, _ = HM.build_params(task=HM.TASK_ALLEGRO_HAND)
    lo, up = np.array(model.dof_lower[:16], np.float32), np.array(model.dof_upper[:16], np.float32)
    st = HostState(n, model=model, params=params)
    scenes.fill_allegro_scene(st, n, lo, up, seed=seed, in_hand=in_hand)
    return model, params, st, lo, up


def test_allegro_physics_is_stable_and_tracks_targets():
    n = 16
    model, params, st, lo, up = setup(n)
    orc = Oracle(model, params, n)
    orc.simulate(st, 60)                         # 1 s
    dof = st["dof_state"].reshape(n, 16, 2)
    root = st["root_state"].reshape(n, 3, 13)
    assert np.isfinite(dof).all() and np.isfinite(root).all()
    # PD drives (kp 3, kd 0.1, effort 0.5) pull the joints to their targets; contacts may block a few
    err = np.abs(dof[..., 0] - st["sim_targets"])
    assert np.median(err) < 0.05, np.median(err)
    assert (dof[..., 0] >= lo - 0.05).all() and (dof[..., 0] <= up + 0.05).all()
    # the cube never sinks through the ground plane and stays near the hand or on the ground
    z = root[:, 1, 2]
    assert (z > 0.0325 - 0.01).all()
    assert np.abs(root[:, 1, 0]).max() < 1.0        # a cube thrown off the hand tumbles on the ground, then rests


def test_allegro_free_cube_falls_under_gravity():
    """A cube released well above the hand accelerates at g until contact."""
    n = 4
    model, params, st, lo, up = setup(n, in_hand=0.0)
    root = st["root_state"].reshape(n, 3, 13)
    root[:, 1, 0:3] = [0.0, 0.3, 1.5]             # clear of the hand
    root[:, 1, 7:13] = 0
    orc = Oracle(model, params, n)
    orc.simulate(st, 12)                          # 0.2 s
    t = 12 * params.dt
    np.testing.assert_allclose(root[:, 1, 9], -9.81 * t, rtol=2e-3)
    h = params.dt / params.substeps               # symplectic Euler: z = z0 - g h^2 n(n+1)/2
    np.testing.assert_allclose(root[:, 1, 2], 1.5 - 0.5 * 9.81 * t * (t + h), atol=5e-4)
