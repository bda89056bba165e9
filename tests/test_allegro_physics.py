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
    # the cube never sinks through the ground plane
    z = root[:, 1, 2]
    assert (z > 0.0325 - 0.01).all()


def _cube_energy(model, root):
    """mechanical energy of the cube: translational + rotational kinetic energy + potential energy (ground z = 0)."""
    m = model.pool_mass[0]
    I0 = np.array(list(model.pool_inertia[0]), np.float64).reshape(3, 3)
    q = root[:, 1, 3:7].astype(np.float64)
    x, y, zq, w = q.T
    R = np.stack([np.stack([1 - 2 * (y * y + zq * zq), 2 * (x * y - zq * w), 2 * (x * zq + y * w)], -1),
                  np.stack([2 * (x * y + zq * w), 1 - 2 * (x * x + zq * zq), 2 * (y * zq - x * w)], -1),
                  np.stack([2 * (x * zq - y * w), 2 * (y * zq + x * w), 1 - 2 * (x * x + y * y)], -1)], 1)
    om = root[:, 1, 10:13].astype(np.float64)
    Iw = R @ I0 @ np.transpose(R, (0, 2, 1))
    v = root[:, 1, 7:10].astype(np.float64)
    return 0.5 * m * (v * v).sum(-1) + 0.5 * np.einsum("ni,nij,nj->n", om, Iw, om) + m * 9.81 * root[:, 1, 2]


def test_allegro_cube_released_by_the_hand_gains_no_energy():
    """The random scene starts with fingers interpenetrating the cube by up to 3.4 cm, and AllegroHand's
    max_depenetration_velocity (1000, AllegroHand.yaml) lets the push-out throw it (up to ~1.6 m/s: it can fly over a
    metre). That throw is the only energy source once the hand lets go. From the call on which no finger touches the
    cube: (1) its mechanical energy (kinetic + rotational + potential) never exceeds its value at release (+1%); (2) from
    one call to the next it grows only by the Baumgarte push-out of a ground penetration present at the start of the
    call (a cube landing at 3 m/s moves 2.6 cm per substep, against a 2 mm speculative margin), by at most the
    potential energy of that depth, m g depth, plus 1% + 1e-4 J."""
    n = 16
    model, params, st, lo, up = setup(n)
    orc = Oracle(model, params, n)
    root = st["root_state"].reshape(n, 3, 13)
    seps = np.array([orc.contacts(st, e)[:, 6].min(initial=0.0) for e in range(n)])
    assert seps.min() < -0.02, "the scene starts with deep finger-cube interpenetration"
    mg = model.pool_mass[0] * 9.81
    released = np.zeros(n, bool)
    e_rel = np.zeros(n)
    e_prev = _cube_energy(model, root)
    checked = pushed = 0
    for c in range(60):
        cts = [orc.contacts(st, e) for e in range(n)]
        # a finger on the cube (object 0): link-link (self-collision) contacts do not count
        touch = np.array([any((int(a) >= 100 and int(b) == 0) or (int(a) == 0 and int(b) >= 100) for a, b in ct[:, 7:9])
                          for ct in cts])
        pen = np.array([max(0.0, -min([float(r[6]) for r in ct if int(r[8]) == -1], default=0.0)) for ct in cts])
        new = ~released & ~touch
        e_rel[new] = e_prev[new]
        released |= ~touch
        orc.simulate(st, 1)
        e_now = _cube_energy(model, root)
        chk = released & ~touch
        grow = e_now - e_prev
        allow = 0.01 * e_prev + 1e-4 + mg * pen
        assert (grow[chk] <= allow[chk]).all(), (c, np.nonzero(chk & (grow > allow)))
        assert (e_now[chk] <= 1.01 * e_rel[chk] + 1e-4).all(), (c, np.nonzero(chk & (e_now > 1.01 * e_rel + 1e-4)))
        checked += int(chk.sum())
        pushed += int((chk & (grow > 0.01 * e_prev + 1e-4)).sum())
        e_prev = e_now
    assert checked > 100 and released.sum() >= 4
    z = root[:, 1, 2]
    assert (z > 0.0325 - 0.01).all()


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
