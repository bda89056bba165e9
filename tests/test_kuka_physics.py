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
    # joint limits hold within 0.05 rad, except where random targets jam the fingers into each other: there the
    # self-collision contacts (v12) and a joint-limit row are conflicting hard constraints, and 8 PGS sweeps leave a
    # compromise (seed 3: a ring-finger twist 0.07 rad over its limit against 20 finger-finger contacts). Such an env
    # must be one with deep self contacts, and stays within 0.1 rad
    viol = np.maximum(dof[..., 0] - up, lo - dof[..., 0]).max(-1)
    for e in np.nonzero(viol > 0.05)[0]:
        cs = orc.contacts(st, int(e))
        self_c = [r for r in cs if r[7] >= 100 and r[8] >= 100]
        assert len(self_c) >= 8 and min(r[6] for r in self_c) < -0.002 and viol[e] < 0.1, (e, viol[e], len(self_c))
    # PD drives (kp 40, kd 5) track the targets unless a contact or an effort limit holds a joint back
    assert np.median(np.abs(dof[..., 0] - st["sim_targets"])) < 0.05
    assert (root[:, 1, 2] > 0.0).all() and (root[:, 1, 2] < 1.5).all()


def friction_schedule(n, scales, mu, dt, simulate, root, dof, force):
    """Coulomb friction on the table (pyramid rows along x / y for a z contact normal, mu = combined friction):
    cuboids rest upright, then flat ones (x extent >= 1.5 x height, so the friction torque cannot tip them) get a
    horizontal push along -x at the centre of mass: half the friction limit for 30 calls, then 1.25 times it for
    12 calls. simulate() runs one gym.simulate; root(), dof() are writable (n, 4, 13) / (n, 23, 2) views or
    copies, force(f) sets this call's (n, 3) object force. Returns the flat-env mask and the recorded states."""
    flat = scales[:, 0, 0] >= 1.5 * scales[:, 0, 2]
    mass = 400.0 * 0.05 ** 3 * scales[:, 0].prod(-1)
    limit = mu * mass * 9.81
    rec = {}

    def run(calls, push):
        for _ in range(calls):
            f = np.zeros((n, 3), np.float32)
            f[flat, 0] = -push * limit[flat]
            force(f)
            dof()[..., 1] = 0                                      # the hand holds still, away from the table
            simulate()

    run(30, 0.0)
    rec["settled"] = root().copy()
    run(30, 0.5)
    rec["held"] = root().copy()
    run(8, 1.25)
    rec["pushed"] = root().copy()
    return flat, rec


def check_friction(flat, rec, mu, dt):
    s, h, p = rec["settled"][:, 1], rec["held"][:, 1], rec["pushed"][:, 1]
    assert flat.sum() >= 5
    # below the limit: static friction holds (no creep beyond 1 mm, at rest)
    assert np.abs(h[:, 0:3] - s[:, 0:3]).max() < 1e-3
    assert np.abs(h[:, 7:10]).max() < 5e-3
    # above it: kinetic friction mu N opposes the push, so the cuboid gains (1.25 - 1) mu g per second
    v_exp = -0.25 * mu * 9.81 * 8 * dt
    np.testing.assert_allclose(p[flat, 7], v_exp, rtol=0.02)
    assert np.abs(p[flat, 8]).max() < 0.05 * abs(v_exp)           # no sideways drift
    assert np.abs(p[flat, 3:5]).max() < 0.05                      # slides upright, does not tip
    assert np.abs(p[~flat, 7:10]).max() < 5e-3                    # unpushed cuboids stay at rest


def test_friction_holds_below_and_slides_above_the_coulomb_limit():
    n = 24
    scene, model, params, st, scales, lo, up = setup(n)
    root = st["root_state"].reshape(n, 4, 13)
    root[:, 1, 7:13] = 0
    root[:, 1, 3:7] = [0, 0, 0, 1]
    root[:, 1, 0:2] = [0.13, -0.09]
    root[:, 1, 2] = 0.53 + 0.025 * scales[:, 0, 2] + 0.002
    orc = Oracle(model, params, n)

    def force(f):
        st["object_force"].reshape(n, -1, 3)[:, 0] = f

    flat, rec = friction_schedule(n, scales, params.friction, params.dt, lambda: orc.simulate(st, 1),
                                  lambda: st["root_state"].reshape(n, 4, 13),
                                  lambda: st["dof_state"].reshape(n, 23, 2), force)
    print("friction: pushed flat cuboids vx", rec["pushed"][flat, 1, 7].round(3).tolist())
    check_friction(flat, rec, params.friction, params.dt)


def drop_schedule(n, scales, simulate, root, dof, calls=60, height=0.10):
    """Flat cuboids (as in friction_schedule) dropped from `height` above their resting height onto the table;
    returns the flat mask and z - z_rest of every env after every call."""
    flat = scales[:, 0, 0] >= 1.5 * scales[:, 0, 2]
    zs = []
    for _ in range(calls):
        dof()[..., 1] = 0
        simulate()
        zs.append(root()[:, 1, 2] - (0.53 + 0.025 * scales[:, 0, 2]))
    return flat, np.array(zs)


def check_drop(flat, zs, root_final, slop):
    z = zs[:, flat]
    impact = np.argmax(z < slop, axis=0)
    assert (impact > 0).all() and (impact < 20).all()
    # penetration peaks at the impact call (1.4 m/s): measured 3.6 mm on this build; it is worked off to the
    # contact slop (the depth the position correction leaves alone) and the cuboid does not bounce back up
    assert -z.min() < 5e-3
    for e in range(z.shape[1]):
        assert z[impact[e] + 1:, e].max() < 0.5 * slop
    np.testing.assert_allclose(z[-10:], -slop, atol=0.2 * slop)
    assert np.abs(root_final[flat, 1, 7:10]).max() < 5e-3             # at rest
    assert np.abs(root_final[flat, 1, 10:13]).max() < 5e-2            # residual rocking (measured 0.023 rad/s)
    # upright to within the slop across the base (measured tilt <= 0.85 deg: quat x, y <= 0.0074)
    assert np.abs(root_final[flat, 1, 3:5]).max() < 1e-2


def test_dropped_cuboids_penetrate_boundedly_and_come_to_rest_at_the_slop():
    n = 24
    scene, model, params, st, scales, lo, up = setup(n)
    root = st["root_state"].reshape(n, 4, 13)
    root[:, 1, 7:13] = 0
    root[:, 1, 3:7] = [0, 0, 0, 1]
    root[:, 1, 0:2] = [0.13, -0.09]
    root[:, 1, 2] = 0.53 + 0.025 * scales[:, 0, 2] + 0.10
    orc = Oracle(model, params, n)
    flat, zs = drop_schedule(n, scales, lambda: orc.simulate(st, 1), lambda: st["root_state"].reshape(n, 4, 13),
                             lambda: st["dof_state"].reshape(n, 23, 2))
    print("drop: peak penetration %.2f mm, final %.3f mm" % (-zs[:, flat].min() * 1e3, zs[-1, flat].mean() * 1e3))
    check_drop(flat, zs, root, params.contact_slop)
