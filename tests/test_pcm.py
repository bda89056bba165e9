"""Persistent contact manifolds (ha_params_t / ha_state_t v13) on the C oracle (CPU).

A candidate pair's narrow phase writes a record of the manifold it emitted (relative pose, per point the two surface
points in their bodies' frames and the normal in side B's frame); while the pair's relative pose stays within
pcm_lin_tol / pcm_cos_tol of that pose, later substeps re-evaluate those points from the current poses instead of
running the narrow phase (PhysX's persistent contact manifolds, inferred: its source is closed). The kernels run the same
expressions (tests/test_gpu_*: contact_cache is compared bit for bit like any physics output). These tests pin the
semantics: records hold the narrow phase's points, refreshed points equal the narrow phase's while nothing moves,
motion past the tolerances rebuilds the record, and resting / sliding behaviour is unchanged."""
import numpy as np

from handarm_hip import model as HM
from oracle import f32
from oracle.oracle_lib import HostState, Oracle
from tests import scenes
from tests.test_kuka_physics import setup


def _params(**kw):
    p, cfg = HM.build_params(task=HM.TASK_ALLEGRO_KUKA)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _resting_cuboids(n, model, st, scales):
    root = st["root_state"].reshape(n, 4, 13)
    root[:, 1, 7:13] = 0
    root[:, 1, 3:7] = [0, 0, 0, 1]
    root[:, 1, 0:2] = [0.12, -0.09]
    root[:, 1, 2] = 0.53 + 0.025 * scales[:, 0, 2] - 0.0005
    return root


def test_record_slots_follow_the_kernel_pair_enumeration():
    """ha_contact_cache_slots: per object its ground, statics, later objects and link hulls, then link hulls x statics,
    then the self pairs (the same count the kernel's env_body and the C oracle derive)."""
    from oracle.oracle_lib import load
    import ctypes as C
    lib = load()
    for task, asset, n_obj in ((HM.TASK_UR5SIH, HM.ASSET, 3), (HM.TASK_UR5SIH, HM.BIN_ASSET, 8),
                               (HM.TASK_ALLEGRO_HAND, HM.ALLEGRO_ASSET, 1), (HM.TASK_ALLEGRO_KUKA, HM.KUKA_ASSET, 1)):
        m = HM.build_model(HM.load_scene(asset))
        n = HM.pcm_slots(m, n_obj)
        assert lib.hao_pcm_slots(C.byref(m), n_obj) == n
        npairs = sum(1 + m.n_static + (n_obj - 1 - o) + m.n_link_hulls for o in range(n_obj)) + m.n_link_hulls * m.n_static
        assert n == npairs + m.n_self_pairs


def test_record_holds_the_narrow_phase_manifold_and_refresh_reproduces_it():
    """A cuboid pressed 0.5 mm into the table: after the first substep its object-table record (slot 1: ground 0, the
    table static 1) holds the points the narrow phase emitted. Re-evaluating them at the pose they were built from gives
    the same points (to float rounding) as the narrow phase at that pose."""
    n = 4
    scene, model, _, st, scales, lo, up = setup(n)
    params = _params(substeps=1)
    root = _resting_cuboids(n, model, st, scales)
    orc = Oracle(model, params, n)
    before = st.copy()
    expect = [orc.contacts(before, e) for e in range(n)]
    orc.simulate(st, 1)
    rec = st["contact_cache"][:, 1]
    for e in range(n):
        cube = [r for r in expect[e] if r[7] == 0 and r[8] == -1]
        k = int(rec[e, 3])
        assert k == len(cube) and 3 <= k <= 4, (e, k, len(cube))
        # relative pose of the cuboid's body frame (origin = root position) in the table frame at build time
        tpos = np.array(model.static_pos[0], np.float32)
        tq = np.array(model.static_quat[0], np.float32)
        q0 = before["root_state"].reshape(n, 4, 13)[e, 1, 3:7]
        p0 = before["root_state"].reshape(n, 4, 13)[e, 1, 0:3]
        tqc = tq * np.array([-1, -1, -1, 1], np.float32)
        np.testing.assert_allclose(rec[e, 0:3], f32.qrot(tqc[None], (p0 - tpos)[None])[0], atol=1e-6)
        # refreshed at the build pose: the two surface points x +- n sep / 2 and the normal
        for t in range(k):
            r = rec[e, 8 + 9 * t: 17 + 9 * t]
            wa = p0 + f32.qrot(q0[None], r[None, 0:3])[0]
            wb = tpos + f32.qrot(tq[None], r[None, 3:6])[0]
            nn = f32.qrot(tq[None], r[None, 6:9])[0]
            x, nrm, sep = cube[t][0:3], cube[t][3:6], cube[t][6]
            np.testing.assert_allclose(nn, nrm, atol=1e-6)
            np.testing.assert_allclose(np.dot(nn, wa - wb), sep, atol=2e-6)
            np.testing.assert_allclose(0.5 * (wa + wb), x, atol=2e-6)
    del root


def test_resting_cuboids_reuse_their_records_and_rest_like_the_narrow_phase():
    """Cuboids resting on the table: after the first substep the object-table pair is refreshed from its record in
    (almost) every substep (with the hand's self pairs the env refreshes more pairs than it has substeps); position,
    velocity and support force match the run without persistent manifolds."""
    n = 8
    scene, model, params, st, scales, lo, up = setup(n)
    _resting_cuboids(n, model, st, scales)
    runs = {}
    for on in (True, False):
        p = _params() if on else _params(pcm_lin_tol=0.0)
        s = st.copy()
        orc = Oracle(model, p, n)
        for _ in range(60):
            s["dof_state"].reshape(n, 23, 2)[..., 1] = 0
            orc.simulate(s, 1)
        runs[on] = s
    on, off = runs[True], runs[False]
    cs = on["contact_stats"]
    assert (cs[:, 5] >= cs[:, 0] - 4).all(), cs[:, [0, 5, 6]]         # the table pair refreshed nearly every substep
    assert (off["contact_stats"][:, 5] == 0).all()
    ro, rf = on["root_state"].reshape(n, 4, 13)[:, 1], off["root_state"].reshape(n, 4, 13)[:, 1]
    # the records reuse points within 1 mm / 2.3 degrees of their build pose: 1 s of rest ends within 2 mm of the run
    # without them (the long thin cuboids settle slowest), and every cuboid rests on its face at the table top
    np.testing.assert_allclose(ro[:, 0:3], rf[:, 0:3], atol=2e-3)
    np.testing.assert_allclose(ro[:, 2], 0.53 + 0.025 * scales[:, 0, 2], atol=1.5e-3)
    # the tall cuboids (scale 3) rock slowly either way (~0.1 rad/s): no faster with the records
    assert np.abs(ro[:, 7:13]).max(1).max() <= np.abs(rf[:, 7:13]).max(1).max() + 0.02
    fo = on["net_contact_force"].reshape(n, 27, 3)[:, 24, 2]
    ff = off["net_contact_force"].reshape(n, 27, 3)[:, 24, 2]
    np.testing.assert_allclose(fo, ff, rtol=0.05)


def test_motion_past_the_tolerance_rebuilds_the_record():
    """A record is reused only while the relative pose stays within the tolerances: a cuboid pushed sideways at
    40 cm/s moves 3.3 mm per substep (friction takes 8 cm/s per substep off; > pcm_lin_tol = 1 mm either way), so its
    table pair runs the narrow phase every substep and its record is rebuilt at each new pose."""
    n = 4
    scene, model, params, st, scales, lo, up = setup(n)
    root = _resting_cuboids(n, model, st, scales)
    root[:, 1, 7] = 0.4
    orc = Oracle(model, params, n)
    orc.simulate(st, 1)
    assert (st["contact_stats"][:, 6] >= 2).all()
    rec = st["contact_cache"][:, 1]
    assert (rec[:, 3] >= 1).all()
    # the record's relative position is the one of the last substep's pose (before its integration step), not the first
    # substep's 3 mm behind it
    tpos = np.array(model.static_pos[0], np.float32)
    x_last = root[:, 1, 0] - root[:, 1, 7] * (params.dt / params.substeps)
    np.testing.assert_allclose(rec[:, 0] + tpos[0], x_last, atol=2e-6)


def test_friction_and_sliding_unchanged_by_persistent_manifolds():
    """The Coulomb behaviour (tests/test_kuka_physics.py) with and without persistent manifolds: a cuboid pushed at
    half the friction limit stays put either way, and one pushed at 1.25x slides at the same speed to within 2%."""
    n = 2
    scene, model, params, st, scales, lo, up = setup(n)
    root = _resting_cuboids(n, model, st, scales)
    root[:, 1, 2] += 0.0005
    mass = 400.0 * 0.05 ** 3 * scales[:, 0].prod(-1)
    res = {}
    for on in (True, False):
        p = _params() if on else _params(pcm_lin_tol=0.0)
        orc = Oracle(model, p, n)
        for fr, tag in ((0.5, "hold"), (1.25, "slide")):
            s = st.copy()
            for _ in range(20):
                s["dof_state"].reshape(n, 23, 2)[..., 1] = 0
                orc.simulate(s, 1)
            x0 = s["root_state"].reshape(n, 4, 13)[:, 1, 0].copy()
            for _ in range(8):
                s["object_force"].reshape(n, 3)[:, 0] = -fr * 9.81 * mass
                s["dof_state"].reshape(n, 23, 2)[..., 1] = 0
                orc.simulate(s, 1)
            r = s["root_state"].reshape(n, 4, 13)[:, 1]
            res[(on, tag)] = (r[:, 0] - x0, r[:, 7].copy())
    for on in (True, False):
        dx, _ = res[(on, "hold")]
        assert np.abs(dx).max() < 1e-3, (on, dx)
    np.testing.assert_allclose(res[(True, "slide")][1], res[(False, "slide")][1], rtol=0.02)


def test_compound_and_clutter_scenes_match_without_drift():
    """The 8-object bin (compound mug in half the envs via the 16-object pool): 30 calls with persistent manifolds
    refresh many pairs, stay finite and keep every object inside the tote like the run without them."""
    n = 8
    scene = HM.load_scene(HM.BIN_ASSET)
    model = HM.build_model(scene)
    params, _ = HM.build_params({"n_objects": 8})
    st = HostState(n, model=model, params=params)
    scenes.fill_bin_scene(st, n, scene, seed=2)
    out = {}
    for on in (True, False):
        p, _ = HM.build_params({"n_objects": 8, **({} if on else {"pcm_lin_tol": 0.0})})
        s = st.copy()
        Oracle(model, p, n).simulate(s, 30)
        out[on] = s
    cs = out[True]["contact_stats"]
    assert cs[:, 5].sum() > 0.1 * (cs[:, 5].sum() + cs[:, 6].sum())      # the objects are still settling
    lo, hi = np.array(scene["bin_extent"][0]), np.array(scene["bin_extent"][1])
    for on in (True, False):
        r = out[on]["root_state"].reshape(n, 12, 13)[:, 4:]
        assert np.isfinite(r).all()
        inside = ((r[..., 0:2] > lo[0:2] - 0.02) & (r[..., 0:2] < hi[0:2] + 0.02)).all(-1)
        assert inside.mean() > 0.95, (on, inside.mean())
