"""The broad phase's box cull (ha_physics.h pair_boxes_near) on the CPU: a numpy restatement of its test, checked for
exactness against the C oracle's narrow phase (which has no such cull). Every link hull and every one-piece pool
object's hull lies inside its ha_model_t.hull_obb box (ha_create refuses a model where one does not), and in settled
and in-hand scenes of the Allegro, Kuka and bin families no object-link or object-object pair the cull declares apart has
a contact in the oracle's list. The kernels skip such pairs; their outputs stay bit-identical to the oracle (the GPU
suite)."""
import numpy as np
import pytest

from handarm_hip import model as HM
from oracle.oracle_lib import HostState, Oracle
from tests import scenes


def _qrot(q, v):
    u, w = q[:3], q[3]
    t = 2.0 * np.cross(u, v)
    return v + w * t + np.cross(u, t)


def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def _qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def boxes_near(ca, qa, ha, cb, qb, hb, lim):
    """pair_boxes_near's 15-axis test: B's box in A's box frame, |R_ij| + 1e-6, unnormalised edge axes."""
    qi = np.array([-qa[0], -qa[1], -qa[2], qa[3]])
    t = _qrot(qi, cb - ca)
    R = _qmat(_qmul(qi, qb))
    AR = np.abs(R) + 1e-6
    for i in range(3):
        if abs(t[i]) > ha[i] + hb @ AR[i] + lim:
            return False
    for j in range(3):
        if abs(t @ R[:, j]) > ha @ AR[:, j] + hb[j] + lim:
            return False
    for i in range(3):
        i1, i2 = (i + 1) % 3, (i + 2) % 3
        for j in range(3):
            j1, j2 = (j + 1) % 3, (j + 2) % 3
            ra = ha[i1] * AR[i2, j] + ha[i2] * AR[i1, j]
            rb = hb[j1] * AR[i, j2] + hb[j2] * AR[i, j1]
            if abs(t[i2] * R[i1, j] - t[i1] * R[i2, j]) > ra + rb + lim:
                return False
    return True


def _hull_verts(m, h):
    return np.array([list(m.verts[m.hull_vert_start[h] + i])[:3] for i in range(m.hull_nverts[h])], np.float64)


@pytest.mark.parametrize("asset", [HM.ASSET, HM.BIN_ASSET, HM.ALLEGRO_ASSET, HM.KUKA_ASSET])
def test_every_culled_hull_lies_inside_its_box(asset):
    """hull_obb boxes (link hulls: fitted, model.py hull_obb; one-piece pool objects: the body-frame bounding box,
    model.py object_box) contain their hulls' vertices - the condition ha_create checks."""
    m = HM.build_model(HM.load_scene(asset))
    boxed = list(range(m.n_link_hulls)) + [m.pool_hull[p] for p in range(m.n_pool) if m.pool_nhull[p] == 1]
    assert len(boxed) > m.n_link_hulls
    for h in boxed:
        ob = np.array(m.hull_obb[h], np.float64)
        R = _qmat(ob[6:10])
        loc = (_hull_verts(m, h) - ob[0:3]) @ R
        assert (np.abs(loc) <= ob[3:6] + 1e-7).all(), h
        if h >= m.n_link_hulls:
            assert list(ob[6:10]) == [0, 0, 0, 1]        # identity: a per-env object scale scales the box


@pytest.mark.parametrize("asset,pool", [(HM.ASSET, HM.POOL_WIDE), (HM.BIN_ASSET, None)])
def test_compound_pieces_lie_inside_their_boxes(asset, pool):
    """Round 6: every piece of a compound object (the mug; the wide pool's concave objects) carries a fitted box
    (model.py hull_obb) that holds its vertices: the piece-pair cull (ha_physics.h piece_mask / piece_boxes_near, the
    oracle's piece_boxes_near) tests those boxes, and ha_create refuses a model whose pieces leave them."""
    m = HM.build_model(HM.load_scene(asset), pool)
    pieces = [m.pool_hull[p] + j for p in range(m.n_pool) if m.pool_nhull[p] > 1 for j in range(m.pool_nhull[p])]
    assert len(pieces) >= (40 if pool else 2)
    for h in pieces:
        ob = np.array(m.hull_obb[h], np.float64)
        assert abs(np.linalg.norm(ob[6:10]) - 1.0) < 1e-6
        loc = (_hull_verts(m, h) - ob[0:3]) @ _qmat(ob[6:10])
        assert (np.abs(loc) <= ob[3:6] + 1e-7).all(), h


def test_piece_pair_box_test_is_the_double_precision_sat():
    """include/ha_obb.h ha_obb_pair_near (the compound piece-pair cull of kernel and oracle, built in box A's frame from
    the relative quaternion) against boxes_near in float64 on posed pieces of the wide pool: every pair it declares
    apart is apart in float64 by more than the margin less 1e-5 m, and every pair it keeps is within the margin plus
    1e-5 m, so it decides as the exact test does up to float32 rounding."""
    import ctypes as C
    from oracle.oracle_lib import load
    lib = load()
    f3 = C.POINTER(C.c_float)
    lib.hao_obb_pair_near.argtypes = [f3] * 6 + [C.c_float]
    m = HM.build_model(HM.load_scene(HM.ASSET), HM.POOL_WIDE)
    pieces = [m.pool_hull[p] + j for p in range(m.n_pool) if m.pool_nhull[p] > 1 for j in range(m.pool_nhull[p])]
    rng = np.random.default_rng(7)
    mg = 0.01
    kept = apart = 0

    def ptr(a):
        return np.ascontiguousarray(a, np.float32).ctypes.data_as(f3)

    def posed(p, q, ob):
        return p + _qrot(q, ob[0:3]), _qmul(q, ob[6:10]), ob[3:6]
    for _ in range(3000):
        h1, h2 = rng.choice(pieces, 2)
        p1 = rng.normal(0, 0.02, 3).astype(np.float32)
        p2 = (p1 + rng.normal(0, 0.05, 3)).astype(np.float32)
        q1, q2 = (q / np.linalg.norm(q) for q in rng.normal(size=(2, 4)))
        q1, q2 = q1.astype(np.float32), q2.astype(np.float32)
        ob1, ob2 = np.array(m.hull_obb[h1], np.float32), np.array(m.hull_obb[h2], np.float32)
        got = lib.hao_obb_pair_near(ptr(p1), ptr(q1), ptr(ob1), ptr(p2), ptr(q2), ptr(ob2), mg)
        a = posed(p1.astype(np.float64), q1.astype(np.float64), ob1.astype(np.float64))
        b = posed(p2.astype(np.float64), q2.astype(np.float64), ob2.astype(np.float64))
        if got:
            kept += 1
            assert boxes_near(*a, *b, mg + 1e-5)
        else:
            apart += 1
            assert not boxes_near(*a, *b, mg - 1e-5)
    assert kept > 300 and apart > 300


def _object_box(m, st, e, o, n_obj):
    A = m.n_actors
    root = st["root_state"].reshape(-1, A, 13)[e, m.actor_object0 + o]
    pool = int(st["object_indices"].reshape(-1, n_obj)[e, o])
    h = m.pool_hull[pool]
    if m.pool_nhull[pool] != 1:
        return None
    scaled = "object_scale" not in st.null
    sc = st["object_scale"].reshape(st.num_envs, n_obj, 3)[e, o].astype(np.float64) if scaled else np.ones(3)
    ob = np.array(m.hull_obb[h], np.float64)
    q = root[3:7].astype(np.float64)
    com = np.array(m.pool_com[pool]) * sc
    p = root[0:3] - _qrot(q, com)
    return p + _qrot(q, ob[0:3] * sc), q, ob[3:6] * sc


def _link_box(m, st, e, h):
    B = m.n_bodies
    L = m.hull_link[h]
    rb = st["rigid_body_state"].reshape(-1, B, 13)[e, m.body_robot0 + L]
    ob = np.array(m.hull_obb[h], np.float64)
    q = rb[3:7].astype(np.float64)
    return rb[0:3] + _qrot(q, ob[0:3]), _qmul(q, ob[6:10]), ob[3:6]


def _check_scene(m, params, st, n, n_obj):
    """every (object, link) / (object, object) pair the box test declares apart has no oracle contact"""
    orc = Oracle(m, params, n)
    mg = params.contact_margin
    culled = touching_culled = 0
    for e in range(n):
        rows = orc.contacts(st, e)
        bodies = {(int(min(r[7], r[8])), int(max(r[7], r[8]))) for r in rows}
        for o in range(n_obj):
            box = _object_box(m, st, e, o, n_obj)
            if box is None:
                continue
            links = {}
            for h in range(m.n_link_hulls):
                near = boxes_near(*box, *_link_box(m, st, e, h), mg + 1e-3)
                L = m.hull_link[h]
                links[L] = links.get(L, False) or near
            for L, near in links.items():
                if not near:
                    culled += 1
                    touching_culled += (o, 100 + L) in bodies
            for o2 in range(o + 1, n_obj):
                box2 = _object_box(m, st, e, o2, n_obj)
                if box2 is not None and not boxes_near(*box, *box2, mg + 1e-3):
                    culled += 1
                    touching_culled += (o, o2) in bodies
    assert touching_culled == 0
    return culled


def test_allegro_in_hand_pairs_the_cull_skips_have_no_contacts():
    from tests.test_allegro_physics import setup
    n = 16
    m, params, st, lo, up = setup(n)
    rng = np.random.default_rng(3)
    orc = Oracle(m, params, n)
    culled = 0
    for k in range(4):
        st["sim_targets"][:] = rng.uniform(lo, up, (n, 16)).astype(np.float32)
        orc.simulate(st, 6)
        culled += _check_scene(m, params, st, n, 1)
    assert culled > 0


def test_kuka_and_bin_pairs_the_cull_skips_have_no_contacts():
    from tests.test_kuka_physics import setup as kuka_setup
    n = 8
    scene, m, params, st, scales, lo, up = kuka_setup(n)
    Oracle(m, params, n).simulate(st, 10)
    c1 = _check_scene(m, params, st, n, 1)
    scene = HM.load_scene(HM.BIN_ASSET)
    m = HM.build_model(scene)
    params, _ = HM.build_params({"n_objects": 8})
    st = HostState(n, model=m, params=params)
    scenes.fill_bin_scene(st, n, scene, seed=1)
    Oracle(m, params, n).simulate(st, 20)
    c2 = _check_scene(m, params, st, n, 8)
    assert c1 > 0 and c2 > 0
