"""Narrow phase completeness on the C oracle (CPU): edge-edge separating axes and clipped face manifolds
(handarm_abi.h v10). PhysX's convex-convex test, which the reference relies on for every object
(V-HACD pieces, multi_object.py:37-43; the AllegroKuka cuboids, allegro_kuka_base.py:508-542), finds edge-edge
contacts and clips overhanging faces; these scenes fail without them.

The GPU is bit-identical to the oracle on the same scenes (tests/test_gpu_edges.py)."""
import numpy as np
import pytest

from handarm_hip import model as HM
from oracle.oracle_lib import HostState, Oracle
from tests import scenes


def _setup(kind, n=4, **cfg):
    scene = scenes.box_pool_scene(scenes.EDGE_BOXES)
    m = HM.build_model(scene)
    p, _ = HM.build_params(cfg or None)
    st = HostState(n, model=m, params=p)
    scenes.fill_box_scene(st, n, kind)
    return scene, m, p, st, Oracle(m, p, n)


def _pair(c, a, b):
    return c[((c[:, 7] == a) & (c[:, 8] == b)) | ((c[:, 7] == b) & (c[:, 8] == a))]


def quat_mat(q):
    x, y, z, w = (float(t) for t in q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def world_hull(hull, pose):
    R = quat_mat(pose[3:7])
    v = np.asarray(hull["verts"], np.float64) @ R.T + np.asarray(pose[0:3], np.float64)
    n = np.asarray(hull["planes"], np.float64)[:, :3] @ R.T
    edges, _ = HM.hull_topology(hull["verts"], hull["planes"])
    e = np.array([v[b] - v[a] for a, b, _, _ in edges])
    return v, n, e


def separation(A, B):
    """Exact separation of two convex polytopes (negative: penetration depth) by brute-force SAT over both hulls'
    face normals and every edge-pair cross product: an independent check of the simulator's contacts."""
    (va, na, ea), (vb, nb, eb) = A, B
    axes = [na, nb]
    cr = np.cross(ea[:, None, :], eb[None, :, :]).reshape(-1, 3)
    ln = np.linalg.norm(cr, axis=1)
    axes.append(cr[ln > 1e-9] / ln[ln > 1e-9, None])
    ax = np.concatenate(axes)
    pa, pb = va @ ax.T, vb @ ax.T
    return float(np.maximum(pa.min(0) - pb.max(0), pb.min(0) - pa.max(0)).max())


def test_hull_topology_of_every_scene_hull():
    """Every hull of every scene: face loops of 3..HA_MAX_FACE_LOOP vertices on their planes, each edge between two
    distinct faces with both ends on both planes, boxes with 12 edges and 6 quads."""
    for path in (HM.ASSET, HM.ALLEGRO_ASSET, HM.KUKA_ASSET, HM.BIN_ASSET):
        sc = HM.load_scene(path)
        hulls = list(sc["link_hulls"]) + [h for o in sc["objects"] for h in (o.get("hulls") or [o["hull"]])]
        hulls += [s["hull"] for s in ([sc["table"]] if sc.get("table") else []) + list(sc.get("statics", []))]
        for h in hulls:
            v = np.asarray(h["verts"], np.float64)
            P = np.asarray(h["planes"], np.float64)
            edges, loops = HM.hull_topology(v, P)
            assert len(loops) == len(P)
            for k, loop in enumerate(loops):
                assert 3 <= len(loop) <= HM.MAX_FACE_LOOP
                idx = [a for a, _ in loop]
                assert np.abs(v[idx] @ P[k, :3] + P[k, 3]).max() < 1e-6
            assert len(edges) <= 4 * (32 if path in (HM.ALLEGRO_ASSET, HM.KUKA_ASSET) else 64)
            for a, b, f0, f1 in edges:
                assert f0 != f1 and P[f0, :3] @ P[f1, :3] < 1 - 1e-6
    e, l = HM.hull_topology(scenes.box_hull_record((0.1, 0.2, 0.3))["verts"],
                            scenes.box_hull_record((0.1, 0.2, 0.3))["planes"])
    assert len(e) == 12 and [len(x) for x in l] == [4] * 6


def test_crossed_boxes_edge_edge_contact():
    """Two boxes whose ridges cross at 90 deg, 0.25-0.75 mm into each other: one contact at the crossing with the
    edge-edge axis as normal (+z, from box 1 to box 0) and the penetration as separation. No face axis finds it:
    with the edge axes disabled the pair has no contact at all."""
    n = 4
    _, m, p, st, orc = _setup("crossed", n)
    rs = st["root_state"].reshape(n, 6, 13)
    for e in range(n):
        c = _pair(orc.contacts(st, e), 0, 1)
        assert len(c) == 1
        np.testing.assert_allclose(c[0, 3:6] * np.sign(c[0, 7] - c[0, 8] + 0.5) * -1, [0, 0, 1], atol=1e-5)
        assert -0.0008 < c[0, 6] < -0.0002
        np.testing.assert_allclose(c[0, 0:2], rs[e, 4, 0:2], atol=1e-4)       # above box 1's centre line
    _, _, _, st2, orc2 = _setup("crossed", n, edge_abs_tol=1e9)
    assert all(len(_pair(orc2.contacts(st2, e), 0, 1)) == 0 for e in range(n))


def test_overhang_manifold_reaches_table_edge():
    """A box 37.5% over the table's far edge: its manifold holds the two corners on the table and the two points
    where its bottom edges cross the table edge (the clipped face), so the support polygon covers its centre."""
    n = 4
    _, m, p, st, orc = _setup("overhang", n)
    rs = st["root_state"].reshape(n, 6, 13)
    for e in range(n):
        c = _pair(orc.contacts(st, e), 2, -1)
        assert len(c) == 4
        on_edge = np.abs(c[:, 0] - scenes.TABLE_X1) < 1e-4
        assert on_edge.sum() == 2
        assert c[:, 0].min() < rs[e, 5, 0] < c[:, 0].max()


def test_overhanging_box_stays_on_table():
    """Physical: the overhanging box rests on the table for 120 env-steps (it would tip over the edge with vertex-only
    contacts, whose support line is its inner edge)."""
    n = 2
    scene, m, p, st, orc = _setup("overhang", n)
    for _ in range(120):
        orc.simulate(st, 3)
    rs = st["root_state"].reshape(n, 6, 13)
    assert np.isfinite(rs).all()
    np.testing.assert_allclose(rs[:, 5, 2], scenes.TABLE_TOP + scenes.EDGE_BOXES[2][2], atol=2e-3)
    up = np.array([quat_mat(q)[:, 2] for q in rs[:, 5, 3:7]])
    assert (up[:, 2] > np.cos(np.radians(3))).all()
    assert np.abs(rs[:, 5, 7:13]).max() < 0.05


def _penetration_run(kind, n=4, steps=120, **cfg):
    """(worst transient, settled) separation over `steps` env-steps, min over envs and over the pairs box 0 -
    table, box 1 - table, box 0 - box 1, by the exact polytope SAT (independent of the simulator's contacts)."""
    scene, m, p, st, orc = _setup(kind, n, **cfg)
    tab = scene["table"]
    table = world_hull(tab["hull"], list(tab["pos"]) + list(tab["quat"]))
    boxes = [o["hull"] for o in scene["objects"]]
    worst, final = 0.0, 0.0
    for step in range(steps):
        orc.simulate(st, 3)
        rs = st["root_state"].reshape(n, 6, 13).astype(np.float64)
        sep = []
        for e in range(n):
            w = [world_hull(boxes[i], rs[e, 3 + i, 0:7]) for i in range(3)]
            sep.append(min(separation(w[0], table), separation(w[1], table), separation(w[0], w[1])))
        worst = min(worst, min(sep))
        final = min(sep)
    assert np.isfinite(st["root_state"]).all()
    return worst, final, p


@pytest.mark.parametrize("kind", ["crossed", "table_edge"])
def test_no_interpenetration_after_120_steps(kind):
    """Physical: boxes touching through edges (ridges crossed on each other, a ridge tipping over the table's edge)
    end 120 env-steps interpenetrating by no more than contact_slop (+0.5 mm of resting load), and never pass through
    each other on the way (transient impacts stay < 6 mm; without the edge-edge axes the crossed boxes sink > 30 mm
    into each other)."""
    worst, final, p = _penetration_run(kind)
    assert final > -(p.contact_slop + 5e-4), f"settled penetration {-final * 1e3:.2f} mm"
    assert worst > -6e-3, f"transient penetration {-worst * 1e3:.2f} mm"
    if kind == "crossed":
        worst_off, _, _ = _penetration_run(kind, n=2, steps=30, edge_abs_tol=1e9)
        assert worst_off < -0.02     # the scene does need the edge axes
