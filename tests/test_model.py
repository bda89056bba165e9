"""Host model packing: DOF/body order, derived topology, spline tables."""
import numpy as np

from handarm_hip import model as HM
from oracle import task_oracle as O


def test_dof_order_matches_reference_conventions():
    scene = HM.load_scene()
    names = [d["name"] for d in scene["robot"]["dofs"]]
    assert names == O.DOF_NAMES
    assert names[14] == "thumb_opposition"        # Ur5SihBase.yaml:8-9 reset pose puts -1.571 here
    links = [l["name"] for l in scene["robot"]["links"]]
    assert len(links) == 29
    assert links[9] == "flange"
    assert [links[i] for i in (28, 15, 21, 24, 18)] == ["thumb_fingertip", "index_fingertip", "middle_fingertip",
                                                       "ring_fingertip", "little_fingertip"]


def test_topology():
    m = HM.build_model(HM.load_scene())
    assert m.n_dofs == 17 and m.n_links == 29
    lv = np.ctypeslib.as_array(m.link_level)[:m.n_links]
    par = np.ctypeslib.as_array(m.link_parent)[:m.n_links]
    assert lv[0] == 0 and all(lv[i] == lv[par[i]] + 1 for i in range(1, m.n_links))
    # 6 arm dofs: 21 ancestor pairs; 4 two-joint fingers: 4*(7+8); thumb 7+8+9
    assert m.n_mpairs == 21 + 4 * 15 + 24
    for k in range(m.n_link_hulls + m.n_pool + 1):
        assert 4 <= m.hull_nverts[k] <= 64 and 4 <= m.hull_nplanes[k] <= 128


def test_spline_tables_equal_oracle():
    p, _ = HM.build_params()
    sp = np.ctypeslib.as_array(p.spline)
    for i, name in enumerate(HM.SPLINE_ORDER):
        n = p.spline_pieces[i]
        np.testing.assert_array_equal(sp[i, :, :n], O.SPLINE_OBJS[name].table())


def test_mug_is_a_compound_of_convex_pieces():
    """f1: the non-convex pool object (025_mug; the reference V-HACDs every object, multi_object.py:37-43) is a set
    of convex pieces (tools/convex_decomp.py): the cavity and the handle gap are open, the pieces stay inside the
    pool bounding sphere, and every other pool object keeps one hull."""
    import numpy as np
    from handarm_hip import model as HM
    for asset in (HM.ASSET, HM.BIN_ASSET):
        m = HM.build_model(HM.load_scene(asset))
        names = [o["name"] for o in HM.load_scene(asset)["objects"]]
        mug = names.index("025_mug")
        assert m.pool_nhull[mug] >= 8
        # the other objects of the 16-object pool keep one hull; the concave ones of the wide pool are compounds
        assert all(m.pool_nhull[i] == 1 for i in range(m.n_pool) if i != mug and names[i] in HM.POOL16)
        assert all(m.pool_nhull[i] >= 4 for i in range(m.n_pool) if names[i] in HM.CONCAVE_POOL)
        assert names[:16] == HM.POOL16 and names[16:] == HM.CONCAVE_POOL
        assert m.n_hulls <= HM.MAX_HULLS and m.pool_hull[mug] + m.pool_nhull[mug] <= m.n_hulls
        pieces = range(m.pool_hull[mug], m.pool_hull[mug] + m.pool_nhull[mug])
        planes = np.ctypeslib.as_array(m.planes)

        def inside(x):
            for k in pieces:
                p = planes[m.hull_plane_start[k]:m.hull_plane_start[k] + m.hull_nplanes[k]]
                if np.all(p[:, :3] @ x + p[:, 3] <= 0):
                    return True
            return False
        verts = np.concatenate([np.ctypeslib.as_array(m.verts)[m.hull_vert_start[k]:m.hull_vert_start[k] + m.hull_nverts[k], :3]
                                for k in pieces])
        c = np.array(m.pool_center[mug][:])
        assert np.linalg.norm(verts - c, axis=1).max() <= m.pool_radius[mug]
        # the mug's axis is z; its cavity (centre column, above the base) is empty space, the wall is not
        lo, hi = verts.min(0), verts.max(0)
        axis = np.array([verts[:, 0].min() + 0.046, 0.5 * (lo[1] + hi[1])])
        assert not inside(np.array([axis[0], axis[1], 0.5 * (lo[2] + hi[2])]))
        assert not inside(np.array([axis[0], axis[1], hi[2] - 0.01]))
        assert inside(np.array([axis[0], axis[1], lo[2] + 0.002]))        # the base slab
