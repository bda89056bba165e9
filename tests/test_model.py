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
