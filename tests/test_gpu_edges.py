"""GPU parity of the completed narrow phase (handarm_abi.h v10: edge-edge SAT axes, clipped face manifolds) against
the C oracle, through the C ABI, on scenes that need it (tests/test_edge_contacts.py checks them physically on the
oracle): bit-identical physics on every env after 1 and 10 gym.simulate calls."""
import numpy as np
import pytest
import torch

from handarm_hip import model as HM
from tests import scenes

pytestmark = pytest.mark.gpu


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def get(sim, name):
    torch.cuda.synchronize()
    return sim.t[name].cpu().numpy()


def _box_sim(kind, n):
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    scene = scenes.box_pool_scene(scenes.EDGE_BOXES)
    sim = HandArmSim(n, "cuda:0", scene=scene)
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_box_scene(st, n, kind, seed=3)
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums"):
            put(sim, k, st[k])
    return sim, Oracle(sim.model, sim.params, n), st


@pytest.mark.parametrize("kind,calls", [("crossed", 1), ("crossed", 10), ("table_edge", 10), ("overhang", 10)])
def test_edge_scenes_match_oracle_bit_for_bit(kind, calls):
    """Crossed ridges (edge-edge axis contact), a ridge across the table edge and a box overhanging it (clipped
    manifolds): every physics output bit-identical to the oracle."""
    n = 64
    sim, orc, st = _box_sim(kind, n)
    sim.simulate(calls)
    orc.simulate(st, calls)
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"{kind} calls {calls}")


def test_crossed_boxes_rest_without_interpenetration_on_gpu():
    """The crossed-ridge boxes after 120 env-steps on the HIP path: the exact polytope SAT of the final poses shows
    no interpenetration beyond contact_slop + 0.5 mm (the oracle-side test shows > 30 mm without edge axes)."""
    from tests.test_edge_contacts import separation, world_hull
    n = 64
    sim, orc, st = _box_sim("crossed", n)
    sim.simulate(360)
    rs = get(sim, "root_state").reshape(n, 6, 13).astype(np.float64)
    assert np.isfinite(rs).all()
    scene = sim.scene
    tab = scene["table"]
    table = world_hull(tab["hull"], list(tab["pos"]) + list(tab["quat"]))
    boxes = [o["hull"] for o in scene["objects"]]
    worst = 0.0
    for e in range(n):
        w = [world_hull(boxes[i], rs[e, 3 + i, 0:7]) for i in range(3)]
        worst = min(worst, separation(w[0], table), separation(w[1], table), separation(w[0], w[1]))
    assert worst > -(sim.params.contact_slop + 5e-4), f"penetration {-worst * 1e3:.2f} mm"


@pytest.mark.parametrize("calls", [1, 10])
def test_kuka_cuboid_edge_on_fingertip_matches_oracle(calls):
    """AllegroKuka (C2): each env's cuboid rests a ridge on the top of its highest fingertip link hull: the
    cuboid-link pair goes through the edge-edge axes and the clipped manifold, and the physics is bit-identical to
    the oracle."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    n = 64
    sim = HandArmSim(n, "cuda:0", task_cfg={"task": HM.TASK_ALLEGRO_KUKA}, task=HM.TASK_ALLEGRO_KUKA)
    m = sim.model
    lo = np.array(m.dof_lower[:23], np.float32)
    up = np.array(m.dof_upper[:23], np.float32)
    st = HostState(n, model=m, params=sim.params)
    scenes.fill_kuka_scene(st, n, lo, up, list(sim.params.reset_pose), get(sim, "object_scale"),
                           list(m.table_pos), seed=4)
    rs = st["root_state"].reshape(n, m.n_actors, 13)
    rs[:, m.actor_object0, 0:3] = [0.0, 0.0, 2.0]               # away while the link poses are computed
    probe = st.copy()
    Oracle(m, sim.params, n).simulate(probe, 1)
    for k in ("dof_state", "sim_targets"):
        st[k][:] = probe[k]
    tips = list(sim.params.ak_fingertip_links)
    body = probe["rigid_body_state"].reshape(n, m.n_bodies, 13)
    # each env's cuboid ridge goes on its highest fingertip (the most exposed one; the others sit under the palm)
    best = [tips[int(np.argmax([scenes.link_hull_world_verts(m, body[e], t)[:, 2].max() for t in tips]))]
            for e in range(n)]
    for t in tips:
        sel = [e for e in range(n) if best[e] == t]
        sub = st.copy()
        scenes.place_cuboid_edge_on_link(sub, m, probe["rigid_body_state"], t)
        rs[sel] = sub["root_state"].reshape(n, m.n_actors, 13)[sel]
    st["rigid_body_state"][:] = probe["rigid_body_state"]
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums", "task_state", "task_scalars"):
            put(sim, k, st[k])
    orc = Oracle(m, sim.params, n)
    # the scene offers ridge-on-fingertip contacts: the narrow phase finds a cuboid-tip pair in most envs (the
    # 5-20 cm cuboids also touch other links, which can crowd the tip out of the reduced manifold)
    hit = [any(int(r[7]) == 100 + best[e] for r in orc.contacts(st, e)) for e in range(n)]
    assert np.mean(hit) >= 0.85, np.mean(hit)
    sim.simulate(calls)
    orc.simulate(st, calls)
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"kuka cuboid edge on fingertip calls {calls}")
