"""Overflow contact chunks (PhysCfg OVF) on the GPU, against the C oracle at the same capacity.

The Ur5Sih (3 objects) and AllegroHand families hold chunk 0 of their contact list in LDS (21 / 12 contacts, the
round-3 layout) and chunks 1..3 in the env's global area (contact entries, constraint rows, PGS row constants), so
a substep keeps up to 84 / 48 contacts instead of dropping the shallowest (PhysX sizes its contact buffer per scene,
ur5sih.py:129-155, AllegroHand.yaml:161-179). These scenes offer more contacts than chunk 0 holds in most envs;
every physics output stays bit-identical to the oracle, and no substep is over the capacity."""
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


def push(sim, st):
    for k in HM.STATE_FIELDS:
        if k in ("stats", "term_sums") or k in HM.null_fields(sim.task):
            continue
        put(sim, k, st[k])


@pytest.mark.parametrize("calls", [1, 4])
def test_ur5sih_pile_in_the_hand_overflows_chunk0_and_matches_oracle(calls):
    """The three objects dropped together into the closed hand just above the table: object-object, object-table and
    many link-object pairs at once."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    n = 64
    sim = HandArmSim(n, "cuda:0")
    assert sim.contact_capacity == 84
    st = HostState(n)
    scenes.fill_scene(st, n, seed=13, near_hand=0.0)
    probe = st.copy()
    Oracle(sim.model, sim.params, n).simulate(probe, 1)
    body = probe["rigid_body_state"].reshape(n, 34, 13)
    rng = np.random.default_rng(13)
    hull_links = sorted({int(sim.model.hull_link[k]) for k in range(sim.model.n_link_hulls)})
    rs = st["root_state"].reshape(n, 6, 13)
    for o in range(3):
        lk = np.array(hull_links)[rng.integers(len(hull_links) // 2, len(hull_links), n)]
        rs[:, 3 + o, 0:3] = body[np.arange(n), sim.model.body_robot0 + lk, 0:3] + rng.uniform(-0.015, 0.015, (n, 3))
        rs[:, 3 + o, 7:13] = 0.0
    push(sim, st)
    sim.t["contact_stats"].zero_()
    sim.simulate(calls)
    Oracle(sim.model, sim.params, n).simulate(st, calls)
    cs = get(sim, "contact_stats")
    over21 = (cs[:, 2] > 21).mean()
    print(f"ur5sih pile: envs offering > 21 contacts in a substep {over21:.2f}, max offered {cs[:, 2].max()}, "
          f"over capacity {cs[:, 1].sum()} of {cs[:, 0].sum()} substeps")
    assert over21 >= 0.25, "the scene must overflow chunk 0 (21 contacts) in many envs"
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"ur5sih overflow calls {calls}")


@pytest.mark.parametrize("seed,calls", [(0, 1), (3, 4)])
def test_allegro_cube_in_the_closing_hand_overflows_chunk0_and_matches_oracle(seed, calls):
    """Fingers at random joint positions around the cube on the palm: finger-cube contacts beyond chunk 0's 12."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    n = 128
    sim = HandArmSim(n, "cuda:0", task=HM.TASK_ALLEGRO_HAND)
    assert sim.contact_capacity == 48
    lo = np.array(sim.model.dof_lower[:16], np.float32)
    up = np.array(sim.model.dof_upper[:16], np.float32)
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_allegro_scene(st, n, lo, up, seed=seed)
    # every finger closing onto the cube: targets at the upper limits
    st["sim_targets"][:] = up
    push(sim, st)
    sim.t["contact_stats"].zero_()
    sim.simulate(calls)
    Oracle(sim.model, sim.params, n).simulate(st, calls)
    cs = get(sim, "contact_stats")
    over12 = (cs[:, 2] > 12).mean()
    print(f"allegro closing hand: envs offering > 12 contacts {over12:.2f}, max offered {cs[:, 2].max()}, "
          f"over capacity {cs[:, 1].sum()} of {cs[:, 0].sum()} substeps")
    assert over12 >= 0.1, "the scene must overflow chunk 0 (12 contacts) in some envs"
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"allegro overflow seed {seed} calls {calls}")


@pytest.mark.parametrize("calls", [1, 4])
def test_kuka_closed_hand_overflows_chunk0_and_matches_oracle(calls):
    """AllegroKuka (ak_simulate_kernel): chunk 0 holds 21 contacts in LDS, chunk 1 (21 more) sits in the env's global
    area. The half-closed hand closing further on the cuboid in its palm offers more than 21 contacts per substep in
    most envs (cube-finger, cube-palm and the hand's self-collision contacts); every physics output and the persistent
    manifolds stay bit-identical to the oracle at the same capacity, and the contact statistics match."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    from tests.test_gpu_fused_steps import kuka_closed_hand_scene
    n = 128
    sim = HandArmSim(n, "cuda:0", task=HM.TASK_ALLEGRO_KUKA)
    assert sim.contact_capacity == 42
    lo = np.array(sim.model.dof_lower[:23], np.float32)
    up = np.array(sim.model.dof_upper[:23], np.float32)
    st = HostState(n, model=sim.model, params=sim.params)
    st["object_scale"][:] = sim.t["object_scale"].cpu().numpy()
    kuka_closed_hand_scene(sim, st, lo, up)
    st["contact_stats"][:] = 0
    push(sim, st)
    sim.simulate(calls)
    Oracle(sim.model, sim.params, n).simulate(st, calls)
    cs = get(sim, "contact_stats")
    over21 = (cs[:, 2] > 21).mean()
    print(f"kuka closed hand: envs offering > 21 contacts {over21:.2f}, max offered {cs[:, 2].max()}, self contacts "
          f"{cs[:, 4].sum()}, refreshed {cs[:, 5].sum()}, over capacity {cs[:, 1].sum()} of {cs[:, 0].sum()} substeps")
    assert over21 >= 0.25, "the scene must overflow chunk 0 (21 contacts) in many envs"
    assert (cs[:, 4] > 0).mean() >= 0.9, "self-collision contacts in (nearly) every env"
    assert (cs[:, :6] == st["contact_stats"][:, :6]).all(), "contact statistics differ from the oracle's"
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"kuka overflow calls {calls}")
