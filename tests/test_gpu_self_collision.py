"""Self-collision of the Allegro actors on the GPU (ah_* / ak_* kernels, ha_model_t v12 self pairs): the finger-finger
and thumb-palm drives of tests/self_collision_scenes.py for 120 gym.simulate calls, jittered per env. Every physics
output is bit-identical to the C oracle, and the GPU's final states hold no link-link interpenetration beyond
contact_slop (measured with the oracle's contact generation)."""
import numpy as np
import pytest
import torch

from handarm_hip import model as HM
from tests import scenes
from tests import self_collision_scenes as SC

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("task", [HM.TASK_ALLEGRO_HAND, HM.TASK_ALLEGRO_KUKA])
def test_self_collision_drives_on_the_gpu(task):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    n = 32
    sim = HandArmSim(n, "cuda:0", task=task)
    m, p = sim.model, sim.params
    assert m.n_self_pairs > 0
    D = m.n_dofs
    lo, up = np.array(m.dof_lower[:D], np.float32), np.array(m.dof_upper[:D], np.float32)
    drives = SC.allegro_drives(lo, up) if task == HM.TASK_ALLEGRO_HAND else SC.kuka_drives(lo, up, list(p.reset_pose))
    names = list(drives)
    rng = np.random.default_rng(5)
    targets = np.stack([drives[names[e % len(names)]] for e in range(n)])
    targets = np.clip(targets + rng.uniform(-0.05, 0.05, targets.shape).astype(np.float32), lo, up)
    st = SC.drive_state(HostState(n, model=m, params=p), m, targets, n)
    for k in HM.STATE_FIELDS:
        if k in ("stats", "term_sums", "task_state", "task_scalars") or k in HM.null_fields(task):
            continue
        sim.t[k].copy_(torch.as_tensor(st[k]).reshape(sim.t[k].shape).to(sim.t[k].dtype))
    sim.simulate(120)
    orc = Oracle(m, p, n)
    orc.simulate(st, 120)
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"self collision {task}")
    gpu = st.copy()
    for k in ("dof_state", "root_state"):
        gpu[k][...] = sim.t[k].cpu().numpy().reshape(gpu[k].shape)
    seps = np.array([SC.min_self_separation(orc, gpu, e) for e in range(n)])
    print(f"task {task}: deepest link-link separation per drive "
          f"{[float(seps[i::len(names)].min()) for i in range(len(names))]}")
    assert seps.min() >= -(p.contact_slop + 5e-4)
    assert (seps < 0).sum() >= n // 4, "the drives must press links together"
