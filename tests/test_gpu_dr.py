"""Domain randomization on the GPU through the C ABI (Ur5Sih family, BASELINE config 4 "DR on"):
* physics reading per-env rows (mass, friction, DOF stiffness / damping / limits, object scale) and the shard's
  randomized gravity matches the C oracle reading the same rows bit for bit;
* the reset launch's first randomization samples every env's row on the device, bit-identical to
  oracle/dr_oracle.py, within the configured ranges (friction on get_bucketed_val's 250-bucket grid);
* the step kernel adds N(0, 0.002) observation noise to obs only (teacher obs untouched).
The reference's Ur5Sih DR flag has no consumer, so config 4's schema is the build's own
(handarm_hip/dr.py UR5SIH_SCHEMA); the engine is the one AllegroKuka's schema runs (tests/test_gpu_dr_schema.py)."""
import numpy as np
import pytest
import torch

from handarm_hip import model as HM
from tests import scenes
from tests.test_gpu_parity import get, make_sim, put

pytestmark = pytest.mark.gpu


def _dr_rows(n, rng, model=None, params=None, scale=False):
    """Nominal rows (handarm_hip/dr.py default_rows) with random link / object masses and frictions, DOF stiffness /
    damping x U[0.5, 2], limits +- N(0, 0.01), and (scale) object scales U[0.8, 1.2]."""
    from handarm_hip import dr as DR
    if model is None:
        model = HM.build_model(HM.load_scene())
    if params is None:
        params, _ = HM.build_params({"dr_enable": 1})
    dr = DR.default_rows(model, params, n)
    dr[:, HM.DR_LINK_MASS:HM.DR_LINK_MASS + HM.MAX_LINKS] = rng.uniform(0.5, 1.5, (n, HM.MAX_LINKS))
    dr[:, HM.DR_OBJ_MASS:HM.DR_OBJ_MASS + HM.MAX_OBJ] = rng.uniform(0.5, 1.5, (n, HM.MAX_OBJ))
    dr[:, HM.DR_LINK_FRIC:HM.DR_LINK_FRIC + HM.MAX_LINKS] = rng.uniform(0.7, 1.3, (n, HM.MAX_LINKS))
    dr[:, HM.DR_OBJ_FRIC:HM.DR_OBJ_FRIC + HM.MAX_OBJ] = rng.uniform(0.7, 1.3, (n, HM.MAX_OBJ))
    for k in (HM.DR_DOF_KP, HM.DR_DOF_KD):
        dr[:, k:k + HM.MAX_DOFS] *= rng.uniform(0.5, 2.0, (n, HM.MAX_DOFS)).astype(np.float32)
    for k in (HM.DR_DOF_LOWER, HM.DR_DOF_UPPER):
        dr[:, k:k + HM.MAX_DOFS] += rng.normal(0, 0.01, (n, HM.MAX_DOFS)).astype(np.float32)
    if scale:
        dr[:, HM.DR_OBJ_SCALE:HM.DR_OBJ_SCALE + HM.MAX_OBJ] = rng.uniform(0.8, 1.2, (n, HM.MAX_OBJ))
    return dr


def test_dr_physics_matches_oracle():
    from oracle.oracle_lib import HostState, Oracle
    n = 128
    sim = make_sim(n, dr_enable=1)
    orc = Oracle(sim.model, sim.params, n)
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_scene(st, n, seed=5, near_hand=0.0)
    st["dr_scale"][:] = _dr_rows(n, np.random.default_rng(0), sim.model, sim.params, scale=True)
    st["dr_global"][HM.DRG_GRAVITY:HM.DRG_GRAVITY + 3] = [0.3, -0.2, -9.5]          # a randomized gravity
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums"):
            put(sim, k, st[k])
    sim.simulate(1)
    orc.simulate(st, 1)
    scenes.assert_physics_bit_identical(sim, st, n, tag="DR rows")
    # heavier objects really are heavier: the resting contact force scales with the sampled mass
    sim2 = make_sim(n, dr_enable=1)
    rows = _dr_rows(n, np.random.default_rng(1), sim.model, sim.params)
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums", "dr_global"):          # sim2 keeps its own (nominal gravity)
            put(sim2, k, rows if k == "dr_scale" else st[k])
    sim2.simulate(60)
    f = get(sim2, "net_contact_force").reshape(n, 34, 3)[:, 31:34, 2]
    mass = np.array([sim2.model.pool_mass[i] for i in range(3)])[get(sim2, "object_indices")]
    scale = get(sim2, "dr_scale")[:, HM.DR_OBJ_MASS:HM.DR_OBJ_MASS + 3]
    np.testing.assert_allclose(np.median(f / (9.81 * mass * scale)), 1.0, rtol=0.15)


def test_dr_sampled_at_reset_matches_oracle_and_ranges():
    """The reset launch's first randomization (every env, vec_task.py:663-665) on the device vs oracle/dr_oracle.py."""
    from oracle import dr_oracle as DO
    n = 512
    sim = make_sim(n, dr_enable=1)
    sim.t["reset_buf"].fill_(1)
    sim.t["episode"].copy_(torch.arange(n, dtype=torch.int32) * 7)
    g0 = get(sim, "dr_global").copy()
    rows0 = get(sim, "dr_scale").copy()
    rb0 = get(sim, "randomize_buf").copy()
    sim.task_reset(HM.FLAG_NO_PHYSICS)
    dr = get(sim, "dr_scale")
    # the oracle: the shard-wide update (Ur5Sih's reset launch resets every env), then every env samples
    g = DO.global_update(sim.params, g0, True, 1)
    assert (get(sim, "dr_global").view(np.int32) == g.view(np.int32)).all()
    pools = get(sim, "object_indices")
    DO.env_pre(sim.params, sim.model, rows0, rb0, np.arange(n, dtype=np.uint32) * 7, pools, np.ones(n, bool), g, False)
    np.testing.assert_array_equal(dr, rows0)
    np.testing.assert_array_equal(get(sim, "randomize_buf"), rb0)
    lm = dr[:, HM.DR_LINK_MASS:HM.DR_LINK_MASS + sim.model.n_links]
    om = dr[:, HM.DR_OBJ_MASS:HM.DR_OBJ_MASS + 3]
    lf = dr[:, HM.DR_LINK_FRIC:HM.DR_LINK_FRIC + sim.model.n_links]
    assert lm.min() >= 0.5 and lm.max() <= 1.5 and abs(lm.mean() - 1.0) < 0.01
    assert om.min() >= 0.5 and om.max() <= 1.5 and om.std() > 0.2
    assert lf.min() >= 0.7 - 1e-6 and lf.max() < 1.3
    grid = (lf - 0.7) / (0.6 / 250)                      # bucket index: integral
    assert np.abs(grid - np.round(grid)).max() < 1e-3
    assert len(np.unique(lm[:, 0])) > n // 2             # independent per env


def test_dr_observation_noise():
    from oracle.oracle_lib import HostState
    n = 2048
    sim = make_sim(n, dr_enable=1)
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_scene(st, n, seed=3)
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums", "dr_scale", "dr_global"):
            put(sim, k, st[k])
    sim.t["reset_buf"][:8] = 1                    # an env reset: the first randomization sets the noise parameters
    sim.task_step(HM.FLAG_NO_PHYSICS)
    d = get(sim, "obs") - get(sim, "teacher_obs")
    assert abs(d.mean()) < 2e-4
    np.testing.assert_allclose(d.std(), 0.002, rtol=0.05)
    torch.cuda.synchronize()
