"""Schema-driven domain randomization (task.randomization_params) on the device against oracle/dr_oracle.py.

The reference's engine: tasks/base/vec_task.py:646-876 (apply_randomizations) + utils/dr_utils.py:71-238, consumed by
AllegroKuka's reset_idx (allegro_kuka_base.py:1248-1249) with the schema of cfg/task/AllegroKuka.yaml:115-207.
* Fused AllegroKuka / AllegroHand steps with the full schemas: dr_scale rows, randomize_buf and the shard-wide
  dr_global state bit-identical to the oracle every step, physics bit-identical with the randomized DOF gains and
  limits, masses, frictions, object scale and gravity, observations (noise included) within 1e-4.
* Distributions per parameter kind (uniform / loguniform / gaussian, scaling / additive, buckets) over 4096 envs.
* Schedules: the observation noise grows with the gym frame count as vec_task.py:692-698 prescribes (linear), and
  stays off before schedule_steps (constant).
The draws come from the device counter hash, not numpy's global generator: parity with the reference is of the
distributions and schedules, not of the individual draws."""
import copy

import numpy as np
import pytest
import torch

from handarm_hip import dr as DR
from handarm_hip import model as HM
from tests.test_gpu_fused_steps import _allegro_window, _kuka_random_scene, _kuka_window, get, need_gpu, put

pytestmark = pytest.mark.gpu


def _kuka_schema(frequency=2):
    s = copy.deepcopy(DR.ALLEGRO_KUKA_SCHEMA)
    s["frequency"] = frequency
    return s


def test_kuka_dr_schema_fused_steps_match_oracle_chain():
    """AllegroKuka.yaml's schema at frame 35000 (the 30000-frame schedules complete, the 40000-frame ones at 0.875),
    re-randomization every 2 steps: rows, counters, shard state bit-identical; physics bit-identical."""
    need_gpu()

    def act(rng, n):
        return rng.uniform(-1, 1, (n, 23)).astype(np.float32)
    sim, hs, _ = _kuka_window("regrasping", 128, _kuka_random_scene, act, cfg={"dr_enable": 1,
                              "randomization_params": _kuka_schema()}, dr_frame=35000)
    rows = hs["dr_scale"]
    kd0 = np.array(list(sim.model.dof_kd)[:23], np.float32)
    assert np.abs(rows[:, HM.DR_DOF_KD:HM.DR_DOF_KD + 23] / kd0 - 1).max() > 0.5        # damping x U_log[0.3, 3]
    assert np.abs(rows[:, HM.DR_OBJ_SCALE] - 1).max() > 0.2                          # object scale U[0.5, 2]
    g = hs["dr_global"]
    assert g.view(np.int32)[HM.DRG_EPOCH] >= 1
    # AllegroKuka.yaml's gravity sits outside sim_params (sim_params: None), which the reference does not read: the
    # gravity stays nominal (handarm_hip/dr.py); AllegroHand.yaml's sim_params.gravity is randomized (test below)
    np.testing.assert_array_equal(g[HM.DRG_GRAVITY:HM.DRG_GRAVITY + 3], np.array([0, 0, -9.81], np.float32))


def test_kuka_privileged_actions_fused_steps_match_oracle_chain():
    """privilegedActions (allegro_kuka_base.py:62-74,1357-1361,1417-1424): 26 actions, the first 3 an ENV_SPACE object
    torque x privilegedActionsTorque; the hand reads actions[:, 3:][:, 7:23] and the arm self.actions[:, :7]."""
    need_gpu()

    def act(rng, n):
        return rng.uniform(-1, 1, (n, 26)).astype(np.float32)
    sim, hs, _ = _kuka_window("regrasping", 128, _kuka_random_scene, act,
                              cfg={"privileged_actions": True, "privileged_actions_torque": 0.5})
    assert sim.params.num_actions == 26 and sim.t["actions"].shape[1] == 26


def test_kuka_dr_and_privileged_through_the_task_class():
    """AllegroKuka(cfg) with task.randomize and env.privilegedActions: the VecTask surface runs the schema (no
    NotImplementedError), obs noise present, randomize_buf counting, 26-wide actions."""
    need_gpu()
    from handarm_hip.tasks import AllegroKuka
    cfg = {"env": {"numEnvs": 64, "privilegedActions": True}, "task": {"randomize": True}}
    env = AllegroKuka(cfg, "cuda:0", "cuda:0")
    assert env.num_actions == 26
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    for _ in range(3):
        env.step(torch.rand((64, 26), device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    assert (env.randomize_buf.cpu().numpy() == 3).all()         # the first randomization leaves the counts running
    gi = env.sim.t["dr_global"].cpu().numpy().view(np.int32)
    assert gi[HM.DRG_FRAME_NEXT] == 3 and gi[HM.DRG_EPOCH] == 1 and gi[HM.DRG_FIRST] == 0


def test_allegro_hand_dr_schema_fused_steps_match_oracle_chain():
    """AllegroHand.yaml's schema (no schedules; setup_only mass and object scale at the first randomization only),
    re-randomization every step."""
    need_gpu()
    s = copy.deepcopy(DR.ALLEGRO_HAND_SCHEMA)
    s["frequency"] = 1
    sim, hs = _allegro_window(128, 6, lambda rng, n: rng.uniform(-1, 1, (n, 16)).astype(np.float32),
                              cfg={"dr_enable": 1, "randomization_params": s})
    rows = hs["dr_scale"]
    assert np.abs(rows[:, HM.DR_OBJ_SCALE] - 1).max() > 0.02                         # U[0.95, 1.05]
    assert abs(hs["dr_global"][HM.DRG_GRAVITY + 2] + 9.81) > 1e-4                  # sim_params.gravity + N(0, 0.4)
    assert rows[:, HM.DR_LINK_MASS:HM.DR_LINK_MASS + sim.model.n_links].std() > 0.2


def _reset_launch_rows(n, frame, schema, task=HM.TASK_ALLEGRO_KUKA):
    """One reset launch with every env resetting at gym frame `frame`: the first randomization on the device and in
    the oracle. Returns (sim, device rows, oracle rows, device dr_global, oracle dr_global)."""
    from handarm_hip.sim import HandArmSim
    from oracle import dr_oracle as DO
    sim = HandArmSim(n, "cuda:0", task_cfg={"task": task, "dr_enable": 1, "randomization_params": schema}, task=task)
    g0 = get(sim, "dr_global").copy()
    g0.view(np.int32)[HM.DRG_FRAME_NEXT] = frame
    put(sim, "dr_global", g0)
    sim.t["reset_buf"].fill_(1)
    ep = (np.arange(n, dtype=np.uint32) * 3).astype(np.uint32)
    put(sim, "episode", ep.view(np.int32))
    rows0, rb0 = get(sim, "dr_scale").copy(), get(sim, "randomize_buf").copy()
    pools = get(sim, "object_indices").reshape(n, -1)
    sim.task_reset(HM.FLAG_NO_PHYSICS)
    g = DO.global_update(sim.params, g0.copy(), True, 1)
    DO.env_pre(sim.params, sim.model, rows0, rb0, ep, pools, np.ones(n, bool), g, False)
    return sim, get(sim, "dr_scale"), rows0, get(sim, "dr_global"), g


def test_dr_distributions_per_parameter_kind():
    """4096 envs sampled at full schedule: every row bit-identical to the oracle, and each kind's distribution."""
    need_gpu()
    n = 4096
    sim, dr, orow, g, og = _reset_launch_rows(n, 10 ** 6, _kuka_schema())
    np.testing.assert_array_equal(dr, orow)
    assert (g.view(np.int32) == og.view(np.int32)).all()
    m, L, D = sim.model, sim.model.n_links, 23
    # uniform scaling: mass x U[0.5, 1.5]
    lm = dr[:, HM.DR_LINK_MASS:HM.DR_LINK_MASS + L]
    assert lm.min() >= 0.5 and lm.max() <= 1.5
    assert abs(lm.mean() - 1.0) < 0.005 and abs(lm.std() - 1 / np.sqrt(12)) < 0.005
    # uniform scaling + 250 buckets over [0.7, 1.3]: on the grid
    lf = dr[:, HM.DR_LINK_FRIC:HM.DR_LINK_FRIC + L]
    grid = (lf - 0.7) / (0.6 / 250)
    assert np.abs(grid - np.round(grid)).max() < 2e-3 and lf.min() >= 0.7 - 1e-6 and lf.max() < 1.3
    assert len(np.unique(lf)) > 200
    # loguniform scaling: log(kd' / kd) ~ U[log 0.3, log 3]
    kd0 = np.array(list(m.dof_kd)[:D], np.float32)
    lr = np.log(dr[:, HM.DR_DOF_KD:HM.DR_DOF_KD + D] / kd0)
    assert lr.min() >= np.log(0.3) - 1e-5 and lr.max() <= np.log(3.0) + 1e-5
    assert abs(lr.mean() - 0.5 * (np.log(0.3) + np.log(3.0))) < 0.02
    assert abs(lr.std() - (np.log(3.0) - np.log(0.3)) / np.sqrt(12)) < 0.02
    ks = np.log(dr[:, HM.DR_DOF_KP:HM.DR_DOF_KP + D] / np.array(list(m.dof_kp)[:D], np.float32))
    assert ks.min() >= np.log(0.75) - 1e-5 and ks.max() <= np.log(1.5) + 1e-5
    # gaussian additive: lower / upper + N(0, 0.01)
    for slot, name in ((HM.DR_DOF_LOWER, "dof_lower"), (HM.DR_DOF_UPPER, "dof_upper")):
        d = dr[:, slot:slot + D] - np.array(list(getattr(m, name))[:D], np.float32)
        assert abs(d.mean()) < 5e-4 and abs(d.std() - 0.01) < 5e-4
    # the object: scale U[0.5, 2] (schedule_steps 1), mass x U[0.5, 1.5]
    sc = dr[:, HM.DR_OBJ_SCALE]
    assert sc.min() >= 0.5 and sc.max() <= 2.0 and abs(sc.mean() - 1.25) < 0.02
    om = dr[:, HM.DR_OBJ_MASS]
    assert om.min() >= 0.5 and om.max() <= 1.5
    # gravity: original + N(0, 0.4) per axis, one draw for the shard
    gv = g[HM.DRG_GRAVITY:HM.DRG_GRAVITY + 3] - np.array([0, 0, -9.81], np.float32)
    assert np.abs(gv).max() < 5 * 0.4


@pytest.mark.parametrize("frame", [0, 10000, 20000, 40000, 80000])
def test_dr_schedule_scales_with_frame_count(frame):
    """vec_task.py:692-698 / dr_utils.py:82-87: linear schedule s = min(frame, steps) / steps. The sampled spreads
    and the noise parameters the first randomization sets at `frame` follow s: the 40000-frame observation / action
    noise scale is s x (0.002, 0.001) / (0.05, 0.015), the 30000-frame mass ranges [1 - 0.5 s, 1 + 0.5 s]."""
    need_gpu()
    n = 1024
    sim, dr, orow, g, og = _reset_launch_rows(n, frame, _kuka_schema())
    np.testing.assert_array_equal(dr, orow)
    assert (g.view(np.int32) == og.view(np.int32)).all()
    s40, s30 = min(frame, 40000) / 40000, min(frame, 30000) / 30000
    np.testing.assert_allclose(g[HM.DRG_OBS:HM.DRG_OBS + 4], [0.001 * s40, 0, 0.002 * s40, 0], rtol=1e-6, atol=1e-12)
    np.testing.assert_allclose(g[HM.DRG_ACT:HM.DRG_ACT + 4], [0.015 * s40, 0, 0.05 * s40, 0], rtol=1e-6, atol=1e-12)
    lm = dr[:, HM.DR_LINK_MASS:HM.DR_LINK_MASS + sim.model.n_links]
    assert lm.min() >= 1 - 0.5 * s30 - 1e-6 and lm.max() <= 1 + 0.5 * s30 + 1e-6
    if s30 > 0.2:
        assert lm.max() - lm.min() > 0.9 * s30


def test_dr_constant_schedule_and_observation_noise_spread():
    """Ur5Sih, NO_PHYSICS steps: a 'constant' schedule keeps the observation noise off before schedule_steps frames
    and at full strength after; the noise (obs - teacher obs) is the oracle's bit for bit, its spread
    sqrt(var^2 + var_corr^2) with the correlated term drawn once per non-env randomization."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle import dr_oracle as DO
    schema = {"frequency": 1, "observations": {"range": [0, 0.01], "range_correlated": [0, 0.005],
                                               "operation": "additive", "distribution": "gaussian",
                                               "schedule": "constant", "schedule_steps": 100}}
    n = 2048
    for frame, on in ((50, False), (150, True)):
        sim = HandArmSim(n, "cuda:0", task_cfg={"dr_enable": 1, "randomization_params": schema})
        g0 = get(sim, "dr_global").copy()
        g0.view(np.int32)[HM.DRG_FRAME_NEXT] = frame
        put(sim, "dr_global", g0)
        sim.t["reset_buf"][: n // 2] = 1
        sim.task_step(HM.FLAG_NO_PHYSICS)
        d = get(sim, "obs") - get(sim, "teacher_obs")
        g = DO.global_update(sim.params, g0.copy(), True, 0)
        assert (get(sim, "dr_global").view(np.int32) == g.view(np.int32)).all()
        np.testing.assert_array_equal(get(sim, "obs"), DO.obs_noise(sim.params, g, get(sim, "teacher_obs")))
        if on:
            np.testing.assert_allclose(d.std(), np.sqrt(0.01 ** 2 + 0.005 ** 2), rtol=0.05)
        else:
            assert np.abs(d).max() == 0.0
