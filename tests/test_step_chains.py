"""CPU checks of the fused-step oracle chains (tests/step_chains.py) that the GPU parity tests
(tests/test_gpu_fused_steps.py) compare the timed step kernels with:
* oracle/f32.py sincos is the C oracle's (and the kernels') ha_sincosf bit for bit;
* each chain runs one step per task family with resets and forces in the window, and stays physical."""
import numpy as np
import pytest

from handarm_hip import model as HM
from oracle import f32
from oracle.oracle_lib import HostState, Oracle, sincos
from tests import scenes, step_chains


def test_f32_sincos_is_the_shared_ha_sincosf_bit_for_bit():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-8, 8, 200000), rng.uniform(0, 6.3, 100000),
                        np.arange(-4096, 4096, dtype=np.float64) * (np.pi / 4)]).astype(np.float32)
    s, c = f32.sincos(x)
    so, co = sincos(x)
    assert (s.view(np.uint32) == so.view(np.uint32)).all() and (c.view(np.uint32) == co.view(np.uint32)).all()
    assert np.abs(s - np.sin(x.astype(np.float64))).max() < 2e-7


def test_uniform01_hash_on_the_2_pow_minus_24_grid():
    u = f32.uniform01(42, np.arange(4096, dtype=np.uint32), np.full(4096, 7, np.uint32), 1003)
    assert u.min() >= 0 and u.max() < 1 and abs(u.mean() - 0.5) < 0.02
    assert np.all(u * 16777216 == np.floor(u * 16777216))


def _kuka_setup(n, sub="regrasping"):
    scene = HM.load_scene(HM.KUKA_ASSET)
    p, cfg = HM.build_params({"task": HM.TASK_ALLEGRO_KUKA, "subtask": sub}, task=HM.TASK_ALLEGRO_KUKA)
    m = HM.build_model(scene, posed=HM.posed_group(HM.TASK_ALLEGRO_KUKA, cfg))
    return scene, m, p, cfg


@pytest.mark.parametrize("sub", ["regrasping", "reorientation", "throw"])
def test_kuka_chain_step_runs_with_resets_and_forces(sub):
    n = 16
    scene, m, p, cfg = _kuka_setup(n, sub)
    lo = np.array(m.dof_lower[:23], np.float32)
    up = np.array(m.dof_upper[:23], np.float32)
    hs = HostState(n, model=m, params=p)
    scales, offs = HM.kuka_env_tables(n, scene, cfg)
    scenes.fill_kuka_scene(hs, n, lo, up, list(p.reset_pose), scales, list(m.table_pos), seed=1)
    hs["task_state"][:, HM.AK_KP:HM.AK_KP + 12] = offs.reshape(n, 12)
    hs["task_state"][:, HM.AK_FORCE_PROB] = 0.5
    hs["dof_position_targets"][:] = hs["sim_targets"]
    hs["reset_buf"][:] = np.arange(n) % 2
    scalars = HM.kuka_tolerance_scalars(cfg["success_tolerance"], cfg)
    rng = np.random.default_rng(0)
    draws = rng.uniform(0, 1, (n, HM.DRAW_STRIDE)).astype(np.float32)
    hs["actions"][:] = rng.uniform(-1, 1, (n, 23))
    orc = Oracle(m, p, n)
    obs, rew, timeout = step_chains.kuka_step(orc, hs, p, lo, up, scalars, draws)
    assert obs.shape == (n, p.num_obs) and np.isfinite(obs).all() and np.isfinite(rew).all()
    assert (hs["progress_buf"][::2] >= 1).all() and (hs["progress_buf"][1::2] == 1).all()
    assert (hs["object_force"] == 0).all()                      # consumed by the simulate call
    assert np.isfinite(hs["rigid_body_state"]).all()


def test_allegro_chain_step_runs_with_resets():
    n = 16
    m = HM.build_model(HM.load_scene(HM.ALLEGRO_ASSET))
    p, _ = HM.build_params({"task": HM.TASK_ALLEGRO_HAND}, task=HM.TASK_ALLEGRO_HAND)
    lo = np.array(m.dof_lower[:16], np.float32)
    up = np.array(m.dof_upper[:16], np.float32)
    hs = HostState(n, model=m, params=p)
    scenes.fill_allegro_scene(hs, n, lo, up, seed=2)
    hs["dof_position_targets"][:] = hs["sim_targets"]
    hs["reset_buf"][:] = np.arange(n) % 2
    hs["reset_goal_buf"][:] = (np.arange(n) % 4 == 1)
    rng = np.random.default_rng(1)
    draws = rng.uniform(-1, 1, (n, HM.DRAW_STRIDE)).astype(np.float32)
    hs["actions"][:] = rng.uniform(-1, 1, (n, 16))
    obs, rew, timeout, cons = step_chains.allegro_step(Oracle(m, p, n), hs, p, lo, up, draws)
    assert obs.shape == (n, 88) and np.isfinite(obs).all() and np.isfinite(cons)
    assert (hs["progress_buf"][1::2] == 1).all()


@pytest.mark.parametrize("bin_scene", [False, True])
def test_ur5sih_chain_step_runs_with_resets(bin_scene):
    n = 8
    scene = HM.load_scene(HM.BIN_ASSET if bin_scene else HM.ASSET)
    m = HM.build_model(scene)
    cfg = {"n_objects": 8} if bin_scene else {"dr_enable": 1}
    p, _ = HM.build_params(cfg)
    hs = HostState(n, model=m, params=p)
    if bin_scene:
        scenes.fill_bin_scene(hs, n, scene, seed=3)
    else:
        scenes.fill_scene(hs, n, seed=3, near_hand=0.0)
    NO, a0 = int(p.n_objects), m.actor_object0
    root = hs["root_state"].reshape(n, m.n_actors, 13)
    hs["object_pos_initial"][:, 0] = root[:, a0:a0 + NO, 0:3]
    hs["object_quat_initial"][:, 0] = root[:, a0:a0 + NO, 3:7]
    hs["obs_cache"][:] = root[:, a0:a0 + NO, 0:7]
    hs["ur5_target"][:] = hs["dof_state"].reshape(n, 17, 2)[:, 0:6, 0]
    hs["reset_buf"][:] = np.arange(n) % 2
    draws = np.zeros((n, HM.DRAW_STRIDE), np.float32)
    draws[:, 1] = np.arange(n) % NO
    draws[:, 2:5] = 0.5
    hs["actions"][:] = np.random.default_rng(4).uniform(-1, 1, (n, 11))
    teacher, obs, rew, timeout = step_chains.ur5sih_step(Oracle(m, p, n), hs, p, m, draws)
    assert teacher.shape == (n, 108 + 13 * NO) and np.isfinite(obs).all()
    assert (hs["progress_buf"][1::2] == 1).all() and (hs["reset_buf"] == 0).all()
    assert (hs["episode"][1::2] == 1).all() and (hs["episode"][::2] == 0).all()
    if not bin_scene:
        d = obs - teacher
        assert 0 < np.abs(d).max() < 0.02                      # N(0, 0.002) observation noise
        rows = hs["dr_scale"][1::2]
        assert rows[:, HM.DR_LINK_MASS:HM.DR_LINK_MASS + 32].min() >= 0.5
