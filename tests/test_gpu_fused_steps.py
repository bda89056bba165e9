"""The timed step kernels, physics on, against their oracle chains (tests/step_chains.py).

bench.py times the fused step launches: ``ak_step_kernel`` (C2 headline), ``ah_step_kernel`` (C3), ``ha_step_kernel``
with DR rows (C4) and ``hb_step_kernel`` (C5). Each is its own template instantiation (own register budget, own
physics capacity), so each is checked here as launched: K = 3 ``ha_task_step`` launches with the physics on, resets
and goal resets in the window (replayed draws), random object forces firing (Kuka), DR rows and observation noise
(C4), against the oracle chain from the same host state:
* physics outputs (dof state, root state, rigid-body states, net contact forces, joint forces) bit-identical;
* done / reset / goal-reset / progress / successes / timeout bit-exact, targets bit-exact;
* observations and rewards within 1e-4 (north_star's tolerance), task state within 1e-4.
"""
import numpy as np
import pytest
import torch

from handarm_hip import model as HM
from tests import scenes, step_chains

pytestmark = pytest.mark.gpu
K = 3


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def get(sim, name):
    torch.cuda.synchronize()
    return sim.t[name].cpu().numpy()


def push_all(sim, hs, skip=("stats", "term_sums")):
    for k in HM.STATE_FIELDS:
        if k in skip or k in HM.null_fields(sim.task):
            continue
        put(sim, k, hs[k])


def pull_all(sim, hs, skip=("stats", "term_sums")):
    for k in HM.STATE_FIELDS:
        if k in skip or k in HM.null_fields(sim.task):
            continue
        hs[k][...] = get(sim, k).reshape(hs[k].shape)


def exact(sim, hs, names, tag):
    for k in names:
        g = get(sim, k).reshape(hs[k].shape)
        o = hs[k]
        bad = g != o
        assert not bad.any(), f"{tag} {k}: {int(bad.sum())} elements differ (envs {np.unique(np.nonzero(bad)[0])[:10]})"


def near(a, b, atol, tag):
    d = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))
    assert np.isfinite(a).all(), f"{tag}: non-finite"
    assert d.max() <= atol, f"{tag}: max |d| {d.max():.3e} > {atol} (envs {np.unique(np.nonzero(d > atol)[0])[:10]})"
    return float(d.max())


# ----------------------------------------------------------------------------- AllegroKuka (C2)
@pytest.mark.parametrize("sub", ["regrasping", "reorientation"])
def test_kuka_fused_step_with_physics_matches_oracle_chain(sub):
    """ak_step_kernel (the C2 headline kernel): goal and env resets in the first step, random forces firing in
    every step, 3 fused steps against kuka_oracle.pre -> physics_oracle -> kuka_oracle.post."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    n = 128
    sim = HandArmSim(n, "cuda:0", task_cfg={"task": HM.TASK_ALLEGRO_KUKA, "subtask": sub}, task=HM.TASK_ALLEGRO_KUKA)
    p, m = sim.params, sim.model
    lo = np.array(m.dof_lower[:23], np.float32)
    up = np.array(m.dof_upper[:23], np.float32)
    hs = HostState(n, model=m, params=p)
    pull_all(sim, hs)                                       # task_state keypoints, force probabilities, scalars
    scenes.fill_kuka_scene(hs, n, lo, up, list(p.reset_pose), hs["object_scale"].copy(), list(m.table_pos), seed=4)
    hs["object_force"][:] = 0
    rng = np.random.default_rng(11)
    hs["dof_position_targets"][:] = hs["sim_targets"]
    hs["reset_buf"][:] = (np.arange(n) % 4 == 0)
    hs["reset_goal_buf"][:] = (np.arange(n) % 4 == 1)
    hs["progress_buf"][:] = rng.integers(1, 50, n)
    hs["task_state"][:, HM.AK_FORCE_PROB] = 0.5
    scalars = hs["task_scalars"].copy()
    push_all(sim, hs)
    orc = Oracle(m, p, n)
    fired = 0
    for t in range(K):
        act = rng.uniform(-1, 1, (n, 23)).astype(np.float32)
        draws = rng.uniform(0, 1, (n, HM.DRAW_STRIDE)).astype(np.float32)
        # the U[-1, 1) slots (ak_task.h AK_DRAW_*): regrasping's object position noise after each goal target, the
        # reset_idx object position noise and the DOF velocity draws (reorientation draws a goal quaternion there)
        slots = ((3, 6), (12, 15), (18, 21), (48, 71)) if sub == "regrasping" else ((18, 21), (48, 71))
        for k0, k1 in slots:
            draws[:, k0:k1] = rng.uniform(-1, 1, (n, k1 - k0))
        draws[:, 72:75] = rng.standard_normal((n, 3))
        hs["actions"][:] = act
        hs["reset_draws"][:] = draws
        put(sim, "actions", act)
        put(sim, "reset_draws", draws)
        fired += int((draws[:, 71] < hs["task_state"][:, HM.AK_FORCE_PROB]).sum())
        sim.task_step(HM.FLAG_REPLAY_DRAWS)
        obs, rew, timeout = step_chains.kuka_step(orc, hs, p, lo, up, scalars, draws)
        tag = f"kuka {sub} step {t}"
        scenes.assert_physics_bit_identical(sim, hs, n, tag=tag)
        exact(sim, hs, ["dof_position_targets", "sim_targets", "goal_state", "reset_buf", "reset_goal_buf",
                        "progress_buf", "successes"], tag)
        assert (get(sim, "timeout_buf").astype(bool) == timeout).all(), tag
        eo = near(get(sim, "obs"), obs, 1e-4, tag + " obs")
        er = near(get(sim, "rew"), rew, 1e-4, tag + " rew")
        cols = [k for k in range(HM.AK_KP) if k != HM.AK_RNG]     # the RNG counter word is device-mode only
        near(get(sim, "task_state")[:, cols], hs["task_state"][:, cols], 1e-4, tag + " task_state")
        print(f"{tag}: obs max |d| {eo:.2e}, rew max |d| {er:.2e}, resets {int(hs['reset_buf'].sum())}")
    assert fired > n // 4, "the random-force branch must fire"


# ----------------------------------------------------------------------------- AllegroHand (C3)
def test_allegro_fused_step_with_physics_matches_oracle_chain():
    """ah_step_kernel (C3): goal and env resets in the first step, 3 fused steps (2 gym.simulate each) against
    the oracle chain, including the joint forces the full_state observation reads."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    n = 128
    sim = HandArmSim(n, "cuda:0", task_cfg={"task": HM.TASK_ALLEGRO_HAND}, task=HM.TASK_ALLEGRO_HAND)
    p, m = sim.params, sim.model
    lo = np.array(m.dof_lower[:16], np.float32)
    up = np.array(m.dof_upper[:16], np.float32)
    hs = HostState(n, model=m, params=p)
    pull_all(sim, hs)
    scenes.fill_allegro_scene(hs, n, lo, up, seed=6)
    rng = np.random.default_rng(12)
    hs["dof_position_targets"][:] = hs["sim_targets"]
    hs["reset_buf"][:] = (np.arange(n) % 4 == 0)
    hs["reset_goal_buf"][:] = (np.arange(n) % 4 == 1)
    hs["progress_buf"][:] = rng.integers(1, 50, n)
    push_all(sim, hs)
    orc = Oracle(m, p, n)
    for t in range(K):
        act = rng.uniform(-1, 1, (n, 16)).astype(np.float32)
        draws = rng.uniform(-1, 1, (n, HM.DRAW_STRIDE)).astype(np.float32)
        hs["actions"][:] = act
        put(sim, "actions", act)
        put(sim, "reset_draws", draws)
        sim.task_step(HM.FLAG_REPLAY_DRAWS)
        obs, rew, timeout, cons = step_chains.allegro_step(orc, hs, p, lo, up, draws)
        tag = f"allegro step {t}"
        scenes.assert_physics_bit_identical(sim, hs, n, tag=tag)
        exact(sim, hs, ["dof_position_targets", "sim_targets", "goal_state", "reset_buf", "reset_goal_buf",
                        "progress_buf", "successes"], tag)
        assert (get(sim, "timeout_buf").astype(bool) == timeout).all(), tag
        eo = near(get(sim, "obs"), obs, 1e-4, tag + " obs")
        er = near(get(sim, "rew"), rew, 1e-4, tag + " rew")
        np.testing.assert_allclose(get(sim, "consecutive_successes")[0], cons, rtol=1e-5, atol=1e-6)
        print(f"{tag}: obs max |d| {eo:.2e}, rew max |d| {er:.2e}")


# ----------------------------------------------------------------------------- Ur5Sih: C4 (DR) and C5 (clutter)
def _ur5sih_case(sim, n, seed, scene_fill):
    from oracle.oracle_lib import HostState
    p, m = sim.params, sim.model
    hs = HostState(n, model=m, params=p)
    pull_all(sim, hs)
    scene_fill(hs)
    rng = np.random.default_rng(seed)
    NO = int(p.n_objects)
    a0 = m.actor_object0
    root = hs["root_state"].reshape(n, m.n_actors, 13)
    # the initial poses a reset puts back: the scene's objects, raised 2 mm
    hs["object_pos_initial"][:, 0] = root[:, a0:a0 + NO, 0:3] + np.array([0, 0, 0.002], np.float32)
    hs["object_quat_initial"][:, 0] = root[:, a0:a0 + NO, 3:7]
    hs["goal_pos"][:] = np.array(p.goal_pos, np.float32)
    hs["target_object_index"][:] = rng.integers(0, NO, n)
    hs["obs_cache"][:] = root[:, a0:a0 + NO, 0:7]
    hs["ur5_target"][:] = hs["dof_state"].reshape(n, 17, 2)[:, 0:6, 0]
    hs["servo"][:] = rng.uniform(-500, 500, (n, 5))
    hs["dof_position_targets"][:] = hs["sim_targets"]
    hs["reset_buf"][:] = (np.arange(n) % 4 == 0)
    hs["progress_buf"][:] = rng.integers(1, 150, n)
    hs["episode"][:] = rng.integers(0, 1000, n)
    return hs, rng


def _ur5sih_window(sim, hs, rng, n, tag0):
    from oracle.oracle_lib import Oracle
    p, m = sim.params, sim.model
    NO = int(p.n_objects)
    push_all(sim, hs)
    orc = Oracle(m, p, n)
    for t in range(K):
        act = rng.uniform(-1, 1, (n, 11)).astype(np.float32)
        draws = np.zeros((n, HM.DRAW_STRIDE), np.float32)
        draws[:, 0] = 0
        draws[:, 1] = rng.integers(0, NO, n)
        draws[:, 2:5] = rng.uniform(0, 1, (n, 3))
        hs["actions"][:] = act
        put(sim, "actions", act)
        put(sim, "reset_draws", draws)
        sim.task_step(HM.FLAG_REPLAY_DRAWS)
        teacher, obs, rew, timeout = step_chains.ur5sih_step(orc, hs, p, m, draws)
        tag = f"{tag0} step {t}"
        names = ["dof_position_targets", "sim_targets", "ur5_target", "servo", "smoothed", "goal_pos",
                 "target_object_index", "object_configuration_indices", "reset_buf", "progress_buf",
                 "goal_reached_before", "episode", "obs_cache"]
        if p.dr_enable:
            names.append("dr_scale")
        exact(sim, hs, names, tag)
        scenes.assert_physics_bit_identical(sim, hs, n, tag=tag)
        assert (get(sim, "timeout_buf").astype(bool) == timeout).all(), tag
        et = near(get(sim, "teacher_obs"), teacher, 1e-4, tag + " teacher obs")
        eo = near(get(sim, "obs"), obs, 1e-4, tag + " obs")
        er = near(get(sim, "rew"), rew, 1e-4, tag + " rew")
        print(f"{tag}: teacher obs max |d| {et:.2e}, obs {eo:.2e}, rew {er:.2e}")


def test_ur5sih_dr_fused_step_with_physics_matches_oracle_chain():
    """ha_step_kernel as C4 runs it (DR on): DR mass / friction rows in the physics, rows re-sampled by the resets
    in the window (device-mode hash), observation noise, reset_idx's extra gym.simulate, 3 x 2 substeps a step."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from tests.test_gpu_dr import _dr_rows
    n = 64
    sim = HandArmSim(n, "cuda:0", task_cfg={"dr_enable": 1})
    assert sim.params.dr_enable == 1

    def fill(hs):
        scenes.fill_scene(hs, n, seed=9, near_hand=0.0)
        hs["dr_scale"][:] = _dr_rows(n, np.random.default_rng(2))
    hs, rng = _ur5sih_case(sim, n, 21, fill)
    _ur5sih_window(sim, hs, rng, n, "ur5sih DR")


def test_bin_fused_step_with_physics_matches_oracle_chain():
    """hb_step_kernel (C5): 8 objects in the tote, 84-contact list, resets in the window."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    n = 64
    sim = HandArmSim(n, "cuda:0", task_cfg={"n_objects": 8}, scene=HM.load_scene(HM.BIN_ASSET))

    def fill(hs):
        scenes.fill_bin_scene(hs, n, sim.scene, seed=8)
    hs, rng = _ur5sih_case(sim, n, 22, fill)
    _ur5sih_window(sim, hs, rng, n, "bin")
