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
from oracle import kuka_oracle as KO
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


def stats_match(sim, hs, tag, cap0=None, over_frac=0.25, self_frac=None, refreshed=False):
    """The timed kernel's contact_stats equal the oracle chain's (substeps, substeps over capacity, max offered, sum
    offered, self-collision contacts offered, manifolds refreshed from their persistent record); column 6 (narrow
    phases run) is the kernel's own diagnostics. cap0: at least over_frac of the envs offered more contacts in a
    substep than chunk 0 holds (the overflow chunks in the env's global area ran); self_frac: at least that fraction of
    the envs offered self-collision contacts; refreshed: some persistent manifold was reused."""
    g = get(sim, "contact_stats").reshape(hs["contact_stats"].shape)
    o = hs["contact_stats"]
    bad = g[:, :6] != o[:, :6]
    assert not bad.any(), f"{tag} contact_stats: {int(bad.any(1).sum())} envs differ (columns {np.nonzero(bad.any(0))[0]})"
    if cap0 is not None:
        fr = float((g[:, 2] > cap0).mean())
        assert fr >= over_frac, f"{tag}: only {fr:.2f} of the envs offered more than chunk 0's {cap0} contacts"
    if self_frac is not None:
        fs = float((g[:, 4] > 0).mean())
        assert fs >= self_frac, f"{tag}: only {fs:.2f} of the envs offered self-collision contacts"
    if refreshed:
        assert g[:, 5].sum() > 0, f"{tag}: no persistent manifold was reused"
    return g


def near(a, b, atol, tag):
    d = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))
    assert np.isfinite(a).all(), f"{tag}: non-finite"
    assert d.max() <= atol, f"{tag}: max |d| {d.max():.3e} > {atol} (envs {np.unique(np.nonzero(d > atol)[0])[:10]})"
    return float(d.max())


# ----------------------------------------------------------------------------- AllegroKuka (C2)
def inject_resets(sim, hs, t, n):
    """Env resets every step of a DR window (a quarter of the envs, rotating), on both sides: the re-randomization
    gate (randomize_buf >= frequency at a reset) then fires inside the window."""
    if t == 0:
        return
    r = np.where((np.arange(n) + t) % 4 == 0, 1, hs["reset_buf"]).astype(np.int64)
    hs["reset_buf"][:] = r
    put(sim, "reset_buf", r)


def dr_exact(sim, hs, tag):
    """The DR state bit for bit: the env rows, the per-env counters, the shard-wide state (ha_dr.h vs dr_oracle)."""
    exact(sim, hs, ["dr_scale", "randomize_buf"], tag)
    g, o = get(sim, "dr_global").view(np.int32), hs["dr_global"].view(np.int32)
    assert (g == o).all(), f"{tag} dr_global differs at {np.nonzero(g != o)[0]}: {g[g != o]} vs {o[g != o]}"


def _kuka_window(sub, n, scene_fn, act_fn, resets=True, force_prob=0.5, seed=11, cfg=None, dr_frame=None):
    """K fused ak_step_kernel launches against kuka_oracle.pre -> physics_oracle -> kuka_oracle.post from the same
    host state (scene_fn(sim, hs) fills it); returns the sim, the host state and the number of random forces fired.
    cfg: extra task config (DR schema, privileged actions); dr_frame: the gym frame count the DR window starts at."""
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    sim = HandArmSim(n, "cuda:0", task_cfg={"task": HM.TASK_ALLEGRO_KUKA, "subtask": sub, **(cfg or {})},
                     task=HM.TASK_ALLEGRO_KUKA)
    p, m = sim.params, sim.model
    lo = np.array(m.dof_lower[:23], np.float32)
    up = np.array(m.dof_upper[:23], np.float32)
    hs = HostState(n, model=m, params=p)
    pull_all(sim, hs)                                       # task_state keypoints, force probabilities, scalars
    scene_fn(sim, hs, lo, up)
    hs["object_force"][:] = 0
    rng = np.random.default_rng(seed)
    hs["dof_position_targets"][:] = hs["sim_targets"]
    hs["reset_buf"][:] = (np.arange(n) % 4 == 0) if resets else 0
    hs["reset_goal_buf"][:] = (np.arange(n) % 4 == 1) if resets else 0
    hs["progress_buf"][:] = rng.integers(1, 50, n)
    hs["task_state"][:, HM.AK_FORCE_PROB] = force_prob
    hs["contact_stats"][:] = 0
    if dr_frame is not None:
        hs["dr_global"].view(np.int32)[HM.DRG_FRAME_NEXT] = dr_frame
    scalars = hs["task_scalars"].copy()
    push_all(sim, hs)
    orc = Oracle(m, p, n)
    fired = 0
    ds, G = KO.draw_slots(p), KO.goal_draws(p)
    for t in range(K):
        act = act_fn(rng, n)
        draws = rng.uniform(0, 1, (n, HM.DRAW_STRIDE)).astype(np.float32)
        # the U[-1, 1) slots (ak_task.h AK_DRAW_*): regrasping's object position noise after each goal target, the
        # reset_idx object position noise and the DOF velocity draws (reorientation draws a goal quaternion there;
        # throw the bucket side first and the object's position noise after the bucket's 4 draws)
        slots = {"regrasping": ((3, 6), (G + 3, G + 6)), "reorientation": (),
                 "throw": ((0, 1), (4, 7), (G, G + 1), (G + 4, G + 7))}[sub]
        slots += ((ds["OBJ"], ds["OBJ"] + 3), (ds["VEL"], ds["VEL"] + 23))
        for k0, k1 in slots:
            draws[:, k0:k1] = rng.uniform(-1, 1, (n, k1 - k0))
        if sub == "throw":                          # bucket offset U[0, 0.4), y U[-1, 0.7)
            for k in (1, G + 1):
                draws[:, k] *= 0.4
            for k in (2, G + 2):
                draws[:, k] = draws[:, k] * 1.7 - 1.0
        draws[:, ds["FORCE_N"]:ds["FORCE_N"] + 3] = rng.standard_normal((n, 3))
        hs["actions"][:] = act
        hs["reset_draws"][:] = draws
        put(sim, "actions", act)
        put(sim, "reset_draws", draws)
        if p.dr_enable:
            inject_resets(sim, hs, t, n)
        if p.ak_force_scale > 0:
            fired += int((draws[:, ds["FORCE_U"]] < hs["task_state"][:, HM.AK_FORCE_PROB]).sum())
        sim.task_step(HM.FLAG_REPLAY_DRAWS)
        obs, rew, timeout = step_chains.kuka_step(orc, hs, p, lo, up, scalars, draws)
        tag = f"kuka {sub} step {t}"
        if p.dr_enable:
            dr_exact(sim, hs, tag)
        scenes.assert_physics_bit_identical(sim, hs, n, tag=tag)
        exact(sim, hs, ["dof_position_targets", "sim_targets", "goal_state", "reset_buf", "reset_goal_buf",
                        "progress_buf", "successes"], tag)
        assert (get(sim, "timeout_buf").astype(bool) == timeout).all(), tag
        eo = near(get(sim, "obs"), obs, 1e-4, tag + " obs")
        er = near(get(sim, "rew"), rew, 1e-4, tag + " rew")
        cols = [k for k in range(HM.AK_KP) if k != HM.AK_RNG]     # the RNG counter word is device-mode only
        near(get(sim, "task_state")[:, cols], hs["task_state"][:, cols], 1e-4, tag + " task_state")
        print(f"{tag}: obs max |d| {eo:.2e}, rew max |d| {er:.2e}, resets {int(hs['reset_buf'].sum())}")
    return sim, hs, fired


def _kuka_random_scene(sim, hs, lo, up):
    scenes.fill_kuka_scene(hs, sim.num_envs, lo, up, list(sim.params.reset_pose), hs["object_scale"].copy(),
                           list(sim.model.table_pos), seed=4)


def _uniform_actions(rng, n):
    return rng.uniform(-1, 1, (n, 23)).astype(np.float32)


@pytest.mark.parametrize("sub", ["regrasping", "reorientation"])
def test_kuka_fused_step_with_physics_matches_oracle_chain(sub):
    """ak_step_kernel (the C2 headline kernel): goal and env resets in the first step, random forces firing in
    every step, 3 fused steps against kuka_oracle.pre -> physics_oracle -> kuka_oracle.post."""
    need_gpu()
    sim, hs, fired = _kuka_window(sub, 128, _kuka_random_scene, _uniform_actions)
    assert fired > 128 // 4, "the random-force branch must fire"
    stats_match(sim, hs, f"kuka {sub}", self_frac=0.25)


def kuka_bucket_at_hand_scene(sim, hs, lo, up, seed=5):
    """Throw: each env's bucket hangs where its hand is (the palm 8-18 cm above the bucket's floor, a few cm off its
    axis), the cuboid inside the bucket: palm / finger hulls against the bucket's wall and floor pieces (link-static
    pairs on the posed statics) and the cuboid against them, in every env at its own bucket pose."""
    from oracle.oracle_lib import Oracle
    n, p, m = sim.num_envs, sim.params, sim.model
    _kuka_random_scene(sim, hs, lo, up)
    rng = np.random.default_rng(seed)
    probe = hs.copy()
    Oracle(m, p, n).simulate(probe, 1)
    palm = probe["rigid_body_state"].reshape(n, m.n_bodies, 13)[:, m.body_robot0 + p.ak_palm_link]
    rs = hs["root_state"].reshape(n, m.n_actors, 13)
    b = rs[:, m.actor_goal]
    b[:] = 0
    b[:, 0:3] = palm[:, 0:3] - np.array([0, 0, 1], np.float32) * rng.uniform(0.08, 0.18, (n, 1)) + \
        np.concatenate([rng.uniform(-0.04, 0.04, (n, 2)), np.zeros((n, 1))], 1)
    b[:, 6] = 1
    rs[:, m.actor_object0, 0:3] = b[:, 0:3] + np.array([0.0, -0.002, 0.06], np.float32)
    rs[:, m.actor_object0, 7:13] = 0
    hs["goal_state"][:, 0:3] = b[:, 0:3] + np.array([0, 0, 0.05], np.float32)


def test_kuka_throw_fused_step_with_physics_matches_oracle_chain():
    """ak_step_kernel on the throw subtask: the bucket's 13 convex pieces as statics carried by actor 3 (ha_model_t
    v14), hanging at each env's hand with the cuboid inside; goal and env resets in the first step move the buckets
    of half the envs (allegro_kuka_throw.py:85-103), so the next steps collide with the new poses. 3 fused steps
    against kuka_oracle.pre -> physics_oracle -> kuka_oracle.post, bit-identical physics."""
    need_gpu()
    sim, hs, fired = _kuka_window("throw", 128, kuka_bucket_at_hand_scene, _uniform_actions)
    assert fired == 0 and sim.model.n_static == 14
    g = stats_match(sim, hs, "kuka throw")
    assert (g[:, 3] > 0).mean() > 0.9, "contacts with the bucket pieces in most envs"


def kuka_closed_hand_scene(sim, hs, lo, up, seed=0):
    """The fingers half closed (40-80% of their range) with their targets at the upper limits and the cuboid in the
    palm (palm_offset from iiwa7_link_7, allegro_kuka_base.py:1430-1436), still: the grasp the C2 bench reaches late in
    its episodes (offered up to 45 contacts per substep): cube-finger, cube-palm and finger-finger contacts at once"""
    from oracle.oracle_lib import Oracle
    from oracle import f32
    n, p, m = sim.num_envs, sim.params, sim.model
    _kuka_random_scene(sim, hs, lo, up)
    rng = np.random.default_rng(seed)
    ds = hs["dof_state"].reshape(n, 23, 2)
    ds[:, 7:, 0] = lo[7:] + (up[7:] - lo[7:]) * rng.uniform(0.4, 0.8, (n, 16)).astype(np.float32)
    ds[:, :, 1] = 0
    hs["sim_targets"][:] = ds[..., 0]
    hs["sim_targets"][:, 7:] = up[7:]
    probe = hs.copy()
    Oracle(m, p, n).simulate(probe, 1)
    palm = probe["rigid_body_state"].reshape(n, m.n_bodies, 13)[:, m.body_robot0 + p.ak_palm_link]
    off = np.broadcast_to(np.array(p.ak_palm_offset, np.float32), (n, 3))
    rs = hs["root_state"].reshape(n, m.n_actors, 13)
    rs[:, m.actor_object0, 0:3] = palm[:, 0:3] + f32.qrot(palm[:, 3:7], off) + rng.uniform(-0.01, 0.01, (n, 3))
    rs[:, m.actor_object0, 7:13] = 0


def test_kuka_fused_step_closed_hand_overflows_chunk0_and_matches_oracle_chain():
    """ak_step_kernel with most envs over chunk 0's 21 contacts (the second chunk in the env's global area: rows,
    row constants and contact entries; the robot blocks of link contacts past the 3 LDS slots in the spill rows) and
    every env offering self-collision contacts: finger targets toward the upper limits (hand actions U[0.6, 1], arm
    still), no resets, against the oracle chain."""
    need_gpu()

    def act(rng, n):
        a = np.zeros((n, 23), np.float32)
        a[:, 7:] = rng.uniform(0.6, 1.0, (n, 16))
        return a
    sim, hs, _ = _kuka_window("regrasping", 128, kuka_closed_hand_scene, act, resets=False, force_prob=0.0)
    g = stats_match(sim, hs, "kuka closed hand", cap0=21, self_frac=0.9, refreshed=True)
    print(f"kuka closed hand: envs over 21 contacts {(g[:, 2] > 21).mean():.2f}, max offered {g[:, 2].max()}, "
          f"self contacts per substep {g[:, 4].sum() / g[:, 0].sum():.1f}, refreshed {g[:, 5].sum()}")


# ----------------------------------------------------------------------------- AllegroHand (C3)
def _allegro_window(n, seed, act_fn, resets=True, force_scale=0.0, cfg=None):
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import HostState, Oracle
    sim = HandArmSim(n, "cuda:0", task_cfg={"task": HM.TASK_ALLEGRO_HAND, "force_scale": force_scale, **(cfg or {})},
                     task=HM.TASK_ALLEGRO_HAND)
    p, m = sim.params, sim.model
    lo = np.array(m.dof_lower[:16], np.float32)
    up = np.array(m.dof_upper[:16], np.float32)
    hs = HostState(n, model=m, params=p)
    pull_all(sim, hs)
    scenes.fill_allegro_scene(hs, n, lo, up, seed=seed)
    rng = np.random.default_rng(12)
    hs["dof_position_targets"][:] = hs["sim_targets"]
    hs["reset_buf"][:] = (np.arange(n) % 4 == 0) if resets else 0
    hs["reset_goal_buf"][:] = (np.arange(n) % 4 == 1) if resets else 0
    hs["progress_buf"][:] = rng.integers(1, 50, n)
    hs["contact_stats"][:] = 0
    push_all(sim, hs)
    orc = Oracle(m, p, n)
    for t in range(K):
        act = act_fn(rng, n)
        draws = rng.uniform(-1, 1, (n, HM.DRAW_STRIDE)).astype(np.float32)
        hs["actions"][:] = act
        put(sim, "actions", act)
        put(sim, "reset_draws", draws)
        if p.dr_enable:
            inject_resets(sim, hs, t, n)
        sim.task_step(HM.FLAG_REPLAY_DRAWS)
        obs, rew, timeout, cons = step_chains.allegro_step(orc, hs, p, lo, up, draws)
        tag = f"allegro step {t}"
        if p.dr_enable:
            dr_exact(sim, hs, tag)
        scenes.assert_physics_bit_identical(sim, hs, n, tag=tag)
        exact(sim, hs, ["dof_position_targets", "sim_targets", "goal_state", "reset_buf", "reset_goal_buf",
                        "progress_buf", "successes"], tag)
        if force_scale > 0:          # the object force state (task_state AH_TS_FORCE) bit for bit
            np.testing.assert_array_equal(get(sim, "task_state")[:, 0:3], hs["task_state"][:, 0:3], err_msg=tag)
        assert (get(sim, "timeout_buf").astype(bool) == timeout).all(), tag
        eo = near(get(sim, "obs"), obs, 1e-4, tag + " obs")
        er = near(get(sim, "rew"), rew, 1e-4, tag + " rew")
        np.testing.assert_allclose(get(sim, "consecutive_successes")[0], cons, rtol=1e-5, atol=1e-6)
        print(f"{tag}: obs max |d| {eo:.2e}, rew max |d| {er:.2e}")
    return sim, hs


def test_allegro_fused_step_with_physics_matches_oracle_chain():
    """ah_step_kernel (C3): goal and env resets in the first step, 3 fused steps (2 gym.simulate each) against
    the oracle chain, including the joint forces the full_state observation reads."""
    need_gpu()
    sim, hs = _allegro_window(128, 6, lambda rng, n: rng.uniform(-1, 1, (n, 16)).astype(np.float32))
    stats_match(sim, hs, "allegro", self_frac=0.25)


def test_allegro_fused_step_with_random_forces_matches_oracle_chain():
    """ah_step_kernel with forceScale 1 (allegro_hand.py:617-625): every env draws a new force each step (replayed
    selection), applied to the first of the step's two physics calls, against the oracle chain."""
    need_gpu()
    sim, hs = _allegro_window(128, 6, lambda rng, n: rng.uniform(-1, 1, (n, 16)).astype(np.float32), force_scale=1.0)
    assert np.abs(hs["task_state"][:, 0:3]).max() > 0.01


def test_allegro_fused_step_closing_hand_overflows_chunk0_and_matches_oracle_chain():
    """ah_step_kernel with the fingers closing on the cube (actions U[0.5, 1]: targets toward the upper limits, no
    resets): envs over chunk 0's 12 contacts (chunks 1-3 in the env's global area) and self-collision contacts in
    most envs, against the oracle chain."""
    need_gpu()
    sim, hs = _allegro_window(128, 0, lambda rng, n: rng.uniform(0.5, 1.0, (n, 16)).astype(np.float32), resets=False)
    g = stats_match(sim, hs, "allegro closing hand", cap0=12, self_frac=0.5)
    assert g[:, 5].sum() == 0 and sim.t["contact_cache"].numel() == 0   # no persistent manifolds in this family
    print(f"allegro closing hand: envs over 12 contacts {(g[:, 2] > 12).mean():.2f}, max offered {g[:, 2].max()}, "
          f"self contacts per substep {g[:, 4].sum() / g[:, 0].sum():.1f}, refreshed {g[:, 5].sum()}")


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
    hs["contact_stats"][:] = 0
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
    stats_match(sim, hs, "ur5sih DR", refreshed=True)


def test_ur5sih_pile_in_hand_fused_step_overflows_chunk0_and_matches_oracle_chain():
    """ha_step_kernel (C4 kernel, DR on) with the three objects dropped together into the hand: more than chunk 0's 21
    contacts in most envs (chunks 1-3 in the env's global area), resets in the window, against the oracle chain."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    from oracle.oracle_lib import Oracle
    from tests.test_gpu_dr import _dr_rows
    n = 64
    sim = HandArmSim(n, "cuda:0", task_cfg={"dr_enable": 1})
    m = sim.model

    def fill(hs):
        scenes.fill_scene(hs, n, seed=13, near_hand=0.0)
        hs["dr_scale"][:] = _dr_rows(n, np.random.default_rng(3))
        probe = hs.copy()
        Oracle(m, sim.params, n).simulate(probe, 1)
        body = probe["rigid_body_state"].reshape(n, m.n_bodies, 13)
        rng = np.random.default_rng(13)
        hull_links = sorted({int(m.hull_link[k]) for k in range(m.n_link_hulls)})
        rs = hs["root_state"].reshape(n, m.n_actors, 13)
        for o in range(3):
            lk = np.array(hull_links)[rng.integers(len(hull_links) // 2, len(hull_links), n)]
            rs[:, m.actor_object0 + o, 0:3] = body[np.arange(n), m.body_robot0 + lk, 0:3] + rng.uniform(-0.015, 0.015, (n, 3))
            rs[:, m.actor_object0 + o, 7:13] = 0.0
    hs, rng = _ur5sih_case(sim, n, 23, fill)
    _ur5sih_window(sim, hs, rng, n, "ur5sih pile")
    g = stats_match(sim, hs, "ur5sih pile", cap0=21, refreshed=True)
    print(f"ur5sih pile: envs over 21 contacts {(g[:, 2] > 21).mean():.2f}, max offered {g[:, 2].max()}, "
          f"refreshed {g[:, 5].sum()}")


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
    g = stats_match(sim, hs, "bin", cap0=21, refreshed=True)
    print(f"bin: envs over 21 contacts {(g[:, 2] > 21).mean():.2f}, max offered {g[:, 2].max()}, refreshed {g[:, 5].sum()}")
