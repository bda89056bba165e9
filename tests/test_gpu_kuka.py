"""GPU parity for the AllegroKuka tasks (config C2), through the C ABI:
* task math (observe / reward / resets / targets / random forces / task state) against the reference-generated
  goldens (bit-exact done masks and counters; float tolerances stated per check), the three subtasks;
* physics against the C oracle after one gym.simulate, with per-env cuboid dimensions and object forces
  (1-ulp-sensitivity-calibrated tolerance, as for Ur5Sih / AllegroHand);
* the VecTask class over a full-size (4096-env) episode.
"""
import os

import numpy as np
import pytest
import torch

from handarm_hip import model as HM
from tests import scenes

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def make_sim(n, **cfg):
    need_gpu()
    from handarm_hip.sim import HandArmSim
    cfg = dict(cfg, task=HM.TASK_ALLEGRO_KUKA)
    return HandArmSim(n, "cuda:0", task_cfg=cfg, task=HM.TASK_ALLEGRO_KUKA)


def close(a, b, rtol, atol, what):
    """assert_allclose that names the failing columns (obs layout: allegro_kuka_base.py:1091-1172)."""
    bad = ~np.isclose(a, b, rtol=rtol, atol=atol)
    if bad.any():
        cols = np.unique(np.nonzero(bad)[-1])
        envs = np.unique(np.nonzero(bad)[0])
        raise AssertionError(f"{what}: {bad.sum()} mismatches, columns {cols.tolist()[:20]}, envs {envs.tolist()[:20]}, "
                             f"max abs {np.abs(a - b)[bad].max():.3e}")


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def get(sim, name):
    torch.cuda.synchronize()
    return sim.t[name].cpu().numpy()


@pytest.mark.parametrize("sub", ["regrasping", "reorientation", "throw"])
def test_kuka_observe_and_reward_against_reference_goldens(sub):
    d = np.load(os.path.join(G, f"kuka_obs_reward_{sub}.npz"))
    S, N = d["rew"].shape
    sim = make_sim(N, subtask=sub)
    np.testing.assert_array_equal(get(sim, "object_scale").reshape(N, 3), d["object_scale"])
    for s in range(S):
        for k, g in [("dof_state", "dof_state"), ("root_state", "root_state"), ("rigid_body_state", "rigid_body_state"),
                     ("goal_state", "goal_state"), ("task_state", "task_state_in"), ("reset_buf", "reset_in"),
                     ("progress_buf", "progress_in"), ("successes", "successes_in")]:
            put(sim, k, d[g][s])
        sim.task_observe(0)
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][s])
        np.testing.assert_array_equal(get(sim, "reset_goal_buf"), d["reset_goal"][s])
        np.testing.assert_array_equal(get(sim, "progress_buf"), d["progress"][s])
        np.testing.assert_array_equal(get(sim, "successes"), d["successes"][s])
        np.testing.assert_allclose(get(sim, "obs"), d["obs"][s], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(get(sim, "rew"), d["rew"][s], rtol=1e-5, atol=1e-4)
        np.testing.assert_allclose(get(sim, "task_state")[:, :32], d["task_state"][s][:, :32], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("sub,privileged", [("regrasping", False), ("reorientation", False), ("throw", False),
                                            ("regrasping", True)])
def test_kuka_step_with_resets_replayed_against_reference_goldens(sub, privileged):
    """The fused step kernel without physics: goal + env resets and random forces from the recorded reference
    draws, hand/arm targets, FK refresh, progress, full_state observations, reward, done, timeout. privileged: the
    26-action variant (its targets read the reference's action slices; the object torque it applies is not a state
    output of a physics-free step: tests/test_kuka_golden.py pins its value against the same golden and
    tests/test_gpu_dr_schema.py its effect on the physics against the oracle chain)."""
    d = np.load(os.path.join(G, f"kuka_steps_{sub}{'_privileged' if privileged else ''}.npz"))
    T, N = d["rew"].shape
    sim = make_sim(N, subtask=sub, privileged_actions=privileged)
    flags = HM.FLAG_NO_PHYSICS | HM.FLAG_REPLAY_DRAWS
    for t in range(T):
        for k, g in [("dof_state", "dof_state"), ("root_state", "root_state"), ("goal_state", "goal_state"),
                     ("dof_position_targets", "targets"), ("sim_targets", "targets"), ("actions", "actions"),
                     ("reset_buf", "reset_in"), ("reset_goal_buf", "reset_goal_in"), ("progress_buf", "progress_in"),
                     ("successes", "successes_in"), ("task_state", "task_state_in"), ("reset_draws", "draws")]:
            put(sim, k, d[g][t])
        sim.task_step(flags)
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][t])
        np.testing.assert_array_equal(get(sim, "reset_goal_buf"), d["reset_goal"][t])
        np.testing.assert_array_equal(get(sim, "progress_buf"), d["progress"][t])
        np.testing.assert_array_equal(get(sim, "successes"), d["successes"][t])
        np.testing.assert_array_equal(get(sim, "timeout_buf").astype(bool), d["timeout"][t])
        np.testing.assert_allclose(get(sim, "dof_position_targets"), d["targets_after"][t], rtol=0, atol=1e-6)
        np.testing.assert_allclose(get(sim, "dof_state"), d["dof_after"][t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(get(sim, "root_state"), d["root_after"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(get(sim, "goal_state"), d["goal_after"][t], rtol=1e-6, atol=1e-6)
        # fingertip / palm rows come from the device FK here and from the C oracle's FK in the goldens
        close(get(sim, "obs"), d["obs"][t], 1e-5, 2e-5, f"obs step {t}")
        # measured max |d| 1.24e-5 over both subtasks (tools/kuka_tol_probe.py)
        np.testing.assert_allclose(get(sim, "rew"), d["rew"][t], rtol=1e-5, atol=1e-4)
        np.testing.assert_allclose(get(sim, "task_state")[:, :32], d["task_state"][t][:, :32], rtol=1e-5, atol=1e-4)


def _oracle_and_sim(n, seed, force):
    from oracle.oracle_lib import HostState, Oracle
    sim = make_sim(n)
    lo = np.array(sim.model.dof_lower[:23], np.float32)
    up = np.array(sim.model.dof_upper[:23], np.float32)
    scales = get(sim, "object_scale")
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_kuka_scene(st, n, lo, up, list(sim.params.reset_pose), scales, list(sim.model.table_pos), seed=seed,
                           object_force=force)
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums", "task_state", "task_scalars"):
            put(sim, k, st[k])
    from oracle.oracle_lib import Oracle as O
    return sim, O(sim.model, sim.params, n), st


@pytest.mark.parametrize("seed,force,calls", [(0, 0.0, 1), (1, 0.5, 1), (1, 0.5, 10)])
def test_kuka_simulate_matches_oracle_bit_for_bit(seed, force, calls):
    """AllegroKuka physics (per-env cuboid dimensions, object forces) vs the C oracle: bit-identical on every env."""
    n = 128
    sim, orc, st = _oracle_and_sim(n, seed, force)
    sim.simulate(calls)
    orc.simulate(st, calls)
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"kuka seed {seed} force {force} calls {calls}")
    assert np.all(get(sim, "object_force") == 0)                 # consumed by the call, like the oracle


def test_kuka_link_contacts_spill_rows_match_oracle():
    """AllegroKuka on split rows (HA_AK_LINK_SLOTS robot blocks in LDS, the rest in the env's global spill rows):
    the cuboid placed inside the hand, on the palm, touches several links at once, so link contacts go past the
    LDS slots. Bit-identical to the C oracle on every env."""
    n = 128
    sim, orc, st = _oracle_and_sim(n, 2, 0.0)
    sim.simulate(1)                  # link poses of this scene
    m = sim.model
    B, A = m.n_bodies, m.n_actors
    body = get(sim, "rigid_body_state").reshape(n, B, 13)
    palm = int(sim.params.ak_palm_link)
    rs = st["root_state"].reshape(n, A, 13)
    rs[:, m.actor_object0, 0:3] = body[:, m.body_robot0 + palm, 0:3]
    rs[:, m.actor_object0, 7:13] = 0.0
    put(sim, "root_state", st["root_state"])
    for k in ("dof_state", "sim_targets", "contact_cache"):     # (the probe call above wrote manifold records)
        put(sim, k, st[k])
    st0 = st.copy()
    sim.simulate(1)
    orc.simulate(st, 1)
    f = get(sim, "net_contact_force").reshape(n, B, 3)[:, m.body_robot0:m.body_robot0 + m.n_links]
    touched = (np.abs(f).sum(-1) > 0).sum(1)
    print("kuka link-contact scene: robot links in contact per env: median %d, max %d" % (np.median(touched), touched.max()))
    assert touched.max() > 3, "no env has the cuboid on several links"
    # link contacts past the LDS slots (HA_AK_LINK_SLOTS = 9) go to the spill rows: most envs of this scene have more
    link = [int(((c[:, 7] >= 100) | (c[:, 8] >= 100)).sum()) for c in (orc.contacts(st0, e) for e in range(n))]
    assert sum(k > 9 for k in link) > n // 4, link
    scenes.assert_physics_bit_identical(sim, st, n, tag="kuka link contacts")


@pytest.mark.parametrize("sub", ["regrasping", "reorientation", "throw"])
def test_kuka_vectask_episode_at_full_size(sub):
    """C2 size (4096 envs): first step resets every env, then 150 random-action steps through the fused kernel;
    everything finite, observations within the +-10 clamp, cuboids stay in the scene, resets happen."""
    need_gpu()
    from handarm_hip.tasks import isaacgym_task_map
    n = 4096
    env = isaacgym_task_map["AllegroKuka"]({"env": {"numEnvs": n, "subtask": sub}}, "cuda:0", "cuda:0")
    obs = env.reset()["obs"]
    assert obs.shape == (n, 117 if sub == "reorientation" else 99)
    g = torch.Generator(device="cuda:0").manual_seed(7)
    resets = 0
    for step in range(150):
        a = torch.rand((n, 23), device="cuda:0", generator=g) * 2 - 1
        obs_dict, rew, reset, extras = env.step(a)
        resets += int(reset.sum())
    torch.cuda.synchronize()
    o = obs_dict["obs"]
    assert torch.isfinite(o).all() and torch.isfinite(rew).all()
    assert o.abs().max() <= 10.0
    z = env.root_state_tensor.view(n, 4, 13)[:, 1, 2]
    # random arm actions (relative targets, up to 10 rad/s) can bat a 50 g cuboid far away; the bulk of the
    # cuboids stays on the table or in the hand, nothing sinks through the ground
    assert (z > -0.01).all() and torch.isfinite(env.root_state_tensor).all()
    assert float(torch.quantile(z, 0.5)) > 0.4 and float(torch.quantile(z, 0.99)) < 2.0
    assert resets > 0
    assert float(extras["true_objective_mean"]) >= 0.0
    lifted = float(env.lifted_object.mean())
    q = [float(torch.quantile(z, f)) for f in (0.0, 0.01, 0.5, 0.99, 1.0)]
    print(f"kuka {sub} full-size: resets {resets}, lifted {lifted:.3f}, z quantiles 0/1/50/99/100% {q}")


def test_apply_rigid_body_force_tensors_local_space():
    """gym.apply_rigid_body_force_tensors(LOCAL_SPACE) through gym_api: a free cuboid (clear of the scene)
    gains R(q) F / m dt on top of gravity in one simulate call, and the force is consumed by it."""
    need_gpu()
    from handarm_hip.gym_api import acquire_gym, gymapi, gymtorch
    n = 64
    gym = acquire_gym()
    sim = gym.create_sim(n, "cuda:0", task=HM.TASK_ALLEGRO_KUKA)
    rng = np.random.default_rng(0)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim)).view(n, 4, 13)
    q = rng.standard_normal((n, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    root[:, 1, 0:3] = torch.tensor([0.0, -0.6, 1.5], device="cuda:0")
    root[:, 1, 3:7] = torch.from_numpy(q).cuda()
    root[:, 1, 7:13] = 0
    f_local = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    forces = torch.zeros((n * 27, 3), device="cuda:0")
    forces.view(n, 27, 3)[:, 24] = torch.from_numpy(f_local).cuda()
    gym.apply_rigid_body_force_tensors(sim, gymtorch.unwrap_tensor(forces), None, gymapi.LOCAL_SPACE)
    gym.simulate(sim)
    v = get(sim, "root_state").reshape(n, 4, 13)[:, 1, 7:10]
    from scipy.spatial.transform import Rotation
    f_world = Rotation.from_quat(q).apply(f_local)
    mass = 400.0 * 0.05 ** 3 * get(sim, "object_scale").reshape(n, 3).prod(-1)
    dt = sim.params.dt
    exp = f_world / mass[:, None] * dt + np.array([0.0, 0.0, -9.81]) * dt
    np.testing.assert_allclose(v, exp, rtol=1e-3, atol=1e-5)
    assert np.all(get(sim, "object_force") == 0)


def test_create_rejects_hulls_beyond_the_family_scratch():
    """The Allegro families' narrow-phase scratch holds hulls of <= 32 vertices / 64 planes (ColLayout): ha_create
    refuses a model with a larger hull instead of overrunning LDS."""
    need_gpu()
    import ctypes as C
    from handarm_hip import _lib
    scene = HM.load_scene(HM.KUKA_ASSET)
    model = HM.build_model(scene)
    params, _ = HM.build_params(task=HM.TASK_ALLEGRO_KUKA)
    lib = _lib.load()
    h = C.c_void_p()
    assert lib.ha_create(C.byref(model), C.byref(params), 4, C.byref(h)) == 0
    lib.ha_destroy(h)
    model.hull_nverts[0] = 40
    h2 = C.c_void_p()
    assert lib.ha_create(C.byref(model), C.byref(params), 4, C.byref(h2)) != 0


def test_create_rejects_compound_pool_objects():
    """The AllegroKuka env block has no compound-object gather buffer (PhysCfg NG = 0): ha_create refuses a pool
    object made of several hulls (HA_E_MODEL) instead of writing past the family's narrow-phase scratch."""
    need_gpu()
    import ctypes as C
    from handarm_hip import _lib
    scene = HM.load_scene(HM.KUKA_ASSET)
    model = HM.build_model(scene)
    params, _ = HM.build_params(task=HM.TASK_ALLEGRO_KUKA)
    lib = _lib.load()
    assert model.pool_hull[0] + 2 <= model.n_hulls
    model.pool_nhull[0] = 2
    h = C.c_void_p()
    assert lib.ha_create(C.byref(model), C.byref(params), 4, C.byref(h)) == -4      # HA_E_MODEL


def test_kuka_friction_cone_on_the_gpu():
    """The Coulomb-friction schedule of test_kuka_physics.py on the kernel: static friction holds a push at half
    the limit, a push at 1.25 times it slides the cuboid with (1.25 - 1) mu g, upright; and the whole 68-call
    trajectory stays bit-identical to the C oracle."""
    from tests.test_kuka_physics import check_friction, friction_schedule
    n = 24
    sim, orc, st = _oracle_and_sim(n, 0, 0.0)
    scales = get(sim, "object_scale").reshape(n, 1, 3)
    root = st["root_state"].reshape(n, 4, 13)
    root[:, 1, 7:13] = 0
    root[:, 1, 3:7] = [0, 0, 0, 1]
    root[:, 1, 0:2] = [0.13, -0.09]
    root[:, 1, 2] = 0.53 + 0.025 * scales[:, 0, 2] + 0.002
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums", "task_state", "task_scalars"):
            put(sim, k, st[k])
    mu, dt = sim.params.friction, sim.params.dt

    def gpu_force(f):
        sim.t["object_force"].view(n, -1, 3)[:, 0] = torch.from_numpy(f).cuda()

    flat, rec = friction_schedule(n, scales, mu, dt, lambda: sim.simulate(1),
                                  lambda: get(sim, "root_state").reshape(n, 4, 13),
                                  lambda: sim.t["dof_state"].view(n, 23, 2), gpu_force)
    check_friction(flat, rec, mu, dt)

    def cpu_force(f):
        st["object_force"].reshape(n, -1, 3)[:, 0] = f

    friction_schedule(n, scales, mu, dt, lambda: orc.simulate(st, 1), lambda: st["root_state"].reshape(n, 4, 13),
                      lambda: st["dof_state"].reshape(n, 23, 2), cpu_force)
    scenes.assert_physics_bit_identical(sim, st, n, tag="kuka friction schedule")


def test_kuka_dropped_cuboids_on_the_gpu():
    """The drop schedule of test_kuka_physics.py on the kernel: bounded penetration at impact, no bounce, rest at
    the contact slop, upright; bit-identical to the C oracle after the 60 calls."""
    from tests.test_kuka_physics import check_drop, drop_schedule
    n = 24
    sim, orc, st = _oracle_and_sim(n, 0, 0.0)
    scales = get(sim, "object_scale").reshape(n, 1, 3)
    root = st["root_state"].reshape(n, 4, 13)
    root[:, 1, 7:13] = 0
    root[:, 1, 3:7] = [0, 0, 0, 1]
    root[:, 1, 0:2] = [0.13, -0.09]
    root[:, 1, 2] = 0.53 + 0.025 * scales[:, 0, 2] + 0.10
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums", "task_state", "task_scalars"):
            put(sim, k, st[k])
    flat, zs = drop_schedule(n, scales, lambda: sim.simulate(1), lambda: get(sim, "root_state").reshape(n, 4, 13),
                             lambda: sim.t["dof_state"].view(n, 23, 2))
    check_drop(flat, zs, get(sim, "root_state").reshape(n, 4, 13), sim.params.contact_slop)
    drop_schedule(n, scales, lambda: orc.simulate(st, 1), lambda: st["root_state"].reshape(n, 4, 13),
                  lambda: st["dof_state"].reshape(n, 23, 2))
    scenes.assert_physics_bit_identical(sim, st, n, tag="kuka drop schedule")


def test_throw_bucket_catches_cuboids_bit_identical_to_oracle():
    """Throw physics on the kernel (ak_simulate_kernel): cuboids of the throw family dropped into buckets hanging at
    per-env places of the arena (the posed statics read each env's actor-3 root state) come to rest on the bucket
    floor, and after 60 calls every physics output is bit-identical to the C oracle; then half the buckets move
    (as _reset_target does between calls) and the next 10 calls stay bit-identical."""
    from oracle.oracle_lib import HostState, Oracle
    n = 64
    sim = make_sim(n, subtask="throw")
    m = sim.model
    assert m.n_static == 14 and m.posed_actor == m.actor_goal
    lo = np.array(m.dof_lower[:23], np.float32)
    up = np.array(m.dof_upper[:23], np.float32)
    st = HostState(n, model=m, params=sim.params)
    scales = get(sim, "object_scale")
    scenes.fill_kuka_scene(st, n, lo, up, list(sim.params.reset_pose), scales, list(m.table_pos), seed=3)
    rng = np.random.default_rng(3)
    root = st["root_state"].reshape(n, 4, 13)
    side = np.where(np.arange(n) % 2 == 0, 1.0, -1.0)
    root[:, 3] = 0
    root[:, 3, 0] = side * rng.uniform(0.55, 0.9, n)
    root[:, 3, 1] = rng.uniform(-1.0, 0.7, n)
    root[:, 3, 2] = rng.uniform(0.0, 1.0, n)
    root[:, 3, 6] = 1
    root[:, 1] = 0
    root[:, 1, 0:3] = root[:, 3, 0:3] + np.c_[rng.uniform(-0.02, 0.02, (n, 2)), np.full(n, 0.15)]
    q = rng.standard_normal((n, 4)).astype(np.float32) * [0.1, 0.1, 0.1, 1.0]
    root[:, 1, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums", "task_state", "task_scalars"):
            put(sim, k, st[k])
    orc = Oracle(m, sim.params, n)
    sim.simulate(60)
    orc.simulate(st, 60)
    scenes.assert_physics_bit_identical(sim, st, n, tag="throw bucket drop")
    obj = get(sim, "root_state").reshape(n, 4, 13)[:, 1]
    b = root[:, 3, 0:3]
    dz = obj[:, 2] - b[:, 2]
    inside = np.hypot(obj[:, 0] - b[:, 0], obj[:, 1] - b[:, 1] + 0.002016) < 0.1
    print(f"throw bucket drop: {inside.mean():.2f} inside, height above the bucket origin "
          f"{np.quantile(dz, [0, 0.5, 1]).round(4).tolist()}")
    assert inside.mean() > 0.9 and (dz[inside] > 0.009).all() and (dz[inside] < 0.2).all()
    root[::2, 3, 0] += 0.4
    put(sim, "root_state", st["root_state"])
    sim.simulate(10)
    orc.simulate(st, 10)
    scenes.assert_physics_bit_identical(sim, st, n, tag="throw buckets moved")
    obj2 = get(sim, "root_state").reshape(n, 4, 13)[:, 1]
    high = root[::2, 3, 2] > 0.1                                # (a bucket on the ground has nothing to fall from)
    assert high.sum() > 8 and (obj2[::2, 2][high] < obj[::2, 2][high] - 0.05).all()   # the moved buckets' cuboids fall
