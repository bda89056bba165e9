"""GPU parity for the AllegroHand task (config C3), through the C ABI:
* task math (observe / reward / resets / targets) against the reference-generated goldens
  (bit-exact done masks and counters; float tolerances stated per check);
* physics against the C oracle after one gym.simulate (1-ulp-sensitivity-calibrated tolerance, as for
  Ur5Sih), and physical properties over a full-size episode.
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
    cfg = dict(cfg, task=HM.TASK_ALLEGRO_HAND)
    return HandArmSim(n, "cuda:0", task_cfg=cfg, task=HM.TASK_ALLEGRO_HAND)


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def get(sim, name):
    torch.cuda.synchronize()
    return sim.t[name].cpu().numpy()


def test_allegro_observe_and_reward_against_reference_goldens():
    d = np.load(os.path.join(G, "allegro_obs_reward.npz"))
    S, N = d["rew"].shape
    sim = make_sim(N)
    for s in range(S):
        for k, g in [("dof_state", "dof_state"), ("dof_force", "dof_force"), ("root_state", "root_state"),
                     ("goal_state", "goal_state"), ("actions", "actions"), ("reset_buf", "reset_in"),
                     ("reset_goal_buf", "reset_goal_in"), ("progress_buf", "progress_in"),
                     ("successes", "successes_in")]:
            put(sim, k, d[g][s])
        sim.task_observe(0)
        np.testing.assert_allclose(get(sim, "obs"), d["obs"][s], rtol=1e-5, atol=2e-6)
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][s])
        np.testing.assert_array_equal(get(sim, "reset_goal_buf"), d["reset_goal"][s])
        np.testing.assert_array_equal(get(sim, "progress_buf"), d["progress"][s])
        np.testing.assert_array_equal(get(sim, "successes"), d["successes"][s])
        np.testing.assert_allclose(get(sim, "rew"), d["rew"][s], rtol=1e-5, atol=1e-4)
        # consecutive_successes inputs of the step: number of resets and sum(successes * resets)
        stats, terms = get(sim, "stats")[0], get(sim, "term_sums")[0]
        assert stats[0] == d["reset"][s].sum()
        np.testing.assert_allclose(terms[0], (d["successes"][s] * d["reset"][s]).sum(), rtol=1e-6)


def test_allegro_step_with_resets_replayed_against_reference_goldens():
    """The fused step kernel without physics: goal + env resets from the recorded reference draws,
    targets from the actions, progress, full_state observations, reward, done, timeout, EWMA."""
    d = np.load(os.path.join(G, "allegro_steps.npz"))
    T, N = d["rew"].shape
    sim = make_sim(N)
    for k, g in [("dof_state", "dof_state"), ("goal_state", "goal_state"), ("dof_position_targets", "targets"),
                 ("reset_buf", "reset_in"), ("reset_goal_buf", "reset_goal_in"), ("successes", "successes_in")]:
        put(sim, k, d[g][0])
    flags = HM.FLAG_NO_PHYSICS | HM.FLAG_REPLAY_DRAWS
    for t in range(T):
        put(sim, "root_state", d["root_state"][t])       # the generator's stand-in for physics between steps
        put(sim, "progress_buf", d["progress_in"][t])
        put(sim, "actions", d["actions"][t])
        dr = np.zeros((N, HM.DRAW_STRIDE), np.float32)        # goldens hold the 48 AllegroHand slots
        dr[:, :d["draws"].shape[-1]] = d["draws"][t]
        put(sim, "reset_draws", dr)
        sim.task_step(flags)
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][t])
        np.testing.assert_array_equal(get(sim, "reset_goal_buf"), d["reset_goal"][t])
        np.testing.assert_array_equal(get(sim, "progress_buf"), d["progress"][t])
        np.testing.assert_array_equal(get(sim, "successes"), d["successes"][t])
        np.testing.assert_array_equal(get(sim, "timeout_buf").astype(bool), d["timeout"][t])
        np.testing.assert_allclose(get(sim, "dof_position_targets"), d["targets_after"][t], rtol=0, atol=1e-6)
        np.testing.assert_allclose(get(sim, "sim_targets"), d["targets_after"][t], rtol=0, atol=1e-6)
        np.testing.assert_allclose(get(sim, "dof_state"), d["dof_after"][t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(get(sim, "root_state"), d["root_after"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(get(sim, "obs"), d["obs"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(get(sim, "rew"), d["rew"][t], rtol=1e-5, atol=1e-4)
        np.testing.assert_allclose(get(sim, "consecutive_successes")[0], d["cons"][t][0], rtol=1e-6)


@pytest.mark.parametrize("variant,cfg", [("full_rel", dict(obs_type="full", relative_control=True)),
                                         ("novel_asym", dict(obs_type="full_no_vel", asymmetric=True)),
                                         ("force", dict(force_scale=1.0)),
                                         ("egg", dict(object_type="egg")), ("pen", dict(object_type="pen"))])
def test_allegro_observation_types_and_relative_control_against_reference_goldens(variant, cfg):
    """The same fused step without physics for observationType "full" (72) + useRelativeControl, "full_no_vel"
    (50) + asymmetric_observations (the states buffer: teacher_obs, 88 floats), forceScale 1 (the object force and
    random_force_prob in task_state) and objectType egg / pen (allegro_variants.npz)."""
    g = np.load(os.path.join(G, "allegro_variants.npz"))
    d = {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith(variant + "/")}
    T, N = d["rew"].shape
    sim = make_sim(N, **cfg)
    assert sim.t["obs"].shape[1] == d["obs"].shape[-1]
    for k, gk in [("dof_state", "dof_state"), ("goal_state", "goal_state"), ("dof_position_targets", "targets"),
                  ("reset_buf", "reset_in"), ("reset_goal_buf", "reset_goal_in"), ("successes", "successes_in")]:
        put(sim, k, d[gk][0])
    flags = HM.FLAG_NO_PHYSICS | HM.FLAG_REPLAY_DRAWS
    for t in range(T):
        put(sim, "root_state", d["root_state"][t])
        put(sim, "progress_buf", d["progress_in"][t])
        put(sim, "actions", d["actions"][t])
        dr = np.zeros((N, HM.DRAW_STRIDE), np.float32)
        dr[:, :d["draws"].shape[-1]] = d["draws"][t]
        put(sim, "reset_draws", dr)
        sim.task_step(flags)
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][t])
        np.testing.assert_array_equal(get(sim, "timeout_buf").astype(bool), d["timeout"][t])
        np.testing.assert_allclose(get(sim, "dof_position_targets"), d["targets_after"][t], rtol=0, atol=1e-6)
        np.testing.assert_allclose(get(sim, "obs"), d["obs"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(get(sim, "rew"), d["rew"][t], rtol=1e-5, atol=1e-4)
        if cfg.get("asymmetric"):
            np.testing.assert_allclose(get(sim, "teacher_obs"), d["states"][t], rtol=1e-5, atol=2e-6)
        ts = get(sim, "task_state")
        np.testing.assert_allclose(ts[:, 3], d["prob_after"][t], rtol=1e-6)          # random_force_prob
        if cfg.get("force_scale", 0) > 0:                                           # rb_forces of the object body
            np.testing.assert_allclose(ts[:, 0:3], d["force_after"][t], rtol=1e-6, atol=1e-9)


def test_allegro_vectask_asymmetric_relative_episode():
    """VecTask surface with the options: obs_dict["obs"] 50 wide, obs_dict["states"] the clamped 88-float states,
    num_states 88; relative control moves the targets by at most dofSpeedScale * dt per step."""
    need_gpu()
    from handarm_hip.tasks import isaacgym_task_map
    n = 256
    env = isaacgym_task_map["AllegroHand"]({"env": {"numEnvs": n, "observationType": "full_no_vel",
                                                    "asymmetric_observations": True, "useRelativeControl": True}},
                                           "cuda:0", "cuda:0")
    assert (env.num_obs, env.num_states) == (50, 88)
    o = env.reset()
    assert o["obs"].shape == (n, 50) and o["states"].shape == (n, 88)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    _, _, d, _ = env.step(torch.zeros((n, 16), device="cuda:0"))
    for _ in range(20):
        prev, was_reset = env.prev_targets.clone(), d.bool().clone()      # envs flagged now reset in the next step
        o, r, d, e = env.step(torch.rand((n, 16), device="cuda:0", generator=g) * 2 - 1)
        moved = (env.prev_targets - prev).abs()[~was_reset]
        assert moved.max().item() <= 20.0 * 0.01667 + 1e-5
        assert o["states"].shape == (n, 88) and torch.isfinite(o["states"]).all()
        assert o["states"].abs().max().item() <= 5.0 and torch.isfinite(o["obs"]).all()
        # the states' object pose columns are the observation's (full_state 48:55 vs full_no_vel 16:23)
        torch.testing.assert_close(o["states"][:, 48:55], o["obs"][:, 16:23])


@pytest.mark.parametrize("obj", ["egg", "pen"])
def test_allegro_egg_and_pen_episode(obj):
    """objectType egg / pen through the VecTask surface: the pool entry in every env, its hull and mass in the physics
    (tools/build_model.py build_egg / build_pen), 60 random-action steps stay finite with the object held or dropped
    onto nothing (no table: a dropped object falls and the env resets), and the physics matches the C oracle bit for
    bit for one gym.simulate of the reset scene."""
    need_gpu()
    from handarm_hip.tasks import isaacgym_task_map
    from oracle.oracle_lib import HostState, Oracle
    n = 256
    env = isaacgym_task_map["AllegroHand"]({"env": {"numEnvs": n, "objectType": obj}}, "cuda:0", "cuda:0")
    assert (env.sim.t["object_indices"] == HM.AH_OBJECT_TYPES[obj]).all()
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(4)
    resets = 0
    for _ in range(60):
        o, r, d, e = env.step(torch.rand((n, 16), device="cuda:0", generator=g) * 2 - 1)
        assert torch.isfinite(o["obs"]).all() and torch.isfinite(r).all()
        resets += int(d.sum())
    assert resets > 0
    sim = env.sim
    hs = HostState(n, model=sim.model, params=sim.params)
    torch.cuda.synchronize()
    for k in HM.STATE_FIELDS:
        if k in hs.arrays and k in sim.t and sim.t[k].numel() == hs[k].size:
            hs[k][...] = sim.t[k].cpu().numpy().reshape(hs[k].shape)
    sim.simulate(1)
    Oracle(sim.model, sim.params, n).simulate(hs, 1)
    scenes.assert_physics_bit_identical(sim, hs, n, tag=obj)


def _oracle_and_sim(n, seed):
    from oracle.oracle_lib import HostState, Oracle
    sim = make_sim(n)
    lo = np.array(sim.model.dof_lower[:16], np.float32)
    up = np.array(sim.model.dof_upper[:16], np.float32)
    st = HostState(n, model=sim.model, params=sim.params)
    scenes.fill_allegro_scene(st, n, lo, up, seed=seed)
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums"):
            put(sim, k, st[k])
    return sim, Oracle(sim.model, sim.params, n), st


@pytest.mark.parametrize("seed,calls", [(0, 1), (1, 1), (1, 10)])
def test_allegro_simulate_matches_oracle_bit_for_bit(seed, calls):
    """AllegroHand physics vs the C oracle: bit-identical on every env, joint forces (dof_force) included."""
    n = 128
    sim, orc, st = _oracle_and_sim(n, seed)
    sim.simulate(calls)
    orc.simulate(st, calls)
    scenes.assert_physics_bit_identical(sim, st, n, tag=f"allegro seed {seed} calls {calls}")


def test_allegro_vectask_episode_at_full_size():
    """C3 size (16384 envs): reset -> 120 random-action steps; everything finite, cube mostly held or
    dropped onto the ground, fall resets fire, consecutive_successes stays a finite average."""
    need_gpu()
    from handarm_hip.tasks import AllegroHand
    n = 16384
    env = AllegroHand({"env": {"numEnvs": n}}, "cuda:0", "cuda:0")
    obs = env.reset()["obs"]
    assert obs.shape == (n, 88)
    g = torch.Generator(device="cuda:0").manual_seed(42)
    resets = 0
    for step in range(120):
        a = torch.rand((n, 16), device="cuda:0", generator=g) * 2 - 1
        obs_dict, rew, reset, extras = env.step(a)
        resets += int(reset.sum())
    torch.cuda.synchronize()
    o = obs_dict["obs"]
    assert torch.isfinite(o).all() and torch.isfinite(rew).all()
    assert o.abs().max() <= 5.0                                   # clipObservations
    z = env.root_state_tensor.view(n, 3, 13)[:, 1, 2]
    assert (z > 0.0).all() and (z < 1.0).all()
    assert resets > 0                                             # the first step resets every env; falls later
    cs = float(extras["consecutive_successes"])
    assert np.isfinite(cs) and cs >= 0.0
    print(f"allegro full-size: resets {resets}, consecutive_successes {cs:.3f}, "
          f"cube z in [{float(z.min()):.3f}, {float(z.max()):.3f}]")
