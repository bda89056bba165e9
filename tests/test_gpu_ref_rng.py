"""The VecTask classes with cfg sim.reference_rng on the GPU: seeded like the reference, their own host draws
(handarm_hip/ref_rng.py) drive the fused kernels, and the steps reproduce the reference's reset indexing and
reset states bit for bit (north_star: "bit-exact for done masks / reset indexing" on identical seeds).

* HandArm (Ur5Sih): four episodes from torch.manual_seed(seed); target_object_index,
  object_configuration_indices and goal_pos after every reset equal the reference's reset_idx from the same seed
  (tests/golden/ur5sih_ref_rng.npz).
* AllegroKuka / AllegroHand: the reference-generated step goldens, replayed through env.step() with the physics
  call switched off (FLAG_NO_PHYSICS, as the goldens have no PhysX): resets, goals, forces and observations
  come out of the product's own draws, not the recorded ones.
"""
import os

import numpy as np
import pytest
import torch

from handarm_hip import model as HM

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def get(sim, name):
    return sim.t[name].cpu().numpy()


def test_ur5sih_reference_rng_episodes():
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    d = np.load(os.path.join(G, "ur5sih_ref_rng.npz"))
    E, N = d["target_idx"].shape
    L = 3
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": N}, "seed": 0, "sim": {"reference_rng": True},
                                         "objects": {"drop": {"num_initial_poses": int(d["num_initial_poses"])}},
                                         "rl": {"reset": {"max_episode_length": L}}}, "cuda:0", "cuda:0")
    # objects already dropped (the drop draws are checked on the CPU: their count depends on the physics)
    env.objects_dropped = True
    put(env.sim, "object_pos_initial", d["object_pos_initial"])
    put(env.sim, "object_quat_initial", d["object_quat_initial"])
    torch.manual_seed(int(d["seed"]))
    gen = torch.Generator(device="cuda:0").manual_seed(3)
    e = -1
    for _ in range(E * L):
        resetting = bool(env.reset_buf.any())
        env.step(torch.rand((N, 11), device="cuda:0", generator=gen) * 2 - 1)
        if resetting:
            e += 1
            np.testing.assert_array_equal(get(env.sim, "target_object_index"), d["target_idx"][e])
            np.testing.assert_array_equal(get(env.sim, "object_configuration_indices"), d["cfg_idx"][e])
            np.testing.assert_array_equal(get(env.sim, "goal_pos"), d["goal_pos"][e])
    assert e == E - 1


@pytest.mark.parametrize("sub", ["regrasping", "reorientation", "throw"])
def test_kuka_reference_rng_steps(sub):
    need_gpu()
    from handarm_hip.tasks import AllegroKuka
    d = np.load(os.path.join(G, f"kuka_steps_{sub}.npz"))
    T, N = d["rew"].shape
    torch.manual_seed(int(d["seed"]))                   # before the task: its __init__ draws random_force_prob
    env = AllegroKuka({"env": {"numEnvs": N, "subtask": sub}, "sim": {"reference_rng": True}}, "cuda:0", "cuda:0")
    np.testing.assert_array_equal(env.random_force_prob.cpu().numpy(), d["random_force_prob_init"])
    env.sim_flags = HM.FLAG_NO_PHYSICS
    sim = env.sim
    for t in range(T):
        for k, g in [("dof_state", "dof_state"), ("root_state", "root_state"), ("goal_state", "goal_state"),
                     ("dof_position_targets", "targets"), ("sim_targets", "targets"), ("reset_buf", "reset_in"),
                     ("reset_goal_buf", "reset_goal_in"), ("progress_buf", "progress_in"),
                     ("successes", "successes_in"), ("task_state", "task_state_in")]:
            put(sim, k, d[g][t])
        env.step(torch.as_tensor(d["actions"][t], device="cuda:0"))
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][t])
        np.testing.assert_array_equal(get(sim, "reset_goal_buf"), d["reset_goal"][t])
        np.testing.assert_array_equal(get(sim, "progress_buf"), d["progress"][t])
        np.testing.assert_array_equal(get(sim, "successes"), d["successes"][t])
        np.testing.assert_allclose(get(sim, "dof_state"), d["dof_after"][t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(get(sim, "root_state"), d["root_after"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(get(sim, "goal_state"), d["goal_after"][t], rtol=1e-6, atol=1e-6)
        # random forces (rb_forces, LOCAL_SPACE) live in the task_state row
        np.testing.assert_allclose(get(sim, "task_state")[:, HM.AK_RB_FORCE:HM.AK_RB_FORCE + 3],
                                   d["task_state"][t][:, HM.AK_RB_FORCE:HM.AK_RB_FORCE + 3], rtol=1e-6, atol=1e-7)


def test_allegro_reference_rng_steps():
    need_gpu()
    from handarm_hip.tasks import AllegroHand
    d = np.load(os.path.join(G, "allegro_steps.npz"))
    T, N = d["rew"].shape
    torch.manual_seed(int(d["seed"]))
    env = AllegroHand({"env": {"numEnvs": N}, "sim": {"reference_rng": True}}, "cuda:0", "cuda:0")
    env.sim_flags = HM.FLAG_NO_PHYSICS
    sim = env.sim
    for k, g in [("dof_state", "dof_state"), ("goal_state", "goal_state"), ("dof_position_targets", "targets"),
                 ("reset_buf", "reset_in"), ("reset_goal_buf", "reset_goal_in"), ("successes", "successes_in")]:
        put(sim, k, d[g][0])
    for t in range(T):
        put(sim, "root_state", d["root_state"][t])
        put(sim, "progress_buf", d["progress_in"][t])
        env.step(torch.as_tensor(d["actions"][t], device="cuda:0"))
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][t])
        np.testing.assert_array_equal(get(sim, "reset_goal_buf"), d["reset_goal"][t])
        np.testing.assert_array_equal(get(sim, "progress_buf"), d["progress"][t])
        np.testing.assert_allclose(get(sim, "dof_state"), d["dof_after"][t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(get(sim, "root_state"), d["root_after"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(get(sim, "obs"), d["obs"][t], rtol=1e-5, atol=2e-6)


def test_ur5sih_reference_rng_draw_order_with_point_clouds(monkeypatch):
    """With sim.reference_rng and a point-cloud observation list, the CPU generator sees the reference's draw order
    (ADVICE round 2): the clouds' torch.randperm of ConfigurableVecTask.__init__'s post_step
    (configurable_vec_task.py:43-44, multi_object.py:806) before any drop draw, every drop's position / rotation
    draws (multi_object_manipulation.py:107-110), one randperm after each initial pose's settle (:149-150), and
    only then the first reset_idx draws (:62-91). The draws go through the recorded wrappers unchanged."""
    need_gpu()
    from handarm_hip import ref_rng as RR
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    seq = []
    real_perm, real_drop, real_reset = torch.randperm, RR.ur5sih_drop_pose, RR.ur5sih_reset_draws

    def perm(*a, **k):
        if "device" not in k and "generator" not in k:
            seq.append("perm")
        return real_perm(*a, **k)

    def drop(n, *a, **k):
        seq.append("drop")
        return real_drop(n, *a, **k)

    def reset(*a, **k):
        seq.append("reset")
        return real_reset(*a, **k)

    monkeypatch.setattr(torch, "randperm", perm)
    monkeypatch.setattr(RR, "ur5sih_drop_pose", drop)
    monkeypatch.setattr(RR, "ur5sih_reset_draws", reset)
    P, N = 2, 16
    obs = ["goal_pos", "ur5_flange_pose", "dof_position_targets", "object_synthetic_pointcloud",
           "ur5sih_synthetic_pointcloud", "goal_synthetic_pointcloud"]
    torch.manual_seed(5)
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": N, "observations": obs}, "sim": {"reference_rng": True},
                                         "objects": {"drop": {"num_initial_poses": P}}}, "cuda:0", "cuda:0")
    env.reset()
    env.step(torch.zeros((N, env.num_acts), device="cuda:0"))
    first_reset = seq.index("reset")
    head = seq[:first_reset]
    assert head[0] == "perm" and head[-1] == "perm" and head.count("perm") == P + 1, head
    # each pose's drop draws form one run between two randperms
    runs = "".join("p" if x == "perm" else "d" for x in head).split("p")[1:-1]
    assert len(runs) == P and all(len(r) >= env.num_objects for r in runs), head


@pytest.mark.parametrize("variant,env_cfg", [("force", {"forceScale": 1.0}), ("pen", {"objectType": "pen"})])
def test_allegro_reference_rng_variants(variant, env_cfg):
    """reference_rng through env.step() for forceScale 1 (the force selection and normals drawn on the host in the
    reference's order) and objectType pen (randomize_rotation_pen): allegro_variants.npz, physics off."""
    need_gpu()
    from handarm_hip.tasks import AllegroHand
    g = np.load(os.path.join(G, "allegro_variants.npz"))
    d = {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith(variant + "/")}
    T, N = d["rew"].shape
    torch.manual_seed(int(d["seed"]))
    env = AllegroHand({"env": dict({"numEnvs": N}, **env_cfg), "sim": {"reference_rng": True}}, "cuda:0", "cuda:0")
    env.sim_flags = HM.FLAG_NO_PHYSICS
    sim = env.sim
    for k, gk in [("dof_state", "dof_state"), ("goal_state", "goal_state"), ("dof_position_targets", "targets"),
                  ("reset_buf", "reset_in"), ("reset_goal_buf", "reset_goal_in"), ("successes", "successes_in")]:
        put(sim, k, d[gk][0])
    for t in range(T):
        put(sim, "root_state", d["root_state"][t])
        put(sim, "progress_buf", d["progress_in"][t])
        env.step(torch.as_tensor(d["actions"][t], device="cuda:0"))
        np.testing.assert_array_equal(get(sim, "reset_buf"), d["reset"][t])
        np.testing.assert_allclose(get(sim, "root_state"), d["root_after"][t], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(get(sim, "obs"), d["obs"][t], rtol=1e-5, atol=2e-6)
        if variant == "force":
            np.testing.assert_allclose(get(sim, "task_state")[:, 0:3], d["force_after"][t], rtol=1e-6, atol=1e-9)
