"""GPU parity of the synthetic point clouds (ha_pointclouds) and the custom observation vector (ha_gather_obs),
called through the C ABI: against the reference goldens (tests/golden/ur5sih_pointclouds_*.npz, made by the
reference's own post_physics_step), against the numpy oracle at a larger size, and through the VecTask with the
point-cloud student list (Ur5SihMultiObjectManipulation.yaml:45).

Tolerance: posed point coordinates within 2e-7 absolute of the goldens (torch CPU may fuse a multiply-add in
its cross products) and within 1e-7 of the oracle (same operation order, -ffp-contract=off); point types,
goal / fingertip clouds, padding and the obs-vector gather bit-exact."""
import os

import numpy as np
import pytest
import torch

from handarm_hip import model as HM
from handarm_hip import observables as OB
from handarm_hip import pointclouds as PCM
from oracle import task_oracle as O

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def cpu(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.mark.parametrize("case", ["student", "all"])
def test_clouds_against_reference_goldens(case):
    need_gpu()
    from handarm_hip.sim import HandArmSim
    d = np.load(os.path.join(G, f"ur5sih_pointclouds_{case}.npz"))
    names = [str(n) for n in d["observations"]]
    pool = [str(n) for n in d["pool"]]
    steps, n = d["target_idx"].shape
    sim = HandArmSim(n, "cuda:0", pool_names=pool)
    order = [str(x) for x in d["post_step_order"]]
    pcs = PCM.SyntheticPointclouds(sim, [x for x in names if x in OB.POINTCLOUDS], pool)
    prev = OB.sees_previous_object_pose(order, "object_synthetic_pointcloud")
    if prev:
        pcs.use_previous_object_pose()
    put(sim, "object_indices", d["object_indices"])
    for s in range(steps):
        put(sim, "root_state", d["root"][s])
        put(sim, "rigid_body_state", d["body"][s])
        put(sim, "goal_pos", d["goal_pos"][s])
        put(sim, "target_object_index", d["target_idx"][s])
        if prev:
            pp = np.zeros((n, 3, 7), np.float32) if s == 0 else d["root"][s - 1].reshape(n, 6, 13)[:, 3:6, 0:7]
            pcs.snapshot_object_pose(torch.from_numpy(np.ascontiguousarray(pp)).cuda())
        pcs.refresh(perm=d["perm"][s])
        for x in pcs.names:
            got = cpu(pcs.outputs[x])
            want = d[x][s]
            np.testing.assert_array_equal(got[..., 3], want[..., 3], err_msg=x)
            np.testing.assert_allclose(got, want, rtol=0, atol=2e-7, err_msg=x)


def test_clouds_against_oracle_2048():
    """Every cloud at 2048 envs on random states against the numpy oracle; invalid device indices do not fault."""
    need_gpu()
    from handarm_hip.sim import HandArmSim
    N = 2048
    rng = np.random.default_rng(7)
    scene = HM.load_scene()
    pool = [o["name"] for o in scene["objects"]]
    sim = HandArmSim(N, "cuda:0", pool_names=pool)
    pcs = PCM.SyntheticPointclouds(sim, OB.POINTCLOUDS, pool)
    root = rng.standard_normal((N, 6, 13)).astype(np.float32)
    root[..., 3:7] /= np.linalg.norm(root[..., 3:7], axis=-1, keepdims=True)
    body = rng.standard_normal((N, sim.num_bodies, 13)).astype(np.float32)
    body[..., 3:7] /= np.linalg.norm(body[..., 3:7], axis=-1, keepdims=True)
    oi = np.stack([rng.permutation(len(pool))[:3] for _ in range(N)])
    tgt = rng.integers(0, 3, N)
    goal = rng.random((N, 3), dtype=np.float32)
    perm = rng.permutation(pcs.P)
    for k, v in [("root_state", root), ("rigid_body_state", body), ("object_indices", oi),
                 ("target_object_index", tgt), ("goal_pos", goal)]:
        put(sim, k, v)
    pcs.refresh(perm=perm)
    table = PCM.object_sample_table(pool)
    a = np.load(PCM.ASSET)
    obj = O.object_pointcloud(root[:, 3:6, 0:7], table[oi], perm)
    want = {"object_synthetic_pointcloud": obj,
            "target_object_synthetic_pointcloud": O.target_pointcloud(obj, tgt, 3),
            "ur5sih_synthetic_pointcloud": O.robot_pointcloud(body, 1 + a["robot_link"], a["robot_samples"]),
            "sih_fingertip_pointcloud": O.fingertip_pointcloud(body, 1 + np.array(PCM.TIP_LINKS)),
            "goal_synthetic_pointcloud": O.goal_pointcloud(goal),
            "relative_goal_synthetic_pointcloud": O.relative_goal_pointcloud(goal, body[:, 1 + PCM.FLANGE_LINK, 0:7])}
    for x, w in want.items():
        got = cpu(pcs.outputs[x])
        np.testing.assert_array_equal(got[..., 3], w[..., 3], err_msg=x)
        np.testing.assert_allclose(got, w, rtol=0, atol=1e-7, err_msg=x)
    # out-of-range target / pool ids (device data) are clamped to entry 0, never read out of bounds
    sim.t["target_object_index"].fill_(7)
    sim.t["object_indices"].fill_(99)
    pcs.refresh(perm=perm)
    torch.cuda.synchronize()
    assert np.isfinite(cpu(pcs.outputs["target_object_synthetic_pointcloud"])).all()
    with pytest.raises(ValueError):
        pcs.refresh(perm=np.zeros(pcs.P, np.int64))


def test_student_list_through_vectask():
    """VecTask with the point-cloud student list: obs = (goal_pos, flange pose, dof targets) gathered on the device
    from the step kernel's row; clouds recomputed from the refreshed tensors by the oracle; obs_dict keys and
    observation_keys as the reference builds them."""
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    N = 64
    student = ["goal_pos", "ur5_flange_pose", "dof_position_targets", "object_synthetic_pointcloud",
               "ur5sih_synthetic_pointcloud", "goal_synthetic_pointcloud"]
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": N, "observations": student}, "seed": 3}, "cuda:0", "cuda:0")
    assert env.num_obs == 27 and env.observation_keys == ["obs", "object_synthetic_pointcloud",
                                                          "ur5sih_synthetic_pointcloud", "goal_synthetic_pointcloud"]
    assert env.observations_start_end == {"goal_pos": (0, 3), "ur5_flange_pose": (3, 10),
                                          "dof_position_targets": (10, 27)}
    obs0 = env.reset()
    assert set(obs0) >= {"obs", "teacher", "object_synthetic_pointcloud"}
    g = torch.Generator(device="cuda:0").manual_seed(0)
    for _ in range(3):
        obs, rew, reset, extras = env.step(torch.rand((N, 11), device="cuda:0", generator=g) * 2 - 1)
    teacher = cpu(env.obs_buf)
    want = np.concatenate([cpu(env.goal_pos), teacher[:, 6:13], teacher[:, 63:80]], 1)
    np.testing.assert_array_equal(cpu(obs["obs"]), want)
    A, B = env.num_actors, env.num_bodies
    root = cpu(env.root_state).reshape(N, A, 13)
    body = cpu(env.body_state).reshape(N, B, 13)
    table = PCM.object_sample_table(env.objects)
    oi = cpu(env.object_indices)
    perm = cpu(env.pointclouds.perm)
    a0 = env.actor_object0
    np.testing.assert_allclose(cpu(obs["object_synthetic_pointcloud"]),
                               O.object_pointcloud(root[:, a0:a0 + 3, 0:7], table[oi], perm), rtol=0, atol=1e-7)
    a = np.load(PCM.ASSET)
    np.testing.assert_allclose(cpu(obs["ur5sih_synthetic_pointcloud"]),
                               O.robot_pointcloud(body, 1 + a["robot_link"], a["robot_samples"]), rtol=0, atol=1e-7)
    np.testing.assert_array_equal(cpu(obs["goal_synthetic_pointcloud"]), O.goal_pointcloud(cpu(env.goal_pos)))
    assert sorted(perm.tolist()) == list(range(128))


def test_full_size_cloud_properties():
    """8192 envs (the C4 shard size) with every cloud: the point types count exactly the valid samples of each
    env's objects, and un-permuting gives the posed samples in order (size-independent properties)."""
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    N = 8192
    names = ["target_object_synthetic_pointcloud", "object_synthetic_pointcloud", "goal_synthetic_pointcloud",
             "ur5_flange_pose"]
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": N, "observations": names}, "seed": 5}, "cuda:0", "cuda:0")
    env.step(torch.zeros((N, 11), device="cuda:0"))
    obj = cpu(env.pointclouds.outputs["object_synthetic_pointcloud"]).reshape(N, 3, 128, 4)
    table = PCM.object_sample_table(env.objects)
    oi = cpu(env.object_indices)
    np.testing.assert_array_equal(obj[..., 3].sum(-1), table[oi][..., 3].sum(-1))
    assert np.all(obj[..., 0:3][obj[..., 3] == 0] == 0)                     # padding zeroed
    perm = cpu(env.pointclouds.perm)
    inv = np.argsort(perm)
    np.testing.assert_array_equal(obj[:, :, inv, 3], table[oi][..., 3])      # unpermuted: valid points first
    tgt = cpu(env.pointclouds.outputs["target_object_synthetic_pointcloud"])
    ti = cpu(env.target_object_index)
    np.testing.assert_array_equal(tgt[..., 0:3], obj[np.arange(N), ti][..., 0:3])
    np.testing.assert_array_equal(tgt[..., 3], 2 * obj[np.arange(N), ti][..., 3])


def test_registered_low_dim_observables_through_vectask():
    """A custom observation list of the registered low-dimensional observables (ur5_joint_state,
    sih_fingertip_angvel, object_quat/linvel/angvel, object_mass/com/inertia, target_object_pos/quat/pos_initial,
    goal_pos, ur5_joint_pos) through the VecTask: ha_gather_obs over the refreshed tensors reproduces the
    reference's obs rows (tests/golden/ur5sih_obs_custom.npz) bit for bit. ur5_joint_pos comes from the step
    kernel's obs row, so the state is put in place and one observe launch refreshes that row first."""
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    d = np.load(os.path.join(G, "ur5sih_obs_custom.npz"))
    names = [str(n) for n in d["observations"]]
    T, N = d["target_idx"].shape
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": N, "observations": names},
                                         "objects": {"dataset": {"ycb": [str(n) for n in d["object_names"]]}}},
                                        "cuda:0", "cuda:0")
    assert env.num_obs == d["obs"].shape[-1] and env.observation_keys == ["obs"]
    put(env.sim, "object_indices", d["object_indices"])
    env._bind_gather_sources()
    for s in range(T):
        put(env.sim, "root_state", d["root"][s])
        put(env.sim, "rigid_body_state", d["body"][s])
        put(env.sim, "dof_state", d["dof"][s])
        put(env.sim, "goal_pos", d["goal_pos"][s])
        put(env.sim, "target_object_index", d["target_idx"][s])
        obs = cpu(env.reset()["obs"])            # VecTask.reset: compute_observations of the bound state
        np.testing.assert_array_equal(obs, d["obs"][s])


def test_custom_teacher_list_through_vectask():
    """A custom teacher list (cfg teacher_observations, observable_vec_task.py:17-18,194-203) next to the default
    student list: obs_dict["teacher"]["obs"] is the concatenation of the listed observables, the same rows the
    reference computes for that list as a student list (tests/golden/ur5sih_obs_custom.npz), bit for bit; the
    student obs stay the default list."""
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    d = np.load(os.path.join(G, "ur5sih_obs_custom.npz"))
    names = [str(n) for n in d["observations"]]
    T, N = d["target_idx"].shape
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": N, "teacher_observations": names},
                                         "objects": {"dataset": {"ycb": [str(n) for n in d["object_names"]]}}},
                                        "cuda:0", "cuda:0")
    assert env.num_teacher_obs == d["obs"].shape[-1] and env.num_obs == 147
    se = env.teacher_observations_start_end                # the attribute (the property keeps the reference's None)
    assert list(se) == [n for n in names if n in se] and max(e for _, e in se.values()) == env.num_teacher_obs
    put(env.sim, "object_indices", d["object_indices"])
    env._bind_gather_sources()
    for s in range(T):
        put(env.sim, "root_state", d["root"][s])
        put(env.sim, "rigid_body_state", d["body"][s])
        put(env.sim, "dof_state", d["dof"][s])
        put(env.sim, "goal_pos", d["goal_pos"][s])
        put(env.sim, "target_object_index", d["target_idx"][s])
        od = env.reset()
        np.testing.assert_array_equal(cpu(od["teacher"]["obs"]), d["obs"][s])
        assert od["obs"].shape == (N, 147)
