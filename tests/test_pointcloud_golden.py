"""Synthetic point-cloud observables on the CPU: the numpy oracle and the host logic
(observable order, obs-vector columns, sample tables) against goldens made by running the reference's own
post_physics_step with the point-cloud lists active (tests/golden/make_goldens.py --pointclouds).

Tolerance: point coordinates within 2e-7 absolute (about 1 ulp at 1 m: torch's CPU cross products may fuse
multiply-adds); point types, goal clouds and index work bit-exact."""
import os

import numpy as np
import pytest

from handarm_hip import observables as OB
from handarm_hip import pointclouds as PCM
from oracle import task_oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["student", "all"]


def load(case):
    return np.load(os.path.join(G, f"ur5sih_pointclouds_{case}.npz"))


def previous_pose(d, s, n_obj=3):
    """object_pos / object_quat as of the previous refresh: make_task's initial refresh ran on all-zero
    tensors, later ones on the previous step's root state (actors goal 0, robot 1, table 2, objects 3..)."""
    if s == 0:
        return np.zeros((d["root"].shape[1] // 6, n_obj, 7), np.float32)
    return d["root"][s - 1].reshape(-1, 6, 13)[:, 3:3 + n_obj, 0:7]


@pytest.mark.parametrize("case", CASES)
def test_post_step_order_matches_reference(case):
    d = load(case)
    order = OB.post_step_order([str(n) for n in d["observations"]], OB.DEFAULT_OBSERVATIONS)
    assert order == [str(n) for n in d["post_step_order"]]
    # the quirk the order carries: the full list refreshes the object cloud before object_pos
    assert OB.sees_previous_object_pose(order, "object_synthetic_pointcloud") == (case == "all")
    assert OB.sees_previous_object_pose(order, "object_bounding_box")


@pytest.mark.parametrize("case", CASES)
def test_oracle_clouds_match_reference(case):
    d = load(case)
    names = [str(n) for n in d["observations"]]
    order = [str(n) for n in d["post_step_order"]]
    table = PCM.object_sample_table([str(n) for n in d["pool"]])
    a = np.load(PCM.ASSET)
    steps, n = d["target_idx"].shape
    oi = d["object_indices"]
    for s in range(steps):
        root = d["root"][s].reshape(n, 6, 13)
        body = d["body"][s].reshape(n, -1, 13)
        pose = previous_pose(d, s) if OB.sees_previous_object_pose(order, "object_synthetic_pointcloud") \
            else root[:, 3:6, 0:7]
        obj = O.object_pointcloud(pose, table[oi], d["perm"][s])
        np.testing.assert_allclose(obj, d["object_synthetic_pointcloud"][s], rtol=0, atol=2e-7)
        rob = O.robot_pointcloud(body, 1 + a["robot_link"], a["robot_samples"])
        np.testing.assert_allclose(rob, d["ur5sih_synthetic_pointcloud"][s], rtol=0, atol=2e-7)
        np.testing.assert_array_equal(O.goal_pointcloud(d["goal_pos"][s]), d["goal_synthetic_pointcloud"][s])
        if "target_object_synthetic_pointcloud" in names:
            np.testing.assert_allclose(O.target_pointcloud(obj, d["target_idx"][s], 3),
                                       d["target_object_synthetic_pointcloud"][s], rtol=0, atol=2e-7)
            np.testing.assert_array_equal(O.fingertip_pointcloud(body, 1 + np.array(PCM.TIP_LINKS)),
                                          d["sih_fingertip_pointcloud"][s])
            np.testing.assert_allclose(O.relative_goal_pointcloud(d["goal_pos"][s], body[:, 1 + PCM.FLANGE_LINK, 0:7]),
                                       d["relative_goal_synthetic_pointcloud"][s], rtol=0, atol=2e-7)


@pytest.mark.parametrize("case", CASES)
def test_obs_vector_columns(case):
    """The student obs vector = (teacher-layout obs row | goal_pos) columns, bit-exact."""
    d = load(case)
    cols = OB.obs_columns([str(n) for n in d["observations"]], 3)
    assert len(cols) == d["obs"].shape[-1] == 27
    for s in range(d["obs"].shape[0]):
        src = [d["teacher"][s], d["goal_pos"][s]]
        got = np.stack([src[a][:, c] for a, c in cols], -1)
        np.testing.assert_array_equal(got, d["obs"][s])


def test_sample_table_area_mode():
    """'area' mode: int(100 * area / mean_area) valid points per object over the configured pool, capped at
    max_num_points, zero padding (multi_object.py:774-786)."""
    a = np.load(PCM.ASSET)
    pool = [str(n) for n in a["object_names"][:5]]
    t = PCM.object_sample_table(pool)
    areas = a["object_areas"][:5]
    want = [min(int(100 * x / areas.mean()), 128) for x in areas]
    assert [int(t[i, :, 3].sum()) for i in range(5)] == want
    for i in range(5):
        assert np.all(t[i, want[i]:] == 0)
        np.testing.assert_array_equal(t[i, :want[i], 0:3], a["object_samples"][i, :want[i]])
    u = PCM.object_sample_table(pool, sample_mode="uniform")
    assert np.all(u[:, :100, 3] == 1) and np.all(u[:, 100:] == 0)
    with pytest.raises(NotImplementedError):
        OB.obs_columns(["ur5_joint_vel"], 3)


def _gather_np(cols, srcs, target):
    """numpy restatement of ha_gather_obs (include/handarm_abi.h): column (source | HA_OBS_SRC_TARGET, c)."""
    N = srcs[0].shape[0]
    out = np.zeros((N, len(cols)), np.float32)
    for j, (s, c) in enumerate(cols):
        src = srcs[s & (OB.SRC_TARGET - 1)]
        off = c + (target * 13 if s & OB.SRC_TARGET else 0)
        out[:, j] = src[np.arange(N), off]
    return out


def test_registered_low_dim_observables_columns_against_reference():
    """The registered low-dimensional observables a custom list can name (ur5_joint_state, sih_fingertip_angvel,
    object_quat/linvel/angvel, object_mass/com/inertia, target_object_pos/quat/pos_initial, goal_pos): their
    ha_gather_obs columns over the refreshed tensors reproduce the reference's obs rows bit for bit
    (tests/golden/ur5sih_obs_custom.npz, generated by the reference's own post_step callbacks)."""
    from handarm_hip import model as HM
    d = np.load(os.path.join(G, "ur5sih_obs_custom.npz"))
    names = [str(n) for n in d["observations"]]
    T, N = d["target_idx"].shape
    scene = HM.load_scene()
    m = HM.build_model(scene, [str(n) for n in d["object_names"]])
    props = np.concatenate([np.ctypeslib.as_array(m.pool_mass)[:m.n_pool, None],
                            np.ctypeslib.as_array(m.pool_com)[:m.n_pool],
                            np.ctypeslib.as_array(m.pool_inertia)[:m.n_pool]], 1).astype(np.float32)
    props = props[d["object_indices"]].reshape(N, -1)
    cols = OB.obs_columns(names, 3, dict(a0=m.actor_object0, body_robot0=m.body_robot0, n_dofs=m.n_dofs))
    assert len(cols) == d["obs"].shape[-1]
    for s in range(T):
        obs_row = np.zeros((N, 147), np.float32)          # the step kernel's row: ur5_joint_pos = dof pos 0..5
        obs_row[:, 0:6] = d["dof"][s].reshape(N, 17, 2)[:, 0:6, 0]
        srcs = [obs_row, d["goal_pos"][s], d["root"][s].reshape(N, -1), d["body"][s].reshape(N, -1),
                d["dof"][s].reshape(N, -1), props]
        np.testing.assert_array_equal(_gather_np(cols, srcs, d["target_idx"][s]), d["obs"][s])
