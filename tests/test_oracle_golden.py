"""Pin the numpy task oracle against golden vectors produced by the reference code itself."""
import os

import numpy as np
import pytest

from oracle import task_oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name))


def test_quat_utils():
    d = load("quat_utils.npz")
    np.testing.assert_array_equal(O.quat_mul(d["a"], d["b"]), d["quat_mul"])
    np.testing.assert_allclose(O.quat_apply(d["a"], d["v"]), d["quat_apply"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(O.quat_conjugate(d["a"]), d["quat_conjugate"])
    np.testing.assert_allclose(O.quat_from_angle_axis(d["ang"], d["axis"]), d["quat_from_angle_axis"], atol=1e-6)
    np.testing.assert_allclose(O.randomize_rotation(d["r0"], d["r1"]), d["randomize_rotation"], atol=1e-6)
    np.testing.assert_array_equal(O.scale(d["x"], d["lo"], d["hi"]), d["scale"])
    np.testing.assert_allclose(O.unscale(d["x"], d["lo"], d["hi"]), d["unscale"], rtol=1e-6)


def test_spline_tables_match_reference_construction():
    d = load("ur5sih_controller.npz")
    for name, sp in O.SPLINE_OBJS.items():
        np.testing.assert_allclose(sp.table(), d["spline_" + name], rtol=1e-6, atol=1e-9)
        np.testing.assert_array_equal(sp.t, d["knots_" + name])


def test_controller_sequence():
    d = load("ur5sih_controller.npz")
    ur5, servo = d["init_ur5_target"], d["init_servo"]
    smoothed = np.zeros_like(servo)
    for s in range(d["actions"].shape[0]):
        tgt, ur5, servo, smoothed = O.controller_step(d["actions"][s], d["dof_pos"][s], ur5, servo, smoothed)
        np.testing.assert_array_equal(ur5, d["ur5_target"][s])
        np.testing.assert_array_equal(smoothed, d["smoothed"][s])
        np.testing.assert_array_equal(servo, d["servo"][s])
        np.testing.assert_allclose(tgt, d["targets"][s], rtol=1e-6, atol=1e-6)


# (fixture, objects, actors, bodies, object actor rows): the default scene and the bin-picking variant
# (BASELINE config 5: 8 objects, bin actor at 3, objects from actor 4; fixture made by make_goldens.py --bin)
OBS_CASES = [("ur5sih_obs_reward.npz", 3, 6, 34, [3, 4, 5]),
             ("ur5sih_obs_reward_bin8.npz", 8, 12, 44, list(range(4, 12)))]


@pytest.mark.parametrize("fixture,no,A,B,actors", OBS_CASES, ids=["default3", "bin8"])
def test_observations_reward_done_sequence(fixture, no, A, B, actors):
    d = load(fixture)
    steps, n = d["rew"].shape
    tracker = O.SuccessTracker(no, n)
    prev = np.zeros((n, no, 7), np.float32)   # make_task's init refresh saw an all-zero root state
    for s in range(steps):
        root = d["root"][s].reshape(n, A, 13)
        body = d["body"][s].reshape(n, B, 13)
        dof = d["dof"][s].reshape(n, 17, 2)
        obs, bbox = O.observations(root, body, dof, d["targets"][s], d["goal_pos"][s], d["target_idx"][s],
                                   d["bbox_from_origin_pos"], d["bbox_from_origin_quat"], d["bbox"][s][..., 7:10], prev,
                                   object_actors=actors)
        assert obs.shape == (n, 108 + 13 * no)
        prev = root[:, actors, 0:7].copy()
        np.testing.assert_allclose(obs, d["obs"][s], rtol=0, atol=2e-7)
        np.testing.assert_allclose(obs, d["teacher"][s], rtol=0, atol=2e-7)
        progress = d["progress_in"][s] + 1
        np.testing.assert_array_equal(progress, d["progress"][s])
        reset, timeout = O.done(progress, d["reset_in"][s])
        np.testing.assert_array_equal(reset, d["reset"][s])
        np.testing.assert_array_equal(timeout, d["timeout"][s])
        rew, reached, terms = O.reward(root, body, d["goal_pos"][s], d["target_idx"][s], d["cfg_idx"][s],
                                       d["object_pos_initial"], object_actors=actors)
        np.testing.assert_allclose(rew, d["rew"][s], rtol=2e-6, atol=2e-6)
        np.testing.assert_allclose([terms[k].mean() for k in d["reward_terms"]], d["log_terms"][s], rtol=1e-5)
        reached_before = reached | d["reached_in"][s]
        np.testing.assert_array_equal(reached_before, d["reached"][s])
        log = tracker.update(*O.success_counts(reset, reached_before, d["object_indices"], d["target_idx"][s], no))
        np.testing.assert_allclose(log.get("overall", np.nan), d["log_overall"][s], rtol=1e-6)
        np.testing.assert_allclose([log.get(i, np.nan) for i in range(no)], d["log_obj"][s], rtol=1e-6)


def test_reset_steady_state():
    d = load("ur5sih_reset.npz")
    n = d["draw_cfg"].shape[0]
    out = O.reset_state(d["root_before"].reshape(n, 6, 13), d["dof_before"].reshape(n, 17, 2), d["draw_cfg"],
                        d["draw_target"], d["draw_goal"], d["object_pos_initial"], d["object_quat_initial"])
    np.testing.assert_array_equal(out["root"].reshape(-1, 13), d["root_after"])
    np.testing.assert_array_equal(out["dof"].reshape(-1, 2), d["dof_after"])
    np.testing.assert_array_equal(out["targets"], d["targets"])
    np.testing.assert_array_equal(out["goal_pos"], d["goal_pos"])
    np.testing.assert_array_equal(out["target_idx"], d["target_idx"])
    np.testing.assert_array_equal(out["cfg_idx"], d["cfg_idx"])
    np.testing.assert_array_equal(out["servo"], d["servo"])
    np.testing.assert_array_equal(out["smoothed"], d["smoothed"])
    np.testing.assert_array_equal(out["ur5_target"], d["ur5_target"])
    assert (d["progress"] == 0).all() and (d["reset"] == 0).all() and (~d["reached"]).all()
