"""Distribution of the device-mode reset draws (the counter hash in ha_task.h: mix32 / uniform01), which the
product uses unless cfg sim.reference_rng asks for the reference's torch draws (tests/test_gpu_ref_rng.py).

The reference draws reset_idx's configuration and target object with torch.randint and the goal noise with
torch.rand (tasks/hand_arm/task/multi_object_manipulation.py:73-91,193-230): uniform and independent. The device
draws cannot equal those values (a different generator), so they are held to the same distributions: over
4096 envs x 8 episodes, chi-square uniformity of the configuration index (num_initial_poses categories), the
target object (3) and the goal noise per axis (binned), contingency-table independence of configuration vs
target and of one episode's target vs the next one's, and the goal noise inside its configured range.

Chi-square thresholds are the 0.9999 quantiles (scipy), so a correct generator fails about once in 10^4 runs
per check; the draws are deterministic for a given seed, so the test does not flake from run to run.
"""
import numpy as np
import pytest
import torch
from scipy import stats

from handarm_hip import model as HM

pytestmark = pytest.mark.gpu

N, E, P = 4096, 8, 4       # P: HA_MAX_INIT_POSES


def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def chi2_uniform(x, k):
    obs = np.bincount(x, minlength=k).astype(np.float64)
    assert obs.size == k, f"values outside [0, {k})"
    exp = x.size / k
    return float(((obs - exp) ** 2 / exp).sum()), k - 1


def chi2_independent(a, ka, b, kb):
    t = np.zeros((ka, kb))
    np.add.at(t, (a, b), 1.0)
    exp = t.sum(1, keepdims=True) * t.sum(0, keepdims=True) / t.sum()
    return float(((t - exp) ** 2 / exp).sum()), (ka - 1) * (kb - 1)


def assert_chi2(stat_dof, what):
    stat, dof = stat_dof
    crit = stats.chi2.ppf(0.9999, dof)
    assert stat < crit, f"{what}: chi2 {stat:.1f} >= {crit:.1f} (dof {dof})"


def test_ur5sih_device_reset_draws_distribution():
    need_gpu()
    from handarm_hip.tasks import Ur5SihMultiObjectManipulation
    env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": N}, "seed": 7,
                                         "objects": {"drop": {"num_initial_poses": P}},
                                         "rl": {"reset": {"max_episode_length": 1}}}, "cuda:0", "cuda:0")
    env.objects_dropped = True             # the initial poses are irrelevant to the draws
    env.sim_flags = HM.FLAG_NO_PHYSICS
    gp, gn = np.asarray(env.sim.params.goal_pos, np.float64), np.asarray(env.sim.params.goal_noise, np.float64)
    gen = torch.Generator(device="cuda:0").manual_seed(1)
    cfg, tgt, goal = [], [], []
    while len(cfg) < E:
        resetting = bool(env.reset_buf.all())
        env.step(torch.rand((N, env.num_acts), device="cuda:0", generator=gen) * 2 - 1)
        if resetting:
            cfg.append(env.sim.t["object_configuration_indices"].cpu().numpy().astype(np.int64))
            tgt.append(env.sim.t["target_object_index"].cpu().numpy().astype(np.int64))
            goal.append(env.sim.t["goal_pos"].cpu().numpy().reshape(N, 3).astype(np.float64))
    cfg, tgt, goal = np.stack(cfg), np.stack(tgt), np.stack(goal)
    NO = env.sim.params.n_objects
    assert_chi2(chi2_uniform(cfg.ravel(), P), "configuration index uniform")
    assert_chi2(chi2_uniform(tgt.ravel(), NO), "target object uniform")
    assert_chi2(chi2_independent(cfg.ravel(), P, tgt.ravel(), NO), "configuration vs target independent")
    assert_chi2(chi2_independent(tgt[:-1].ravel(), NO, tgt[1:].ravel(), NO), "target of consecutive episodes")
    # goal noise: uniform on [-noise, noise] per axis around goal_pos (multi_object_manipulation.py:175-184)
    u = (goal - gp) / np.where(gn > 0, gn, 1.0)
    for k in range(3):
        if gn[k] <= 0:
            np.testing.assert_array_equal(goal[..., k], np.float32(gp[k]))
            continue
        assert u[..., k].min() >= -1.0 - 1e-5 and u[..., k].max() <= 1.0 + 1e-5
        bins = np.clip(((u[..., k].ravel() + 1.0) * 10).astype(np.int64), 0, 19)
        assert_chi2(chi2_uniform(bins, 20), f"goal noise axis {k} uniform")
    # every env's episodes differ (the episode counter enters the hash)
    assert (tgt != tgt[0]).any(0).mean() > 0.9
