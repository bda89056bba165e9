"""Seed-faithful draws on the host (handarm_hip/ref_rng.py, cfg sim.reference_rng) against the reference's own
draws from the same seed (north_star: "bit-exact for done masks / reset indexing" on identical seeds).

The goldens come from running the reference (tests/golden/make_goldens.py --rng, make_goldens_kuka.py,
make_goldens_allegro.py): the torch global generator is seeded, then the reference's reset_idx /
pre_physics_step draw in their own order. Here the product's host draw functions run from the same seed and
must reproduce every draw bit for bit. The kernels consume these draws through HA_FLAG_REPLAY_DRAWS
(tests/test_gpu_ref_rng.py runs the VecTask classes that way on the GPU).
"""
import os

import numpy as np
import torch

from handarm_hip import model as HM
from handarm_hip import ref_rng as RR

G = os.path.join(os.path.dirname(__file__), "golden")


def test_ur5sih_reset_draws_reproduce_reference_episodes():
    """Four all-env reset_idx calls from one seed: target object, object configuration and goal position."""
    d = np.load(os.path.join(G, "ur5sih_ref_rng.npz"))
    E, N = d["target_idx"].shape
    P = int(d["num_initial_poses"])
    c = HM.build_params()[1]
    torch.manual_seed(int(d["seed"]))
    for e in range(E):
        dr = RR.ur5sih_reset_draws(N, P, 3).numpy()
        np.testing.assert_array_equal(dr[:, 0].astype(np.int64), d["cfg_idx"][e])
        np.testing.assert_array_equal(dr[:, 1].astype(np.int64), d["target_idx"][e])
        # the kernel's goal arithmetic (ha_task.h task_reset), restated in float32
        f = np.float32
        goal = np.array(c["goal_pos"], f) + (f(2) * (dr[:, 2:5] - f(0.5))) * np.array(c["goal_noise"], f)
        np.testing.assert_array_equal(goal, d["goal_pos"][e])


def test_ur5sih_drop_draws_reproduce_reference():
    """The drop loop's per-object draws (_get_random_object_pos 'drop' + _get_random_quat) for a sequence of
    env subsets, from one seed."""
    d = np.load(os.path.join(G, "ur5sih_ref_rng.npz"))
    c = HM.build_params()[1]
    np.testing.assert_array_equal(np.array(c["drop_pos"], np.float32), d["drop_cfg_pos"])
    np.testing.assert_array_equal(np.array(c["drop_noise"], np.float32), d["drop_cfg_noise"])
    torch.manual_seed(int(d["seed"]) + 1)
    pos, quat = [], []
    for n in d["drop_counts"]:
        p, q = RR.ur5sih_drop_pose(int(n), c["drop_pos"], c["drop_noise"])
        pos.append(p.numpy())
        quat.append(q.numpy())
    np.testing.assert_array_equal(np.concatenate(pos), d["drop_pos"])
    np.testing.assert_array_equal(np.concatenate(quat), d["drop_quat"])


def _kuka(sub):
    d = np.load(os.path.join(G, f"kuka_steps_{sub}.npz"))
    T, N = d["rew"].shape
    c = HM.build_params({"subtask": sub}, task=HM.TASK_ALLEGRO_KUKA)[1]
    torch.manual_seed(int(d["seed"]))
    kd = RR.KukaDraws(N, sub, tuple(c["force_prob_range"]), float(c["force_scale"]))
    np.testing.assert_array_equal(kd.prob.numpy(), d["random_force_prob_init"])
    fired = 0
    fu = 2 * kd.G + 53                      # the force-selection slot (ak_task.h AK_DRAW_FORCE_U)
    for s in range(T):
        D, raw = kd.step(d["reset_in"][s], d["reset_goal_in"][s])
        D = D.numpy()
        np.testing.assert_array_equal(D[:, :fu], d["draws"][s][:, :fu], err_msg=f"{sub} step {s} reset draws")
        if c["force_scale"] <= 0:           # throw: no force draws at all (allegro_kuka_base.py:1399)
            assert raw["force_u"] is None and (d["draws"][s][:, fu:] == 0).all()
            continue
        np.testing.assert_array_equal(raw["force_u"].numpy(), d["draws"][s][:, fu])
        sel = D[:, fu] == 0.0
        np.testing.assert_array_equal(sel, d["draws"][s][:, fu] < kd.prob.numpy())
        np.testing.assert_array_equal(D[sel, fu + 1:fu + 4], d["draws"][s][sel, fu + 1:fu + 4])
        fired += int(sel.sum())
        # the task_state row the reference left after this step holds its random_force_prob
        np.testing.assert_array_equal(kd.prob.numpy(), d["task_state"][s][:, HM.AK_FORCE_PROB])
    return fired


def test_kuka_draws_reproduce_reference_regrasping():
    assert _kuka("regrasping") > 0          # the random-force branch fires in this fixture


def test_kuka_draws_reproduce_reference_reorientation():
    assert _kuka("reorientation") > 0


def test_kuka_draws_reproduce_reference_throw():
    assert _kuka("throw") == 0              # forceScale 0 (env/throw.yaml)


def test_allegro_draws_reproduce_reference():
    d = np.load(os.path.join(G, "allegro_steps.npz"))
    T, N = d["rew"].shape
    torch.manual_seed(int(d["seed"]))
    ad = RR.AllegroDraws(N)
    for s in range(T):
        D = ad.step(d["reset_in"][s], d["reset_goal_in"][s]).numpy()
        w = 45                      # allegro_steps.npz records the torch_rand_float draws (slots 0-44)
        np.testing.assert_array_equal(D[:, :w], d["draws"][s][:, :w], err_msg=f"step {s}")


def test_allegro_force_draws_reproduce_reference():
    """forceScale 1 (allegro_variants.npz "force"): random_force_prob's torch.rand at reset, the force selection
    torch.rand(N) and the selected envs' torch.randn in the reference's order, and the host's selection (slot 50)."""
    g = np.load(os.path.join(G, "allegro_variants.npz"))
    d = {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith("force/")}
    T, N = d["rew"].shape
    torch.manual_seed(int(d["seed"]))
    ad = RR.AllegroDraws(N, force_scale=1.0)
    for s in range(T):
        D = ad.step(d["reset_in"][s], d["reset_goal_in"][s]).numpy()
        w = d["draws"].shape[-1]
        np.testing.assert_array_equal(D[:, :w], d["draws"][s], err_msg=f"step {s}")
        np.testing.assert_array_equal(ad.prob.numpy(), d["prob_after"][s])
