"""GPU diagnostic for the AllegroKuka step-golden tolerances (tests/test_gpu_kuka.py): per output, the largest
|GPU - reference golden| over every step, env and column, and the reward terms (task_state rewards_episode sums,
HA_AK_REW_EP, in allegro_kuka_base.py:361-374 order) that carry it. Usage (GPU box): python tools/kuka_tol_probe.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
from handarm_hip import model as HM  # noqa: E402
from handarm_hip.sim import HandArmSim  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def put(sim, name, arr):
    t = sim.t[name]
    t.copy_(torch.as_tensor(np.ascontiguousarray(arr)).reshape(t.shape).to(t.dtype))


def get(sim, name):
    torch.cuda.synchronize()
    return sim.t[name].cpu().numpy()


for sub in ("regrasping", "reorientation"):
    d = np.load(os.path.join(G, f"kuka_steps_{sub}.npz"))
    T, N = d["rew"].shape
    sim = HandArmSim(N, "cuda:0", task_cfg={"task": HM.TASK_ALLEGRO_KUKA, "subtask": sub}, task=HM.TASK_ALLEGRO_KUKA)
    flags = HM.FLAG_NO_PHYSICS | HM.FLAG_REPLAY_DRAWS
    worst = {}
    for t in range(T):
        for k, g in [("dof_state", "dof_state"), ("root_state", "root_state"), ("goal_state", "goal_state"),
                     ("dof_position_targets", "targets"), ("sim_targets", "targets"), ("actions", "actions"),
                     ("reset_buf", "reset_in"), ("reset_goal_buf", "reset_goal_in"), ("progress_buf", "progress_in"),
                     ("successes", "successes_in"), ("task_state", "task_state_in"), ("reset_draws", "draws")]:
            put(sim, k, d[g][t])
        sim.task_step(flags)
        for k, g in [("dof_state", "dof_after"), ("root_state", "root_after"), ("obs", "obs"), ("rew", "rew"),
                     ("task_state", "task_state")]:
            a, b = get(sim, k).reshape(N, -1), d[g][t].reshape(N, -1)
            if k == "task_state":
                a, b = a[:, :32], b[:, :32]
            err = np.abs(a.astype(np.float64) - b)
            col = int(np.argmax(err.max(0)))
            if err.max() >= worst.get(k, (-1,))[0]:
                worst[k] = (float(err.max()), t, col, float(np.abs(b).max()))
            if k == "task_state":
                rw = err[:, HM.AK_REW_EP:HM.AK_REW_EP + 12].max(0)
                worst.setdefault("terms", np.zeros(12))
                worst["terms"] = np.maximum(worst["terms"], rw)
            if k == "dof_state":
                worst["dof_bits"] = max(worst.get("dof_bits", 0), int((a.view(np.uint32) != b.astype(np.float32).view(np.uint32)).sum()))
    print(f"== {sub}")
    for k, v in worst.items():
        if k == "terms":
            print("  reward-term sums max |d|:", {HM.AK_REWARD_KEYS[i]: float(f"{x:.3g}") for i, x in enumerate(v)})
        elif k == "dof_bits":
            print("  dof_state elements not bit-equal:", v)
        else:
            print(f"  {k:10s} max |d| {v[0]:.3e} at step {v[1]} col {v[2]} (max |ref| {v[3]:.3g})")
