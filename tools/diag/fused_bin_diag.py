"""Diagnostic (GPU): where does the fused hb_step_kernel differ from the oracle chain? Runs the bin window of
tests/test_gpu_fused_steps.py step 0, then replays the same step on a second sim with the simulate kernel
(controller / reset from the chain, physics by ha_simulate / ha_simulate_envs) and compares all three."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
from handarm_hip import model as HM  # noqa: E402
from handarm_hip.sim import HandArmSim  # noqa: E402
from oracle.oracle_lib import Oracle  # noqa: E402
from tests import scenes, step_chains  # noqa: E402
from tests.test_gpu_fused_steps import _ur5sih_case, push_all, put, get  # noqa: E402

n = 64
sim = HandArmSim(n, "cuda:0", task_cfg={"n_objects": 8}, scene=HM.load_scene(HM.BIN_ASSET))
hs, rng = _ur5sih_case(sim, n, 22, lambda h: scenes.fill_bin_scene(h, n, sim.scene, seed=8))
p, m = sim.params, sim.model
push_all(sim, hs)
h0 = hs.copy()
act = rng.uniform(-1, 1, (n, 11)).astype(np.float32)
draws = np.zeros((n, HM.DRAW_STRIDE), np.float32)
draws[:, 1] = rng.integers(0, 8, n)
draws[:, 2:5] = rng.uniform(0, 1, (n, 3))
hs["actions"][:] = act
put(sim, "actions", act)
put(sim, "reset_draws", draws)
sim.t["contact_stats"].zero_()
sim.task_step(HM.FLAG_REPLAY_DRAWS)
orc = Oracle(m, p, n)
step_chains.ur5sih_step(orc, hs, p, m, draws)
cs = get(sim, "contact_stats")
resets = h0["reset_buf"] != 0
for k in ("sim_targets", "dof_position_targets", "servo", "ur5_target"):
    g = get(sim, k).reshape(hs[k].shape)
    print(k, "differs in envs", np.nonzero((g != hs[k]).reshape(n, -1).any(1))[0].tolist())
for k in scenes.PHYSICS_OUTPUTS:
    g = get(sim, k).reshape(n, -1)
    o = hs[k].reshape(n, -1)
    bad = np.nonzero((g.view(np.uint32) != o.view(np.uint32)).any(1))[0]
    print(f"{k}: differing envs {bad.tolist()}, reset {resets[bad].astype(int).tolist()}, "
          f"max offered {cs[bad, 2].tolist()}, over-capacity substeps {cs[bad, 1].tolist()}")
print("envs with > 84 contacts offered:", np.nonzero(cs[:, 2] > 84)[0].tolist(), "max offered overall", cs[:, 2].max())
# the same step with the simulate kernel for the physics (chain's task math, GPU physics)
sim2 = HandArmSim(n, "cuda:0", task_cfg={"n_objects": 8}, scene=HM.load_scene(HM.BIN_ASSET))
h2 = h0.copy()
h2["actions"][:] = act
orc.controller(h2)
# mirror ur5sih_step's reset part on the host, physics on the GPU
from oracle import task_oracle as TO  # noqa: E402
root = h2["root_state"].reshape(n, m.n_actors, 13)
dof = h2["dof_state"].reshape(n, 17, 2)
actors = np.arange(m.actor_object0, m.actor_object0 + 8)
rids = np.nonzero(h2["reset_buf"])[0]
for e in rids:
    root[e, actors, 0:3] = h2["object_pos_initial"][e, 0]
    root[e, actors, 3:7] = h2["object_quat_initial"][e, 0]
    root[e, actors, 7:13] = 0
    rp = np.array(list(p.reset_pose)[:17], np.float32)
    dof[e, :, 0] = rp
    dof[e, :, 1] = 0
    h2["sim_targets"][e] = rp
push_all(sim2, h2)
sim2.simulate(1, env_ids=torch.as_tensor(rids.astype(np.int32), device="cuda:0"))
sim2.simulate(3)
for k in scenes.PHYSICS_OUTPUTS:
    g1 = get(sim, k).reshape(n, -1)
    g2 = get(sim2, k).reshape(n, -1)
    o = hs[k].reshape(n, -1)
    b12 = np.nonzero((g1.view(np.uint32) != g2.view(np.uint32)).any(1))[0]
    b2o = np.nonzero((g2.view(np.uint32) != o.view(np.uint32)).any(1))[0]
    print(f"{k}: step kernel vs simulate kernel differ in {b12.tolist()}; simulate kernel vs oracle chain {b2o.tolist()}")
