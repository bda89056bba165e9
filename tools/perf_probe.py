"""Time one gym.simulate() call of the HIP kernel at full shard size under scene variants (GPU)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from handarm_hip import model as HM  # noqa: E402
from handarm_hip.sim import HandArmSim  # noqa: E402
from oracle.oracle_lib import HostState  # noqa: E402
from tests import scenes  # noqa: E402


def run(n, label, objects=True, iters=None, calls=5, **cfg):
    sim = HandArmSim(n, "cuda:0", task_cfg=cfg or None)
    st = HostState(n)
    scenes.fill_scene(st, n, seed=0)
    if not objects:
        st["collision_enabled"][:] = 0
    for k in HM.STATE_FIELDS:
        if k not in ("stats", "term_sums"):
            sim.t[k].copy_(torch.as_tensor(st[k]).reshape(sim.t[k].shape).to(sim.t[k].dtype))
    sim.simulate(1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    sim.simulate(calls)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / calls
    print(f"{label:40s} n={n:6d}  {ms:8.3f} ms/call  {ms / 2 * 1e3 / n:8.3f} us/substep/env  "
          f"{n / (3 * ms) * 1e3:10.0f} env-steps/s-equiv", flush=True)


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    run(n, "objects off (articulation + drives)", objects=False)
    run(n, "default scene")
    run(n, "default scene, 4 solver iters", solver_iters=4)
    run(n // 4, "default scene, quarter envs")
    run(n * 2, "default scene, double envs")
