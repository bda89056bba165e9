"""How well the longest-first dispatch order predicts each env's span (diagnostic build libhandarm_hip_envt.so,
-DHA_ENVT; GPU box).

    python3 tools/diag/order_quality.py [allegro_hand|allegro_kuka|ur5sih|binpick] [envs] [warm steps]

Times K consecutive steps' workgroup spans per env and prints: the step-to-step correlation of an env's span, and for
the envs dispatched last (the last 10% of the launch slots) their spans against the launch's median - a launch whose
last envs are long has a tail the order did not foresee."""
import ctypes as C
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [R, os.path.join(R, "isaacgym-hand-arm_amd")]
from handarm_hip import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(R, "isaacgym-hand-arm_amd", "handarm_hip", "libhandarm_hip_envt.so")
import bench  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "allegro_hand"
key = next(k for k, v in bench.CONFIGS.items() if v[0] == task)
n = int(sys.argv[2]) if len(sys.argv) > 2 else bench.CONFIGS[key][1]
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 30


class A:
    wide_pool = False; subtask = "regrasping"; pointclouds = False; no_dr = False


env = bench.make_env(task, n, 42, "cuda:0", A())
env.reset()
g = torch.Generator(device="cuda:0").manual_seed(42)
acts = [torch.rand((n, env.num_acts), device="cuda:0", generator=g) * 2 - 1 for _ in range(16)]
lib = env.sim.lib
lib.ha_profile_env_times.argtypes = [C.c_void_p, C.c_int]
prev = None
for k in range(warm + 4):
    env.step(acts[k % 16])
    torch.cuda.synchronize()
    if k < warm:
        continue
    buf = np.zeros(2 * n, np.uint64)
    lib.ha_profile_env_times(buf.ctypes.data, n)
    t = buf.reshape(n, 2).astype(np.int64)
    order = env.sim._env_order.cpu().numpy()           # slot q ran env order[q]
    dur_slot = (t[:, 1] - t[:, 0]) / 100.0
    start_slot = (t[:, 0] - t[:, 0].min()) / 100.0
    end = (t[:, 1] - t[:, 0].min()).max() / 100.0
    dur = np.empty(n)
    dur[order] = dur_slot
    late = np.argsort(start_slot)[-n // 10:]             # the slots dispatched last
    msg = (f"step {k}: launch {end:7.1f} us, median span {np.median(dur):6.1f}, last-dispatched 10%: median "
           f"{np.median(dur_slot[late]):6.1f} p90 {np.percentile(dur_slot[late], 90):6.1f} max {dur_slot[late].max():6.1f}")
    if prev is not None:
        msg += f" | corr(span, previous step's span) {np.corrcoef(dur, prev)[0, 1]:.3f}"
    print(msg, flush=True)
    prev = dur
