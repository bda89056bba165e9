"""Per-step time and contact load over one whole C4 episode (diagnostic; GPU box).

Usage: python tools/diag/episode_timeline.py [num_envs (8192)] [--nodr]
Ur5Sih, 16-object YCB pool, DR on (bench config 4 shard), random actions: the reset, 20 warm steps, then 220 steps
timed one by one with events on the task's stream; prints 20-step buckets (mean / max ms, contacts offered per
substep, resets) and the slowest single steps."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
from handarm_hip import model as HM  # noqa: E402
from handarm_hip.tasks import Ur5SihMultiObjectManipulation  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 8192
pool = HM.POOL16
env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": n}, "seed": 42, "task": {"randomize": "--nodr" not in sys.argv},
                                     "objects": {"dataset": {"ycb": pool}}}, "cuda:0", "cuda:0")
env.reset()
na = env.num_acts
g = torch.Generator(device="cuda:0").manual_seed(42)
acts = [torch.rand((n, na), device="cuda:0", generator=g) * 2 - 1 for _ in range(16)]
for k in range(20):
    env.step(acts[k % 16])
torch.cuda.synchronize()
T = 220
ev = [torch.cuda.Event(enable_timing=True) for _ in range(T + 1)]
offered, resets = [], []
stream = torch.cuda.current_stream()
for k in range(T):
    env.sim.contact_stats(reset=True)
    ev[k].record(stream)
    env.step(acts[k % 16])
    ev[k + 1].record(stream)
    torch.cuda.synchronize()
    cs = env.sim.contact_stats()
    offered.append(cs["offered_mean"])
    resets.append(int(env.reset_buf.sum().item()))
ms = np.array([ev[k].elapsed_time(ev[k + 1]) for k in range(T)])
print(f"C4 shard n={n}: mean {ms.mean():.3f} ms/step over {T} steps, p50 {np.median(ms):.3f}, max {ms.max():.3f} "
      f"(step {int(ms.argmax())})", flush=True)
for b in range(0, T, 20):
    sl = slice(b, b + 20)
    print(f"  steps {b:3d}-{b + 19:3d}: mean {ms[sl].mean():7.3f} ms  max {ms[sl].max():7.3f} ms  contacts offered/substep "
          f"{np.mean(offered[sl]):6.2f}  resets {sum(resets[sl])}", flush=True)
top = np.argsort(ms)[-5:][::-1]
print("  slowest steps: " + ", ".join(f"{int(k)}: {ms[k]:.2f} ms ({resets[k]} resets)" for k in top), flush=True)
