"""Drop-initialisation probe (bin-picking scene): after the drop rounds, where are the objects that are still
outside the bin extent, and which pool objects are they? Usage (GPU box): python tools/drop_probe.py [N] [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from handarm_hip import model as HM  # noqa: E402
from handarm_hip.tasks import Ur5SihMultiObjectManipulation  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 2048
rounds = int(args[1]) if len(args) > 1 else 30
nobin = "--nobin" in sys.argv          # the C4 scene: no bin, 3 objects of the 16-object pool on the table
no = 3 if nobin else 8
pool = HM.POOL16
cfg = {"env": {"numEnvs": n}, "seed": 42, "objects": {"num_objects": no, "dataset": {"ycb": pool},
                                                        "drop": {"max_rounds": rounds, "place_remaining": False}}}
if not nobin:
    cfg["bin"] = {"asset": "hard_bin"}
env = Ur5SihMultiObjectManipulation(cfg, "cuda:0", "cuda:0")
env._drop_initialisation()
torch.cuda.synchronize()
A, a0 = env.num_actors, env.actor_object0
rs = env.root_state.view(n, A, 13)[:, a0:a0 + no].cpu().numpy()
lo, hi = np.array(env.bin_extent[0]), np.array(env.bin_extent[1])
pos = rs[..., 0:3]
inside = ((pos >= lo) & (pos <= hi)).all(-1)
print(f"objects outside after the drop: {int((~inside).sum())} of {inside.size}")
idx = env.object_indices.cpu().numpy()
bad = np.argwhere(~inside)
for e, o in bad[:40]:
    p = pos[e, o]
    why = [f"{'xyz'[k]}{'<' if p[k] < lo[k] else '>'}" for k in range(3) if p[k] < lo[k] or p[k] > hi[k]]
    print(f"env {e} obj {o} {pool[idx[e, o]]:22s} pos {np.round(p, 3)} vel {np.round(np.linalg.norm(rs[e, o, 7:10]), 3)} "
          f"out {' '.join(why)}")
from collections import Counter
print("by object:", Counter(pool[idx[e, o]] for e, o in bad).most_common())
print("by axis:", Counter(tuple(k for k in range(3) if pos[e, o, k] < lo[k] or pos[e, o, k] > hi[k]) for e, o in bad))

# --settle K: step K more physics calls and follow the objects that were outside (do they come to rest?)
if "--settle" in sys.argv:
    K = int(sys.argv[sys.argv.index("--settle") + 1])
    track = [(int(e), int(o)) for e, o in bad]
    for k in range(K // 100):
        env.sim.simulate(100)
        torch.cuda.synchronize()
        rs2 = env.root_state.view(n, A, 13)[:, a0:a0 + no].cpu().numpy()
        sp = np.array([np.linalg.norm(rs2[e, o, 7:10]) for e, o in track])
        allsp = np.linalg.norm(rs2[..., 7:10], axis=-1)
        print(f"settle +{100 * (k + 1)}: tracked speed median {np.median(sp):.4f} max {sp.max():.4f}; all objects "
              f"speed p99 {np.percentile(allsp, 99):.4f} max {allsp.max():.4f}, >0.01: {int((allsp > 0.01).sum())}",
              flush=True)
    for e, o in track[:12]:
        print(f"  env {e} obj {o} {pool[idx[e, o]]:22s} pos {np.round(rs2[e, o, 0:3], 3)} "
              f"quat {np.round(rs2[e, o, 3:7], 3)} vel {np.round(rs2[e, o, 7:13], 3)}")
