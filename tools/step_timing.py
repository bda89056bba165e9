"""Per-step wall-clock vs GPU-event timing of a VecTask (diagnostic). Usage: python tools/step_timing.py [task]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
import torch  # noqa: E402

from handarm_hip.tasks import isaacgym_task_map  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "AllegroKuka"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
env = isaacgym_task_map[task]({"env": {"numEnvs": n}}, "cuda:0", "cuda:0")
env.reset()
a = torch.rand((n, env.num_acts), device="cuda:0") * 2 - 1
for _ in range(10):
    env.step(a)
torch.cuda.synchronize()
walls, gpus = [], []
for k in range(40):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    env.step(a)
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    walls.append(((t1 - t0) * 1e3, (t2 - t0) * 1e3))
    gpus.append(e0.elapsed_time(e1))
for k in range(0, 40, 4):
    print(f"step {k}: host issue {walls[k][0]:.3f} ms, issue+sync {walls[k][1]:.3f} ms, gpu {gpus[k]:.3f} ms")
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(40):
    env.step(a)
torch.cuda.synchronize()
print(f"pipelined: {(time.perf_counter() - t0) / 40 * 1e3:.3f} ms/step")
t0 = time.perf_counter()
for k in range(40):
    env.sim.task_step(0)
torch.cuda.synchronize()
print(f"bare task_step: {(time.perf_counter() - t0) / 40 * 1e3:.3f} ms/step")
