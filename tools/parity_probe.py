"""GPU-vs-oracle physics parity probe (diagnostic; test infrastructure: it loads the C oracle as the checker).

For every kernel family it sets up the scenes the GPU tests use, runs `calls` gym.simulate calls on the device
(through the C ABI) and in oracle/physics_oracle.c from the same float32 state, and prints per output tensor the
fraction of envs whose rows are bit-identical and the max abs difference.

    python tools/parity_probe.py [--calls 1,3] [--n 128]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]

FIELDS = ("dof_state", "root_state", "rigid_body_state", "net_contact_force", "dof_force")


def compare(tag, sim, st, n):
    import torch
    torch.cuda.synchronize()
    worst = 1.0
    parts = []
    for k in FIELDS:
        if k not in sim.t or sim.t[k] is None or st[k] is None:
            continue
        g = sim.t[k].cpu().numpy().reshape(n, -1)
        o = np.asarray(st[k]).reshape(n, -1)
        same = (g.view(np.uint32) == o.view(np.uint32)).all(1) if g.dtype == np.float32 else (g == o).all(1)
        frac = same.mean()
        worst = min(worst, frac)
        parts.append(f"{k} {frac * 100:.1f}% max|d| {np.abs(g - o).max():.2e}")
    print(f"{tag}: " + " | ".join(parts), flush=True)
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", default="1,3")
    ap.add_argument("--n", type=int, default=128)
    a = ap.parse_args()
    from tests import test_gpu_allegro as TA
    from tests import test_gpu_bin as TB
    from tests import test_gpu_kuka as TK
    from tests import test_gpu_parity as TP
    n = a.n
    worst = 1.0
    for calls in [int(x) for x in a.calls.split(",")]:
        for seed in (0, 1, 2):
            sim, orc, st = TP._oracle_and_sim(n, seed)
            sim.simulate(calls)
            orc.simulate(st, calls)
            worst = min(worst, compare(f"ur5sih seed {seed} calls {calls}", sim, st, n))
        for seed, force in ((0, 0.0), (1, 0.5)):
            sim, orc, st = TK._oracle_and_sim(n, seed, force)
            sim.simulate(calls)
            orc.simulate(st, calls)
            worst = min(worst, compare(f"kuka seed {seed} force {force} calls {calls}", sim, st, n))
        for seed in (0, 1):
            sim, orc, st = TA._oracle_and_sim(n, seed)
            sim.simulate(calls)
            orc.simulate(st, calls)
            worst = min(worst, compare(f"allegro seed {seed} calls {calls}", sim, st, n))
        for seed in (0, 1):
            sim, orc, st = TB._bin_oracle_and_sim(n, seed)
            sim.simulate(calls)
            orc.simulate(st, calls)
            worst = min(worst, compare(f"bin seed {seed} calls {calls}", sim, st, n))
    print(f"worst bit-identical env fraction: {worst:.4f}")


if __name__ == "__main__":
    main()
