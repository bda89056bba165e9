#!/usr/bin/env python3
"""Camera kernel probe (GPU box): ha_render_camera on a simulated state at several env counts and resolutions.

Reports the HIP-event mean per launch, rays per second and the image bytes written per second.
Usage: python tools/camera_probe.py [--envs 1024 8192] [--res 160x90 640x480] [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from handarm_hip import cameras as CAM  # noqa: E402
from handarm_hip.sim import HandArmSim  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, nargs="+", default=[1024, 8192])
    ap.add_argument("--res", nargs="+", default=["160x90", "640x480"])
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from oracle.oracle_lib import HostState
    from tests import scenes
    for N in args.envs:
        sim = HandArmSim(N, "cuda:0")
        st = HostState(N, model=sim.model, params=sim.params)
        scenes.fill_scene(st, N, seed=0)
        for k in ("root_state", "dof_state", "sim_targets", "object_indices", "goal_pos"):
            sim.t[k].copy_(torch.from_numpy(np.ascontiguousarray(st[k])).reshape(sim.t[k].shape).to(sim.t[k].dtype))
        sim.simulate(10)
        for res in args.res:
            W, H = (int(v) for v in res.split("x"))
            if N * W * H > 8192 * 160 * 90 * 4:
                continue
            cam = CAM.CameraSensor(sim, [0.28, 1.05, 0.9], [0.213, 0.213, -0.674, 0.674], 87, (W, H))
            for _ in range(3):
                cam.render()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                cam.render()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.iters
            rays = N * W * H
            out_bytes = rays * (4 + 4 + 16)
            print(f"envs {N:6d} {W}x{H}: {ms:.3f} ms per launch, {rays / ms / 1e6:.2f} G rays/s, "
                  f"{out_bytes / ms / 1e6:.0f} GB/s of images written", flush=True)
            del cam
        del sim
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
