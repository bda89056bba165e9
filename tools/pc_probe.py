#!/usr/bin/env python3
"""Point-cloud kernel probe: ha_pointclouds alone on random states at several env counts (GPU box).

Reports the HIP-event mean per launch and algorithmic GB/s (bench.pointcloud_bytes_per_env) against the 8 TB/s
HBM peak, for the point-cloud student list (object, robot, goal clouds) and for every cloud.
Usage: python tools/pc_probe.py [--envs 8192 65536] [--iters 50]
       python tools/pc_probe.py --variants   (each tools/probes/libhandarm_hip_pc_*.so built by --build-variants,
                                             one subprocess per variant)
"""
import subprocess
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from handarm_hip import model as HM  # noqa: E402
from handarm_hip import observables as OB  # noqa: E402
from handarm_hip import pointclouds as PCM  # noqa: E402
from handarm_hip.sim import HandArmSim  # noqa: E402


VARIANTS = {"nt_global": "-DHA_PC_NT_STORE=1 -DHA_PC_STAGE_TABLES=0",
            "plain_global": "-DHA_PC_NT_STORE=0 -DHA_PC_STAGE_TABLES=0",
            "nt_staged": "-DHA_PC_NT_STORE=1 -DHA_PC_STAGE_TABLES=1",
            "plain_staged": "-DHA_PC_NT_STORE=0 -DHA_PC_STAGE_TABLES=1"}
PROBES = os.path.join(ROOT, "tools", "probes")


def build_variants():
    from handarm_hip import build
    for name, flags in VARIANTS.items():
        out = os.path.join(PROBES, f"libhandarm_hip_pc_{name}.so")
        cmd = ["/opt/rocm/bin/hipcc", f"--offload-arch={build.ARCH}", *build.FLAGS, *flags.split(), "-I", build.INCLUDE,
               "-o", out, os.path.join(build.CSRC, "handarm_hip.hip")]
        subprocess.check_call(cmd)
        print("built", out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, nargs="+", default=[8192, 65536])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--lib", default=None, help="library to load instead of the in-tree build (variant probes)")
    ap.add_argument("--build-variants", action="store_true")
    ap.add_argument("--variants", action="store_true")
    args = ap.parse_args()
    if args.build_variants:
        return build_variants()
    if args.variants:
        for name in VARIANTS:
            lib = os.path.join(PROBES, f"libhandarm_hip_pc_{name}.so")
            print(f"--- variant {name}", flush=True)
            subprocess.check_call([sys.executable, __file__, "--lib", lib, "--iters", str(args.iters), "--envs",
                                   *[str(n) for n in args.envs]])
        return
    if args.lib:
        from handarm_hip import _lib
        _lib.LIB_PATH = args.lib
    pool = [o["name"] for o in HM.load_scene()["objects"]]
    lists = {"student": [n for n in bench.PC_STUDENT if n in OB.POINTCLOUDS], "all": OB.POINTCLOUDS}
    for N in args.envs:
        sim = HandArmSim(N, "cuda:0", pool_names=pool)
        g = torch.Generator(device="cuda:0").manual_seed(0)
        rs = sim.t["root_state"].view(N, -1, 13)
        rs.copy_(torch.randn(rs.shape, device="cuda:0", generator=g))
        rs[..., 3:7] /= rs[..., 3:7].norm(dim=-1, keepdim=True)
        bs = sim.t["rigid_body_state"].view(N, -1, 13)
        bs.copy_(torch.randn(bs.shape, device="cuda:0", generator=g))
        bs[..., 3:7] /= bs[..., 3:7].norm(dim=-1, keepdim=True)
        sim.t["object_indices"].copy_(torch.randint(0, len(pool), (N, 3), device="cuda:0", generator=g))
        for name, names in lists.items():
            pcs = PCM.SyntheticPointclouds(sim, names, pool, generator=g)
            for _ in range(5):
                pcs.refresh()
            sim.enable_kernel_timing(args.iters)
            for _ in range(args.iters):
                pcs.refresh()
            torch.cuda.synchronize()
            ms = statistics.mean(pcs.kernel_times_ms(args.iters))
            b = bench.pointcloud_bytes_per_env(pcs)
            gbs = b * N / (ms * 1e-3) / 1e9
            print(f"envs {N:6d} {name:8s}: {b} B/env, {b * N / 1e6:.1f} MB/launch, {ms * 1e3:.1f} us, "
                  f"{gbs:.0f} GB/s = {gbs / bench.HBM_PEAK_GBS:.3f} of peak", flush=True)
            del pcs
        del sim
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
