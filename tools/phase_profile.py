"""Per-phase cycle shares of one substep (diagnostic build libhandarm_hip_prof.so, -DHA_PROFILE).

Build: hipcc ... -DHA_PROFILE -o handarm_hip/libhandarm_hip_prof.so ; run on the GPU box.
Shares are meaningful, absolute lengths are not (the stamps add barriers)."""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
from handarm_hip import _lib, build  # noqa: E402

PROF_LIB = os.path.join(build.PKG, "libhandarm_hip_prof.so")
PHASES = ["fk", "dynamics(CRBA+RNEA)", "chol+Minv+free+objects", "detect", "contact rows J,Y", "joint rows", "PGS",
          "forces+integrate"]

if __name__ == "__main__":
    if "--build" in sys.argv:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", *build.FLAGS, "-DHA_PROFILE", "-I", build.INCLUDE,
               "-o", PROF_LIB, os.path.join(build.CSRC, "handarm_hip.hip")]
        subprocess.check_call(cmd)
        sys.exit(0)
    _lib.LIB_PATH = PROF_LIB
    import torch
    from tools.perf_probe import run
    lib = _lib.load()
    lib.ha_profile_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 96)()
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    n = int(args[0]) if args else 8192

    def report(label):
        torch.cuda.synchronize()
        lib.ha_profile_read(buf, 1)
        tot = sum(buf[:8])
        print(f"{label}: contacts/substep {buf[8] / max(buf[9], 1):.2f}", flush=True)
        print("  " + "  ".join(f"{PHASES[i]} {100.0 * buf[i] / tot:5.1f}%" for i in range(8)), flush=True)
        sub = max(buf[9], 1)
        for k, name in enumerate(["obj-ground", "obj-static", "obj-obj", "link-obj", "link-static"]):
            print(f"    narrow {name:10s}: {buf[15 + k] / sub:6.2f} pairs/substep, {buf[20 + k] / sub:6.2f} with contacts, "
                  f"{100.0 * buf[10 + k] / tot:5.1f}% of substep cycles", flush=True)
        print("    hull-hull split: " + "  ".join(f"{nm} {100.0 * buf[25 + i] / tot:5.1f}%" for i, nm in
              enumerate(["setup", "SAT A", "SAT B", "incident", "emit", "edge-edge", "clip"])), flush=True)
        for k, name in enumerate(["obj-ground", "obj-static", "obj-obj", "link-obj", "link-static"]):
            row = [buf[32 + 8 * k + i] for i in range(7)]
            if sum(row):
                print(f"      {name:11s}: " + "  ".join(f"{nm} {100.0 * v / tot:5.1f}%" for nm, v in
                      zip(["setup", "SAT A", "SAT B", "incident", "emit", "edge-edge", "clip"], row)), flush=True)

    if any(f in sys.argv for f in ("--bench-scene", "--kuka", "--bin", "--allegro", "--c4")):
        # the bench workload: VecTask after its first (reset) steps, random actions
        from handarm_hip.tasks import AllegroHand, AllegroKuka, Ur5SihMultiObjectManipulation
        if "--allegro" in sys.argv:
            n = int(args[0]) if args else 16384
            env = AllegroHand({"env": {"numEnvs": n}, "seed": 42}, "cuda:0", "cuda:0")
        elif "--kuka" in sys.argv:
            n = int(args[0]) if args else 4096
            env = AllegroKuka({"env": {"numEnvs": n}, "seed": 42}, "cuda:0", "cuda:0")
        elif "--bin" in sys.argv:       # bench --task binpick (config 5 shard)
            from handarm_hip import model as HM
            pool = [o["name"] for o in HM.load_scene()["objects"]]
            env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": n}, "seed": 42, "bin": {"asset": "hard_bin"},
                                                 "objects": {"num_objects": 8, "dataset": {"ycb": pool}}},
                                                "cuda:0", "cuda:0")
        elif "--c4" in sys.argv:        # bench config 4: 16-object YCB pool, DR on (--nomug: the pool without the mug)
            from handarm_hip import model as HM
            pool = [o["name"] for o in HM.load_scene()["objects"]]
            if "--nomug" in sys.argv:
                pool = [p for p in pool if "mug" not in p]
            env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": n}, "seed": 42, "task": {"randomize": True},
                                                 "objects": {"dataset": {"ycb": pool}}}, "cuda:0", "cuda:0")
        else:
            env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": n}, "seed": 42}, "cuda:0", "cuda:0")
        env.reset()
        na = env.num_acts
        g = torch.Generator(device="cuda:0").manual_seed(42)
        for _ in range(20):
            env.step(torch.rand((n, na), device="cuda:0", generator=g) * 2 - 1)
        torch.cuda.synchronize()
        lib.ha_profile_read(buf, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            env.step(torch.rand((n, na), device="cuda:0", generator=g) * 2 - 1)
        e1.record()
        torch.cuda.synchronize()
        print(f"bench scene n={n}: {e0.elapsed_time(e1) / 10:.3f} ms/step (profiled build)", flush=True)
        report("bench scene")
        sys.exit(0)
    for objects in (False, True):
        lib.ha_profile_read(buf, 1)
        run(n, "objects on" if objects else "objects off", objects=objects)
        report("objects on" if objects else "objects off")
