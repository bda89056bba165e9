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
    buf = (C.c_ulonglong * 16)()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    for objects in (False, True):
        lib.ha_profile_read(buf, 1)
        run(n, "objects on" if objects else "objects off", objects=objects)
        torch.cuda.synchronize()
        lib.ha_profile_read(buf, 1)
        tot = sum(buf[:8])
        print("  " + "  ".join(f"{PHASES[i]} {100.0 * buf[i] / tot:5.1f}%" for i in range(8)), flush=True)
