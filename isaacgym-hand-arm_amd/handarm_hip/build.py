"""Build libhandarm_hip.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build() and the tests."""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(PKG), "csrc")
INCLUDE = os.path.join(os.path.dirname(os.path.dirname(PKG)), "include")
LIB = os.path.join(PKG, "libhandarm_hip.so")
SOURCES = ["handarm_hip.hip"]
HEADERS = ["ha_device.h", "ha_physics.h", "ha_dr.h", "ha_task.h", "ah_task.h", "ak_task.h", "ha_pointcloud.h", "ha_camera.h"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-Wno-unused-result"]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, h) for h in ("handarm_abi.h", "ha_fmath.h", "ha_obb.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", *FLAGS, "-I", INCLUDE, "-o", LIB + ".tmp",
           *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
