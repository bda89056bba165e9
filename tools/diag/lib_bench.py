"""Diagnostic: bench.py on a variant library build (A/B of timing and PMC traffic; not a product path).

    python3 tools/diag/lib_bench.py LIB TASK [bench args...]     (LIB relative to isaacgym-hand-arm_amd/handarm_hip/)
"""
import os
import runpy
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [R, os.path.join(R, "isaacgym-hand-arm_amd")]
from handarm_hip import _lib  # noqa: E402

lib, task = sys.argv[1], sys.argv[2]
_lib.LIB_PATH = os.path.join(R, "isaacgym-hand-arm_amd", "handarm_hip", "libhandarm_hip.so" if lib == "product" else lib)
sys.argv = [os.path.join(R, "bench.py"), "--task", task, "--no-cpu-baseline"] + sys.argv[3:]
runpy.run_path(os.path.join(R, "bench.py"), run_name="__main__")
