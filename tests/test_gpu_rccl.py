"""RCCL on the GPU box: the nccl backend (RCCL on ROCm) brought up by handarm_hip.parallel's path with one rank per
GPU. The gpurun box has one GPU, so the group has one rank: this executes RCCL's init, the all-reduce that
parallel.describe() uses to report the world size, and an all-reduce of a step kernel's device counters (the
payload reduce_episode_stats sends at N > 1), which one rank must leave unchanged. The N > 1 arithmetic is covered by
the gloo world-2 tests (tests/test_parallel.py); the driver runs the 8-GPU bench."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys, json
sys.path[:0] = [os.environ["HA_ROOT"], os.path.join(os.environ["HA_ROOT"], "isaacgym-hand-arm_amd")]
import torch, torch.distributed as dist
from handarm_hip import parallel
from handarm_hip.tasks import isaacgym_task_map
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
info = parallel.describe()
env = isaacgym_task_map["AllegroKuka"]({"env": {"numEnvs": 256}}, "cuda:0", "cuda:0")
env.reset()
for _ in range(5):
    env.step(torch.zeros((256, env.num_acts), device="cuda:0"))
ts = env.sim.t["task_state"].clone()
red = ts.clone()
dist.all_reduce(red)
torch.cuda.synchronize()
out = {"info": info, "same": bool(torch.equal(ts, red)), "backend": dist.get_backend()}
dist.destroy_process_group()
print("RESULT " + json.dumps(out))
"""


def test_rccl_group_and_all_reduce_of_step_counters():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, HA_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    import json
    out = json.loads(line[len("RESULT "):])
    assert out["backend"] == "nccl" and out["info"] == {"backend": "nccl", "world_size": 1}
    assert out["same"]
