#!/usr/bin/env bash
# A/B of the clutter family's LDS link slots (HB_LINK_SLOTS): the product build (2) against a -DHB_LINK_SLOTS=8
# build at handarm_hip/libhandarm_hip_kl8.so (hipcc with build.FLAGS + -DHB_LINK_SLOTS=8), after the bin GPU tests.
# Result (round 1): 2 slots 16.25 ms / 0.50 M env-steps/s, 8 slots 18.4 ms / 0.44 M (8192 envs).
R=$PWD
python -u -m pytest tests/test_gpu_bin.py -x -q -s --timeout 240 --timeout-method thread > gpurun_out/bintests2.log 2>&1 || { echo "bin tests failed"; tail -30 gpurun_out/bintests2.log; exit 1; }
tail -3 gpurun_out/bintests2.log
for i in 1 2; do
timeout -k 10 200 python bench.py --task binpick --no-cpu-baseline > gpurun_out/ab_kl2_$i.json || exit 1
timeout -k 10 200 python -c "
import sys, runpy; sys.path[:0]=['isaacgym-hand-arm_amd']
from handarm_hip import _lib; _lib.LIB_PATH='$R/isaacgym-hand-arm_amd/handarm_hip/libhandarm_hip_kl8.so'
sys.argv=['bench.py','--task','binpick','--no-cpu-baseline']; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/ab_kl8_$i.json || exit 1
done
for f in gpurun_out/ab_*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), d['roofline']['kernel_avg_ms'])"; done
