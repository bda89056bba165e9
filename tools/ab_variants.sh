#!/usr/bin/env bash
# A/B of diagnostic library builds on one bench task: bash tools/ab_variants.sh TASK lib1.so lib2.so ...
# (paths relative to isaacgym-hand-arm_amd/handarm_hip/; "product" = libhandarm_hip.so). Two alternating rounds,
# one bench process per (build, round); prints value and mean step-kernel ms per run.
R=$PWD; TASK=$1; shift
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for L in "$@"; do
    [ "$L" = product ] && L=libhandarm_hip.so
    timeout -k 10 200 python -c "
import sys, runpy; sys.path[:0]=['isaacgym-hand-arm_amd']
from handarm_hip import _lib; _lib.LIB_PATH='$R/isaacgym-hand-arm_amd/handarm_hip/$L'
sys.argv=['bench.py','--task','$TASK','--no-cpu-baseline']; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/ab_${L%.so}_$i.json || exit 1
    python -c "import json; d=json.loads([l for l in open('gpurun_out/ab_${L%.so}_$i.json') if l.startswith('{')][-1]); e=d.get('episode_window'); print('$L round $i', round(d['value']), round(d['roofline']['kernel_avg_ms'], 3), ('episode %d %.3f ms' % (e['value'], e['ms_per_step'])) if e else '')"
  done
done
