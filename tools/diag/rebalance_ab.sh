#!/usr/bin/env bash
# Dispatch-order refresh interval (HA_REBALANCE: fused steps between two refreshes, 0 = identity order) on the bench
# tasks, alternating: bash tools/diag/rebalance_ab.sh "TASK ..." "R ..."   (GPU box; prints value and kernel ms)
TASKS=${1:-"allegro_kuka allegro_hand"}; RS=${2:-"4 2 1"}
for t in $TASKS; do
  for rep in 1 2; do
    for r in $RS; do
      HA_REBALANCE=$r timeout -k 10 300 python bench.py --task $t --no-cpu-baseline > gpurun_out/rb_${t}_$r.json 2>/dev/null || exit 1
      python -c "import json; d=json.loads([l for l in open('gpurun_out/rb_${t}_$r.json') if l.startswith('{')][-1]); e=d.get('episode_window'); print('$t rebalance $r', round(d['value']), round(d['roofline']['kernel_avg_ms'],3), ('episode %d %.3f' % (e['value'], e['ms_per_step'])) if e else '')"
    done
  done
done
