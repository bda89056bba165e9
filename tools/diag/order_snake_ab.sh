#!/usr/bin/env bash
# Alternate-block reversal of the dispatch order (HA_ORDER_SNAKE = block size, 0 = plain longest-first), alternating
# runs: bash tools/diag/order_snake_ab.sh "TASK ..." "S ..."   (GPU box; prints value and kernel ms)
TASKS=${1:-"allegro_kuka allegro_hand"}; SS=${2:-"0 256"}
for t in $TASKS; do
  for rep in 1 2; do
    for sn in $SS; do
      HA_ORDER_SNAKE=$sn timeout -k 10 300 python bench.py --task $t --no-cpu-baseline > gpurun_out/sn_${t}_$sn.json 2>/dev/null || exit 1
      python -c "import json; d=json.loads([l for l in open('gpurun_out/sn_${t}_$sn.json') if l.startswith('{')][-1]); e=d.get('episode_window'); print('$t snake $sn', round(d['value']), round(d['roofline']['kernel_avg_ms'],3), ('episode %d %.3f' % (e['value'], e['ms_per_step'])) if e else '')"
    done
  done
done
