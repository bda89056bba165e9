#!/usr/bin/env bash
# Dispatch-order cost: the workgroup-span estimate (HA_ORDER_COST=time, HandArmSim's default) vs the contacts offered
# (HA_ORDER_COST=contacts; any other value is rejected by HandArmSim), alternating
# runs: bash tools/diag/order_cost_ab.sh "TASK ..."   (GPU box; prints value and kernel ms)
TASKS=${1:-"allegro_kuka allegro_hand ur5sih"}
for t in $TASKS; do
  for rep in 1 2; do
    for c in contacts time; do
      HA_ORDER_COST=$c timeout -k 10 300 python bench.py --task $t --no-cpu-baseline > gpurun_out/oc_${t}_$c.json 2>/dev/null || exit 1
      python -c "import json; d=json.loads([l for l in open('gpurun_out/oc_${t}_$c.json') if l.startswith('{')][-1]); e=d.get('episode_window'); print('$t cost $c', round(d['value']), round(d['roofline']['kernel_avg_ms'],3), ('episode %d %.3f' % (e['value'], e['ms_per_step'])) if e else '')"
    done
  done
done
