#!/usr/bin/env bash
# Diagnostic A/B of library builds: bench value + PMC HBM traffic of the task's step kernel per build.
# Usage (GPU box): bash tools/diag/ab_traffic.sh TASK KERNEL ENVS lib1.so|product ...
R=$PWD; TASK=$1; K=$2; ENVS=$3; shift 3; O=$R/gpurun_out
for L in "$@"; do
  N=${L%.so}
  B="python3 $R/tools/diag/lib_bench.py $L $TASK --steps 20 --warmup 5"
  bash "$R/tools/gpu_round.sh" \
    "abt_${N}_${TASK}|200|$B > $O/abt_${N}_${TASK}.json" \
    "abt_f|200|cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/abtf -- $B" \
    "abt_w|200|cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/abtw -- $B" \
    "abt_t|60|python $R/tools/pmc_traffic.py --fetch $O/abtf --write $O/abtw --envs $ENVS --kernel $K --out $O/abt_traffic_${N}_${TASK}.json && rm -rf $O/abtf $O/abtw" || exit 1
  python3 - <<PY
import json
d = json.loads([l for l in open("$O/abt_${N}_${TASK}.json") if l.startswith("{")][-1])
t = json.load(open("$O/abt_traffic_${N}_${TASK}.json"))
print("$N $TASK: %.3f M env-steps/s, kernel %.3f ms, HBM %.1f KB/env (write %.0f KiB raw)" % (d["value"] / 1e6,
      d["roofline"]["kernel_avg_ms"], t["hbm_bytes_per_env"] / 1e3, t["write_size_kib_raw"]))
PY
done
