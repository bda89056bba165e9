#!/usr/bin/env bash
# GPU-box profiling pass for one round and task: bench line, rocprofv3 kernel stats, PMC HBM traffic and SQ
# counters of the task's step kernel.
# Usage: bash tools/profile_round.sh rNN [allegro_kuka|ur5sih|allegro_hand|binpick|ur5sih_wide]   (outputs under
# gpurun_out/; ur5sih_wide (C4w) shares ha_step_kernel with C4 and writes sq_/traffic_ha_step_kernel_C4w.json)
set -o pipefail
R=$PWD; TAG=${1:-r01}; TASK=${2:-allegro_kuka}; O=$R/gpurun_out; WL=""
case $TASK in
  allegro_kuka) K=ak_step_kernel; ENVS=4096; SFX="" ;;
  ur5sih) K=ha_step_kernel; ENVS=8192; SFX="_ur5sih" ;;
  allegro_hand) K=ah_step_kernel; ENVS=16384; SFX="_allegro" ;;
  binpick) K=hb_step_kernel; ENVS=8192; SFX="_binpick" ;;
  ur5sih_wide) K=ha_step_kernel; ENVS=8192; SFX="_c4w"; WL=C4w ;;
  *) echo "unknown task $TASK"; exit 2 ;;
esac
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
B="python3 $R/bench.py --task $TASK --steps 20 --warmup 5 --no-cpu-baseline"
bash "$R/tools/gpu_round.sh" \
  "bench|600|python $R/bench.py --task $TASK --cpu-seconds 6 > $O/${TAG}_bench${SFX}.json" \
  "ks|400|$P --kernel-trace --stats --output-format csv -d $O/ks -- $B" \
  "ksx|60|cp $O/ks/*/*_kernel_stats.csv $O/${TAG}_bench${SFX}_kernel_stats.csv && rm -rf $O/ks" \
  "pmcf|400|$P --pmc FETCH_SIZE --output-format csv -d $O/pmcf -- $B" \
  "pmcw|400|$P --pmc WRITE_SIZE --output-format csv -d $O/pmcw -- $B" \
  "traffic|60|python $R/tools/pmc_traffic.py --fetch $O/pmcf --write $O/pmcw --envs $ENVS --kernel $K ${WL:+--workload $WL} --out $O/traffic_$K${WL:+_$WL}.json && python $R/tools/pmc_extract.py $O/pmcf --kernel $K --out $O/${TAG}_pmc_fetch${SFX}.csv --delete && python $R/tools/pmc_extract.py $O/pmcw --kernel $K --out $O/${TAG}_pmc_write${SFX}.csv --delete" \
  "sq1|400|$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/sq1 -- $B" \
  "sq1x|60|python $R/tools/pmc_extract.py $O/sq1 --kernel $K --out $O/${TAG}_sq1${SFX}.csv --delete > $O/${TAG}_sq1${SFX}_summary.txt" \
  "sq2|400|$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA --output-format csv -d $O/sq2 -- $B" \
  "sq2x|60|python $R/tools/pmc_extract.py $O/sq2 --kernel $K --out $O/${TAG}_sq2${SFX}.csv --delete > $O/${TAG}_sq2${SFX}_summary.txt" \
  "sq3|400|$P --pmc SQ_THREAD_CYCLES_VALU --output-format csv -d $O/sq3 -- $B" \
  "sq3x|60|python $R/tools/pmc_extract.py $O/sq3 --kernel $K --out $O/${TAG}_sq3${SFX}.csv --delete > $O/${TAG}_sq3${SFX}_summary.txt" \
  "sqsum|60|python $R/tools/sq_summary.py $O/${TAG}_sq1${SFX}.csv $O/${TAG}_sq2${SFX}.csv $O/${TAG}_sq3${SFX}.csv --kernel $K --envs $ENVS ${WL:+--workload $WL} --out $O/sq_$K${WL:+_$WL}.json"
