#!/usr/bin/env bash
# GPU-box profiling pass for one round: default bench line, rocprofv3 kernel stats, PMC HBM traffic and
# SQ counters of ha_step_kernel. Usage: bash tools/profile_round.sh rNN   (outputs under gpurun_out/)
set -o pipefail
R=$PWD; TAG=${1:-r01}; O=$R/gpurun_out
P="cd /tmp && export TMPDIR=/tmp && rocprofv3"
B="python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline"
bash "$R/tools/gpu_round.sh" \
  "bench|600|python $R/bench.py > $O/${TAG}_bench.json" \
  "ks|400|$P --kernel-trace --stats --output-format csv -d $O/ks -- $B" \
  "ksx|60|cp $O/ks/*/*_kernel_stats.csv $O/${TAG}_bench_kernel_stats.csv && rm -f $O/ks/*/*_kernel_trace.csv" \
  "pmcf|400|$P --pmc FETCH_SIZE --output-format csv -d $O/pmcf -- $B" \
  "pmcw|400|$P --pmc WRITE_SIZE --output-format csv -d $O/pmcw -- $B" \
  "traffic|60|python $R/tools/pmc_traffic.py --fetch $O/pmcf --write $O/pmcw --envs 8192 --out $O/traffic_step_kernel.json && python $R/tools/pmc_extract.py $O/pmcf --out $O/${TAG}_pmc_fetch_step.csv --delete && python $R/tools/pmc_extract.py $O/pmcw --out $O/${TAG}_pmc_write_step.csv --delete" \
  "sq1|400|$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/sq1 -- $B" \
  "sq1x|60|python $R/tools/pmc_extract.py $O/sq1 --out $O/${TAG}_sq1_step.csv --delete > $O/${TAG}_sq1_summary.txt" \
  "sq2|400|$P --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA --output-format csv -d $O/sq2 -- $B" \
  "sq2x|60|python $R/tools/pmc_extract.py $O/sq2 --out $O/${TAG}_sq2_step.csv --delete > $O/${TAG}_sq2_summary.txt"
