#!/usr/bin/env bash
# Round-3 final GPU pass 3: GPU suite, smoke, the default bench line, the C2 kernel stats, and a C2 kernel trace
bash tools/gpu_round.sh \
  "gputest|600|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "benchall|500|python -u bench.py > gpurun_out/r03_bench_all.json" \
  "ks|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/ks -- python3 $PWD/bench.py --task allegro_kuka --steps 20 --warmup 5 --no-cpu-baseline" \
  "ksx|60|cp gpurun_out/ks/*/*_kernel_stats.csv gpurun_out/r03_bench_kernel_stats.csv && cp gpurun_out/ks/*/*_kernel_trace.csv gpurun_out/r03_kernel_trace_kuka.csv && rm -rf gpurun_out/ks"
