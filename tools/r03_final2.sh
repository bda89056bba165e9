#!/usr/bin/env bash
# Round-3 final GPU pass 2 (dispatch order every 4 steps, custom teacher lists): GPU suite, smoke, default bench
# line with CPU baselines, C2 profile set
bash tools/gpu_round.sh \
  "gputest|600|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "benchall|500|python -u bench.py > gpurun_out/r03_bench_all.json" && \
bash tools/profile_round.sh r03 allegro_kuka
