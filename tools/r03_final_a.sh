#!/usr/bin/env bash
# Round-3 GPU pass A: GPU suite, smoke, default bench line, then the C2 / C3 profile sets (outputs in gpurun_out/)
bash tools/gpu_round.sh \
  "gputest|600|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "benchall|400|python -u bench.py > gpurun_out/r03_bench_all.json" && \
bash tools/profile_round.sh r03 allegro_kuka && bash tools/profile_round.sh r03 allegro_hand
