#!/usr/bin/env bash
# Round-3 final GPU pass: GPU suite, smoke, the default bench line (with CPU baselines), then all four profile sets
bash tools/gpu_round.sh \
  "gputest|600|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
  "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "benchall|500|python -u bench.py > gpurun_out/r03_bench_all.json" && \
for t in allegro_kuka allegro_hand ur5sih binpick; do bash tools/profile_round.sh r03 $t || exit $?; done
