#!/usr/bin/env bash
# Quick GPU iteration: bit-for-bit physics tests of every family, then the default bench (all configs, no CPU
# baseline). Usage (on the GPU box): bash tools/quick_gpu.sh TAG
TAG=${1:-q}
bash tools/gpu_round.sh \
  "${TAG}_bits|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kuka.py tests/test_gpu_allegro.py tests/test_gpu_bin.py tests/test_gpu_dr.py -x -q --timeout 200 --timeout-method thread" \
  "${TAG}_bench|400|python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/${TAG}_bench.json"
