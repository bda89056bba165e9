#!/usr/bin/env bash
# Round-4 GPU check: parity tests of the new paths, the whole GPU suite, the default bench and phase profiles of the
# Allegro configs (self-collision cost). Usage (GPU box): bash tools/r04_round_a.sh TAG
TAG=${1:-r4}
bash tools/gpu_round.sh \
  "${TAG}_new|400|python -u -m pytest tests/test_gpu_self_collision.py tests/test_gpu_fused_steps.py tests/test_gpu_overflow.py -x -v --timeout 200 --timeout-method thread" \
  "${TAG}_all|500|python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread" \
  "${TAG}_bench|400|python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/${TAG}_bench.json" \
  "${TAG}_prof_kuka|200|python -u tools/phase_profile.py --kuka" \
  "${TAG}_prof_allegro|200|python -u tools/phase_profile.py --allegro"
