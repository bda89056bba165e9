#!/usr/bin/env bash
# Round-3 A/B pass (GPU box): parity of the product build, the divergent-pair diagnostics, dispatch order on/off,
# the sphere pre-cull on/off, and the contact-capacity layouts. Outputs under gpurun_out/.
L=$PWD/isaacgym-hand-arm_amd/handarm_hip
T="-q --timeout 200 --timeout-method thread"
bash tools/gpu_round.sh \
  "bits|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kuka.py tests/test_gpu_allegro.py tests/test_gpu_bin.py tests/test_gpu_edges.py tests/test_gpu_dr.py -x $T" \
  "xdiv|200|HA_LIB=$L/libhandarm_hip_xdiv.so python -u -m pytest tests/test_gpu_kuka.py tests/test_gpu_allegro.py tests/test_gpu_edges.py $T" \
  "xdivloop|200|HA_LIB=$L/libhandarm_hip_xdivloop.so python -u -m pytest tests/test_gpu_kuka.py tests/test_gpu_edges.py $T" \
  "rb0|200|HA_REBALANCE=0 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/rb0.json" \
  "rb8|200|HA_REBALANCE=8 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/rb8.json" \
  "nocull|200|HA_NP_FLAGS=4 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/nocull.json" \
  "abk|300|AB_ROUNDS=1 bash tools/ab_variants.sh allegro_kuka libhandarm_hip_c21.so && cp gpurun_out/ab_libhandarm_hip_c21_1.json gpurun_out/ab_ak_c21.json" \
  "aba|300|AB_ROUNDS=1 bash tools/ab_variants.sh allegro_hand libhandarm_hip_c21.so libhandarm_hip_ahc12.so && cp gpurun_out/ab_libhandarm_hip_c21_1.json gpurun_out/ab_ah_c21.json"
