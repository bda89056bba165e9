#!/usr/bin/env bash
# Round-3 A/B 4: AllegroKuka with 3 LDS link slots (S after the rows in the union), and the dispatch-order interval
L=$PWD/isaacgym-hand-arm_amd/handarm_hip
T="-q --timeout 200 --timeout-method thread"
bash tools/gpu_round.sh "bits|300|python -u -m pytest tests/test_gpu_kuka.py tests/test_gpu_edges.py -x $T" \
  "kl3bits|300|HA_LIB=$L/libhandarm_hip_kl3.so python -u -m pytest tests/test_gpu_kuka.py tests/test_gpu_edges.py -x $T" && \
AB_ROUNDS=2 bash tools/ab_variants.sh allegro_kuka product libhandarm_hip_kl3.so > gpurun_out/ab_kl3.txt 2>&1
for rb in 0 4 16; do for t in allegro_kuka allegro_hand ur5sih; do HA_REBALANCE=$rb AB_ROUNDS=1 bash tools/ab_variants.sh $t product > gpurun_out/ab_rb${rb}_$t.txt 2>&1; done; done
