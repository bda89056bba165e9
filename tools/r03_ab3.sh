#!/usr/bin/env bash
# Round-3 A/B 3: parity of the recomputed clutter rows, then product vs stored rows on C5, then the bench line
T="-q --timeout 200 --timeout-method thread"
bash tools/gpu_round.sh "bits|400|python -u -m pytest tests/test_gpu_bin.py tests/test_gpu_parity.py tests/test_gpu_dr.py tests/test_gpu_kuka.py -x $T" && \
AB_ROUNDS=2 bash tools/ab_variants.sh binpick product libhandarm_hip_norc.so > gpurun_out/ab_recompute_binpick.txt 2>&1
bash tools/gpu_round.sh "benchall|400|python -u bench.py --no-cpu-baseline > gpurun_out/r03c_bench_all.json"
HA_LIB=$PWD/isaacgym-hand-arm_amd/handarm_hip/libhandarm_hip_segsat.so bash tools/gpu_round.sh "segbits|300|python -u -m pytest tests/test_gpu_kuka.py tests/test_gpu_allegro.py tests/test_gpu_edges.py tests/test_gpu_bin.py -x $T"
for t in allegro_kuka allegro_hand ur5sih; do AB_ROUNDS=2 bash tools/ab_variants.sh $t product libhandarm_hip_segsat.so > gpurun_out/ab_segsat_$t.txt 2>&1; done
