#!/usr/bin/env bash
# Round-3 A/B 2: parity of the wavefront-scope wsync build, then product vs the workgroup-barrier build per task
T="-q --timeout 200 --timeout-method thread"
bash tools/gpu_round.sh "bits|400|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kuka.py tests/test_gpu_allegro.py tests/test_gpu_bin.py tests/test_gpu_edges.py tests/test_gpu_dr.py tests/test_gpu_pointcloud.py tests/test_gpu_camera.py -x $T" && \
for t in allegro_kuka allegro_hand ur5sih binpick; do AB_ROUNDS=2 bash tools/ab_variants.sh $t product libhandarm_hip_wblk.so > gpurun_out/ab_wsync_$t.txt 2>&1; done
