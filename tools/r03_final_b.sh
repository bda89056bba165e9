#!/usr/bin/env bash
# Round-3 GPU pass B: joint-row exchange A/B, C5 phase profile, then the C4 / C5 profile sets (gpurun_out/)
AB_ROUNDS=2 bash tools/ab_variants.sh allegro_hand product libhandarm_hip_jser.so > gpurun_out/ab_jser_ah.txt 2>&1
AB_ROUNDS=2 bash tools/ab_variants.sh allegro_kuka product libhandarm_hip_jser.so > gpurun_out/ab_jser_ak.txt 2>&1
bash tools/gpu_round.sh "pbin|200|python -u tools/phase_profile.py --bin" && \
bash tools/profile_round.sh r03 ur5sih && bash tools/profile_round.sh r03 binpick
