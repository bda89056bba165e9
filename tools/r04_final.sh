#!/usr/bin/env bash
# Round-4 closing measurements on one GPU box (run in two or three gpurun calls by PART):
#   PART=a: the GPU suite, smoke, the default bench line (all configs, CPU baselines, episode windows)
#   PART=b: rocprof kernel stats + PMC traffic / SQ passes of the C2 and C3 step kernels (tools/profile_round.sh)
#   PART=c: the same for C4 and C5, then phase profiles and workgroup spans
TAG=${TAG:-r04}; PART=${1:-a}
case $PART in
  a) bash tools/gpu_round.sh \
       "${TAG}_gpu_suite|600|python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
       "${TAG}_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
       "${TAG}_bench_all|900|python -u bench.py > gpurun_out/${TAG}_bench_all.json" ;;
  b) bash tools/profile_round.sh "$TAG" allegro_kuka && bash tools/profile_round.sh "$TAG" allegro_hand ;;
  c) bash tools/profile_round.sh "$TAG" ur5sih && bash tools/profile_round.sh "$TAG" binpick ;;
  d) bash tools/gpu_round.sh \
       "${TAG}_phase_kuka|200|python -u tools/phase_profile.py --kuka > gpurun_out/${TAG}_phase_profile_kuka.txt" \
       "${TAG}_phase_allegro|300|python -u tools/phase_profile.py --allegro > gpurun_out/${TAG}_phase_profile_allegro.txt" \
       "${TAG}_phase_c4|300|HA_PROFILE_POOL=1 HA_PROFILE_WARM=120 python -u tools/phase_profile.py --c4 > gpurun_out/${TAG}_phase_profile_c4_late.txt" \
       "${TAG}_envt_kuka|200|python -u tools/phase_profile.py --kuka --envt-only > gpurun_out/${TAG}_env_spans_kuka.txt" \
       "${TAG}_envt_c4|300|HA_PROFILE_POOL=1 HA_PROFILE_WARM=120 python -u tools/phase_profile.py --c4 --envt-only > gpurun_out/${TAG}_env_spans_c4_late.txt" \
       "${TAG}_timeline_c4|300|python -u tools/diag/episode_timeline.py > gpurun_out/${TAG}_episode_timeline_c4.txt" ;;
esac
