#!/usr/bin/env bash
# Persistent-manifold A/B on the GPU box: each task's bench line with the default tolerances, with the records off
# (HA_PCM=off: same binary, every candidate pair runs its narrow phase) and with looser tolerances.
# Usage: bash tools/diag/pcm_ab.sh TAG "TASK ..." "TOL ..."   (TOL: off or lin,cos)
TAG=${1:-pcm}
TASKS=${2:-"allegro_kuka allegro_hand ur5sih binpick"}
TOLS=${3:-"default off 1e-3,0.9998"}
for t in $TASKS; do
  for tol in $TOLS; do
    if [ "$tol" = default ]; then unset HA_PCM; else export HA_PCM=$tol; fi
    out=gpurun_out/${TAG}_${t}_${tol//,/_}.json
    timeout -k 10 300 python bench.py --task $t --no-cpu-baseline --steps 40 > $out 2>/dev/null || exit 1
    python - "$out" "$t" "$tol" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
e = d.get('episode_window')
c = d.get('contacts', {})
print(f"{sys.argv[2]:13s} pcm {sys.argv[3]:14s} {d['value']:12.0f} env-steps/s  kernel {d['roofline']['kernel_avg_ms']:.3f} ms"
      f"  refreshed {c.get('pcm_refreshed_per_substep', 0):.2f} narrow {c.get('narrow_phases_per_substep', 0):.2f}"
      + (f"  episode {e['value']:.0f} ({e['ms_per_step']:.3f} ms)" if e else ""))
PY
  done
done
unset HA_PCM
