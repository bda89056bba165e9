#!/usr/bin/env bash
# Run GPU steps in order; stop at the first step that hung, crashed or faulted (rc 124/137/134/139/>128).
# Usage: tools/gpu_round.sh "name|timeout|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (timeout ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "=== stopping: step $name ended abnormally (rc=$rc)"; exit $rc
  fi
done
exit 0
