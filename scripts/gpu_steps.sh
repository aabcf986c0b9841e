#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/.
# Usage: scripts/gpu_steps.sh "name|seconds|command" ...
# An ordinary failure (exit 1/2) is logged and the next step runs; a timeout,
# abort, segfault or kill (124/134/137/139, or >128) stops the whole call.
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start )) s" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then status=$rc; fi
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "=== fatal rc=$rc: stopping" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit $status
