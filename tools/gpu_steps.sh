#!/bin/bash
# Run GPU steps in order; stop at the first fault / abort / timeout / signal
# (exit codes 124, 134, 137, 139 or >128), continue past plain test failures.
# usage: tools/gpu_steps.sh "name|timeout|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== step $name (timeout ${to}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== step $name rc=$rc ($(( $(date +%s) - start ))s)" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit 0
