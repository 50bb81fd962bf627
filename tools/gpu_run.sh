#!/bin/bash
# Run GPU steps in order, each under its own time limit.  A step that ends in
# a timeout (124/137), abort (134), segfault (139) or any signal ends the whole
# script: nothing else touches the GPU after a fault.  Ordinary test failures
# (exit 1/2) are recorded and the next step runs.
# usage: tools/gpu_run.sh "<seconds>|<name>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
mkdir -p gpurun_out
rc_all=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc after $(( $(date +%s) - start )) s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping: step $name ended abnormally ($rc)"; exit $rc
  fi
  if grep -qE "Memory access fault|PRK_ERR_DEVICE|HSA_STATUS_ERROR|hipErrorLaunchFailure|illegal memory|page fault|GPU core dump" "gpurun_out/$name.log"; then
    echo "=== stopping: step $name shows a device fault"; exit 99
  fi
  [ $rc -ne 0 ] && rc_all=$rc
done
exit $rc_all
