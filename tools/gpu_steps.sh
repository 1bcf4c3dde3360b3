#!/bin/bash
# Run a sequence of GPU steps on the box, each under its own time limit; stop at the first
# step that faults / aborts / segfaults / times out (exit status other than 0 or 1).
# Usage: tools/gpu_steps.sh "<secs>|<name>|<cmd>" ...
# Output of each step goes to gpurun_out/<name>.log; a summary line per step is printed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done
