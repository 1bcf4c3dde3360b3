#!/bin/bash
# Round-6 GPU check 37: end-of-round full-size driver protocol rehearsals at N = 2 and N = 4 (all
# ranks on one MI355X over gloo + the xGMI transport decision), after the attention changes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
( while sleep 50; do date >> gpurun_out/tick37.log; done ) &
TICK=$!
bash tools/gpu_steps.sh \
  "300|rh2|bash tools/rehearsal_full.sh 2" \
  "500|rh4|bash tools/rehearsal_full.sh 4"
rc=$?
kill $TICK
exit $rc
