#!/bin/bash
# Round-6 validation: the whole GPU suite (the N-rank rehearsal test separately, with a progress
# ticker), smoke(), the headline bench and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/tick.log; done ) &
TICK=$!
bash tools/gpu_steps.sh \
  "1000|suite|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k 'not rehearsal' -p no:cacheprovider" \
  "700|suite_rh|python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k rehearsal -p no:cacheprovider" \
  "300|smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|bench|python -u bench.py" \
  "300|prof_final|bash tools/prof_step.sh r6final6"
rc=$?
kill $TICK
exit $rc
