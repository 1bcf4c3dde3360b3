#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "700|suite3|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k 'not rehearsal' -p no:cacheprovider"
