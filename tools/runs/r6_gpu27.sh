#!/bin/bash
# Round-6 GPU check 27: transpose-reduced bias partials in every attention backward variant --
# attention + model GPU tests, then the timed-step kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|attn_tests|python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attention and not decode'" \
  "400|model_tests|python3 -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread" \
  "300|prof|bash tools/prof_step.sh r6bias"
