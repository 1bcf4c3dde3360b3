#!/bin/bash
# Round-6 GPU check 32: QKV GEMM RoPE epilogue with the 8 row blocks' positions loaded before the
# accumulator drain (one dependent load per block instead of two) -- RoPE GEMM + model tests,
# step A/B against the previous build (same box, interleaved), the QKV+RoPE call in the trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|tests|python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k 'rope or qkv or model or train'" \
  "600|bench|bash tools/ab_so.sh 'new old new old new old' python3 bench.py" \
  "300|prof|bash tools/prof_step.sh r6ropeq"
