#!/bin/bash
# Round-6 GPU check 48: QKV GEMM RoPE epilogue with the cos / sin table values two row blocks
# ahead (two register sets) -- RoPE GEMM tests, per-call time in the step trace, step A/B vs the
# previous build (same box, interleaved).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|tests|python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k 'rope or qkv or model or train'" \
  "900|bench|bash tools/ab_so.sh 'new old new old new old new old' python3 bench.py"
