#!/bin/bash
# Round-6 GPU check 46: barrier row in the 32x32x16 TN (weight-gradient) main loop (hook
# gemm4_br_tn, default 0) -- bitwise training check at 0 / 1 / 2, GEMM tests with the new build,
# step A/B of the hook.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "300|bitwise|python3 tools/tn_br_bitwise.py" \
  "400|tests|python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k 'gemm or tn'" \
  "1000|ab|python3 tools/ab_attr.py --rounds 4 '' 'ext:gemm4_br_tn(1)' 'ext:gemm4_br_tn(2)' -- --steps 20"
