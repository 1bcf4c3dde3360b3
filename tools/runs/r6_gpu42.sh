#!/bin/bash
# Round-6 GPU check 42: barrier row 1 in the SwiGLU / SwiGLU-backward / RoPE forms and 2 in the non-temporal-store forms (was: barrier row 2 in the SwiGLU / SwiGLU-backward / RoPE / non-temporal-store
# GEMM forms too -- GEMM + model GPU tests (fused forms checked bitwise against the separate
# kernels), step A/B against the plain-forms-only build (same box, interleaved).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "500|tests|python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k 'gemm or swiglu or rope or model or train or bitwise or reproducib'" \
  "900|bench|bash tools/ab_so.sh 'new old new old new old new old' python3 bench.py"
