#!/bin/bash
# Round-6 GPU check 26: the attention backward's QKV bias-gradient partials as a transpose
# reduction (lane32_sums: 31 lane exchanges per 32 values instead of 160 ds_bpermute) -- bias
# tests, context probe and step A/B against the previous build (same box, interleaved).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "300|attn_tests|python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attention and not f32 and not decode'" \
  "300|ctx|bash tools/ab_so.sh 'new old new old' python3 tools/attn_ctx_probe.py --n 20" \
  "500|bench|bash tools/ab_so.sh 'new old new old' python3 bench.py"
