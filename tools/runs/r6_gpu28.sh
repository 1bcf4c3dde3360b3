#!/bin/bash
# Round-6 GPU check 28: attention backward epilogues with the RoPE position load issued early (dQ:
# with the block's prologue; dK/dV: before dV's stores and column sums, which run under it) and
# the fp32 attention's bias partials as a transpose reduction -- attention + fp32 tests, context
# probe and step A/B against the previous build (same box, interleaved).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "300|attn_tests|python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fp32_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attention or f32 or fp32'" \
  "300|ctx|bash tools/ab_so.sh 'new old new old' python3 tools/attn_ctx_probe.py --n 20" \
  "500|bench|bash tools/ab_so.sh 'new old new old' python3 bench.py"
