#!/bin/bash
# Round-6 GPU check 25: attention kernels alone vs in step-like context (cache flushed, after a
# GEMM, with inverse RoPE + bias gradient) -- where the step's extra ~0.09 ms per layer comes from.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "200|ctx_bwd|python3 tools/attn_ctx_probe.py" \
  "200|ctx_fwd|python3 tools/attn_ctx_probe.py --fwd"
