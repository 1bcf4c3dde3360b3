#!/bin/bash
# Round-6 GPU check 30: after the bias-partials fix -- backward implementations as the step calls
# them (RoPE + bias), the dK/dV DIAG split, and the fp32 (reference default) training step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "200|impls|python3 tools/attn_ctx_probe.py --impls 4 6 7 9 --n 20" \
  "200|diag|python3 tools/attn_probe.py --bwd --diag --impl 4 --iters 5" \
  "300|fp32|python3 bench.py --fp32 --model reference --seq-len 1000 --steps 10 --warmup 3"
