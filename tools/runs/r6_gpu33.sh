#!/bin/bash
# Round-6 GPU check 33: the non-temporal-store GEMM variants as per-shape candidates (timed alone)
# vs excluded -- same-box interleaved bench A/B (ops.gemm_select.NT_STORES).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "900|ab_nt|python3 tools/ab_attr.py --rounds 3 '' 'ops.gemm_select.NT_STORES=False' -- --steps 20"
