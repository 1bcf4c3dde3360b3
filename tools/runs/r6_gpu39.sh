#!/bin/bash
# Round-6 GPU check 39: end-of-round re-check of the A/B hooks whose balance the attention
# bias fix could have moved (attention stagger / cross-block prefetch, GEMM barrier row).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "900|ab_hooks|python3 tools/ab_attr.py --rounds 3 '' 'ext:attn_stagger(2)' 'ext:attn_prefetch(0)' 'ext:gemm4_br(1)' -- --steps 20"
