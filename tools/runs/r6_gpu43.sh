#!/bin/bash
# Round-6 GPU check 43: screen of the remaining GEMM A/B hooks with barrier row 2 as the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "1000|ab_screen|python3 tools/ab_attr.py --rounds 3 '' 'ext:gemm4_sched(1)' 'ext:gemm4_m32k(2)' 'ext:gemm4_swb_depth(1)' 'ext:gemm4_group_m(8)' -- --steps 20"
