#!/bin/bash
# Round-6 GPU check 40: GEMM barrier-row hook (rows of MFMAs before each step's barrier), 6 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "1000|ab_br|python3 tools/ab_attr.py --rounds 6 '' 'ext:gemm4_br(1)' 'ext:gemm4_br(2)' -- --steps 20"
