#!/bin/bash
# Round-6 GPU check 14: GEMM tile-row group size A/B on the headline step; where the stray
# (non-dpfs) kernels of the bf16 / fp32 steps come from.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "600|ab_gm|bash tools/ab_env.sh DPFS_GEMM_GROUP_M '4 16 8 4 16 8'" \
  "200|stray16|python -u tools/find_stray_kernels.py" \
  "200|stray32|python -u tools/find_stray_kernels.py --fp32"
