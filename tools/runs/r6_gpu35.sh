#!/bin/bash
# Round-6 GPU check 35: end-of-round same-box A/B of ours-only GEMMs (default) vs hipBLASLt
# competing per shape (DPFS_GEMM_LIB=1), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "900|ab_lib|bash tools/ab_env.sh DPFS_GEMM_LIB '0 1 0 1 0 1' --steps 20"
