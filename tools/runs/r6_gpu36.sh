#!/bin/bash
# Round-6 GPU check 36: NN data-gradient GEMMs vs the same products in the NT layout on a
# pre-transposed weight (would a transposed weight shadow pay?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "400|nnnt|python3 tools/nn_vs_nt_probe.py --rounds 5 --iters 10"
