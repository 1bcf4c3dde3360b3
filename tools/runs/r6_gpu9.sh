#!/bin/bash
# Round-6 GPU check 9: forward with scale + running max folded into the MFMAs (impl 8): oracle /
# rescale tests, per-call A/B, headline A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "240|t_fwd8|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'test_attention'" \
  "240|probe_fwd8|python -u tools/attn_probe.py --impl 4 8 4 8 --iters 20 && python -u tools/attn_probe.py --impl 4 8 4 8 --iters 10 --hd 128 --H 32 --T 4096 --B 2" \
  "400|ab_fwd8|bash tools/ab_env.sh DPFS_ATTN_IMPL '0 8 0 8'"
