#!/bin/bash
# Round-6 GPU check 18: where a short-K NT GEMM tile's time goes (gemm4 DIAG split: step-entry
# wait / body / epilogue per tile) for lm_head and gate|up, default schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|gdiag|python -u tools/gemm4_probe.py --layouts nt --shapes lmhead gateup qkv --scheds 0 --rounds 1 --iters 5 --diag --no-blas"
bash tools/gpu_steps.sh \
  "600|suite2|python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k 'not rehearsal' -p no:cacheprovider"
