#!/bin/bash
# Round-6 GPU check 11: per-shape GEMM timings of the GPT-2 small step (v4 vs hipBLASLt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "500|gprobe|python -u tools/gemm4_probe.py --rounds 3 --iters 10 --scheds 1"
