#!/bin/bash
# Round-6 GPU check 44: end-of-round per-shape GEMM table (default schedule, barrier row 2) vs hipBLASLt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "400|shapes|python3 tools/gemm4_probe.py --rounds 4 --iters 10 --scheds 0"
