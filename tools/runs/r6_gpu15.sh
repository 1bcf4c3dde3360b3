#!/bin/bash
# Round-6 GPU check 15: call sites of the stray (non-dpfs) kernels; per-shape GEMM table at the default schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "200|stray16b|python -u tools/find_stray_kernels.py" \
  "200|stray32b|python -u tools/find_stray_kernels.py --fp32" \
  "500|gprobe0|python -u tools/gemm4_probe.py --rounds 4 --iters 10 --scheds 0"
