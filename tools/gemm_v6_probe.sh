#!/bin/bash
# v3 (impl 3) vs v6 8-phase (impl 4) vs hipBLASLt on the GPT-2 small TP 1 step's GEMM shapes
# (M = 32 x 1024 tokens; (N, K) per projection: QKV, Wo, gate|up, down, lm_head), all three
# layouts, with the relative error of each implementation against fp32 torch.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for layout in ${LAYOUTS:-nt nn tn}; do
  for nk in 2304,768 768,768 4096,768 768,2048 50304,768; do
    N=${nk%,*}; K=${nk#*,}
    python tools/gemm_probe.py --layout "$layout" --M 32768 --N "$N" --K "$K" --impl 3 4 --iters 20 --blas --check
  done
done
