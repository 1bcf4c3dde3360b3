#!/bin/bash
# Round-6 GPU check 12: knob sweep on the shapes where hipBLASLt leads (gate|up NT / NN, lm_head NT, down NT).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "500|gsweep|python -u tools/gemm4_probe.py --rounds 3 --iters 10 --layouts nt nn --shapes gateup lmhead down --scheds 0 2 1 --bn 192 256 --group-m 1 2 8 16 --br 1 2 --sk"
