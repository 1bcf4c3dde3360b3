#!/bin/bash
# Round-6 GPU check 13: knob sweep around the DEFAULT schedule (gemm4_sched 0 = FAST SCHED 1) on the shapes
# where hipBLASLt leads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "500|gsweep2|python -u tools/gemm4_probe.py --rounds 4 --iters 10 --layouts nt nn --shapes gateup lmhead --scheds 1 0 --bn 192 256 --group-m 1 2 8 16 --br 1 2"
