#!/bin/bash
# Round-6 GPU check 29: the step's dispatch sequence (per-call GEMM times by position / grid) and
# the GEMM shape choices, vs the same GEMMs timed alone (NT with bias, default schedule).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
R=$PWD
bash tools/gpu_steps.sh \
  "300|seq|cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d $R/gpurun_out/pseq -o run -- python3 $R/bench.py --steps 2 --warmup 5 > $R/gpurun_out/pseq.log 2>&1 && python3 $R/tools/step_sequence.py $R/gpurun_out/pseq/run_results.db > $R/gpurun_out/step_seq.txt; rm -rf $R/gpurun_out/pseq; head -5 $R/gpurun_out/step_seq.txt" \
  "200|choices|DPFS_SHOW_GEMM=1 python3 bench.py --steps 5 --warmup 3" \
  "300|iso|python3 tools/gemm4_probe.py --rounds 4 --iters 10 --scheds 0 --no-blas --layouts nt nn --bias"
