#!/bin/bash
# Round-6 GPU check 22: fp32 GEMM with 32-deep K stages; fp32 model tests; fp32 bench + trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|t_f32b|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'attention_f32 or gemm_f32 or gemm_unaligned'" \
  "300|t_f32m|python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_fp32_gpu.py" \
  "240|bench_fp32c|python -u bench.py --fp32 --model reference --seq-len 1000 --steps 10 --warmup 3" \
  "300|prof_fp32d|BENCH_ARGS='--fp32 --model reference --seq-len 1000' bash tools/prof_step.sh r6fp32d"
