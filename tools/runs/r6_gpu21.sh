#!/bin/bash
# Round-6 GPU check 21: fp32 attention with the next tile's loads in flight under the MFMAs and
# exp2: tests, fp32 bench vs the reference's eager fp32 on the same box, step trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|t_f32|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'attention_f32 or gemm_f32' tests/test_fp32_gpu.py" \
  "240|bench_fp32b|python -u bench.py --fp32 --model reference --seq-len 1000 --steps 10 --warmup 3" \
  "240|bench_fp32_refb|python -u bench.py --fp32 --model reference --seq-len 1000 --impl reference --steps 10 --warmup 3" \
  "300|prof_fp32c|BENCH_ARGS='--fp32 --model reference --seq-len 1000' bash tools/prof_step.sh r6fp32c"
