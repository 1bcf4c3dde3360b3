#!/bin/bash
# Round-6 GPU check 2: fp32 native kernels + training, CE bookkeeping, embedding sort, bench,
# step traces (bf16 headline and fp32 reference preset).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "400|t_new|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'f32 or ce_finalize or emb_sort or fused6 or stream_k'" \
  "400|t_fp32|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp32_gpu.py" \
  "300|bench|python -u bench.py" \
  "300|bench_fp32_ours|python -u bench.py --fp32 --model reference --seq-len 1000 --steps 10 --warmup 3" \
  "300|bench_fp32_ref|python -u bench.py --fp32 --model reference --seq-len 1000 --impl reference --steps 10 --warmup 3" \
  "300|prof_bf16|bash tools/prof_step.sh r6bf16" \
  "300|prof_fp32|BENCH_ARGS='--fp32 --model reference --seq-len 1000' bash tools/prof_step.sh r6fp32"
