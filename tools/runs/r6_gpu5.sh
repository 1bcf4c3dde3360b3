#!/bin/bash
# Round-6 GPU check 5: any-alignment bf16 GEMMs (kernel + uneven-vocab TP step with torch GEMMs
# poisoned), then the full-size N=8 driver protocol rehearsed on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "240|t_gemm|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'gemm_f32 or gemm_unaligned'" \
  "300|t_uneven|python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_fp32_gpu.py" \
  "600|rehearsal8|bash tools/rehearsal_full.sh 8"
