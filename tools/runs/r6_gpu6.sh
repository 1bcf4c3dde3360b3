#!/bin/bash
# Round-6 GPU check 6: the 64-keys-per-wave dK/dV kernel (impl 7): bitwise vs impl 4, per-call
# A/B at the GPT-2 small and LLaMA-like shapes, kernel trace; the headline step with gap analysis.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "240|t_dkdv4|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'dkdv4 or (test_attention and 4) or gemm_unaligned or gemm_f32'" \
  "240|probe_dkdv4|python -u tools/attn_probe.py --bwd --impl 4 7 4 7 --iters 20" \
  "300|prof_dkdv4|cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d \$GRAFT_REPO_ROOT/gpurun_out/pk4 -o run -- python3 \$GRAFT_REPO_ROOT/tools/attn_probe.py --bwd --impl 7 --iters 10 && python3 \$GRAFT_REPO_ROOT/tools/prof_summary.py \$GRAFT_REPO_ROOT/gpurun_out/pk4/run_results.db --top 8 > \$GRAFT_REPO_ROOT/gpurun_out/sum_dkdv4.txt; rm -rf \$GRAFT_REPO_ROOT/gpurun_out/pk4" \
  "400|ab_bwd7|bash tools/ab_env.sh DPFS_ATTN_IMPL '0,4 0,7 0,4 0,7'" \
  "300|prof_gap|bash tools/prof_step.sh r6gap"
