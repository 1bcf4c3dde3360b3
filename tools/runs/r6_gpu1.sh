#!/bin/bash
# Round-6 GPU check 1: fused attention backward numerics + timing, stream-K error word, bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|t_fused|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'fused6 or stream_k'" \
  "150|probe|python -u tools/attn_probe.py --bwd --impl 4 6 --iters 20" \
  "200|prof_attn|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o attn -- python3 tools/attn_probe.py --bwd --impl 6 --iters 10" \
  "300|bench4|python -u bench.py" \
  "300|bench6|DPFS_ATTN_IMPL=0,6 python -u bench.py"
