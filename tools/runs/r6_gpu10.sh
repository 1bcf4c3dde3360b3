#!/bin/bash
# Round-6 GPU check 10: backward with K pre-scaled (impl 4 now; 9 = the old form): tests, per-call
# A/B, headline A/B; forward impl 8 combined.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|t_ksc|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'attention'" \
  "240|probe_ksc|python -u tools/attn_probe.py --bwd --impl 9 4 9 4 --iters 20 && python -u tools/attn_probe.py --bwd --impl 9 4 9 4 --iters 10 --hd 128 --H 32 --T 4096 --B 2" \
  "500|ab_ksc|bash tools/ab_env.sh DPFS_ATTN_IMPL '0,9 0,4 8,4 0,9 0,4 8,4'"
