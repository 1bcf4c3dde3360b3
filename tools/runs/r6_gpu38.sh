#!/bin/bash
# Round-6 GPU check 38: attention backward tile tails reordered -- the second query tile's /
# key half's exps under the first one's dV^T / dQ^T MFMAs, its dS under the last ones (same
# accumulation order per accumulator: bitwise vs the previous build), tests, kernel + step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "150|dump|bash tools/ab_so.sh 'new old' python3 tools/attn_bwd_dump.py && bash tools/ab_so.sh 'new old' python3 tools/attn_bwd_dump.py --hd 128 && python3 tools/attn_bwd_dump.py --compare new old && python3 tools/attn_bwd_dump.py --compare new old --hd 128; rm -f gpurun_out/attn_bwd_*.pt" \
  "300|attn_tests|python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attention and not decode'" \
  "300|ctx|bash tools/ab_so.sh 'new old new old' python3 tools/attn_ctx_probe.py --impls 4 --n 30" \
  "600|bench|bash tools/ab_so.sh 'new old new old new old' python3 bench.py"
