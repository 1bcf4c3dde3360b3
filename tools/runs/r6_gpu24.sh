#!/bin/bash
# Round-6 GPU check 24: attention backward with the cross-block prefetch branch moved after the
# exps (the exps of the first query / key half interleave with the second half's MFMAs again):
# bitwise vs the previous build, attention GPU tests, kernel and step A/B (same box, interleaved).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "150|dump|bash tools/ab_so.sh 'new old' python3 tools/attn_bwd_dump.py && bash tools/ab_so.sh 'new old' python3 tools/attn_bwd_dump.py --hd 128 && python3 tools/attn_bwd_dump.py --compare new old && python3 tools/attn_bwd_dump.py --compare new old --hd 128" \
  "300|attn_tests|python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k 'attention and not f32 and not decode'" \
  "400|probe|bash tools/ab_so.sh 'new old new old' python3 tools/attn_probe.py --bwd --impl 4 --iters 20" \
  "500|bench|bash tools/ab_so.sh 'new old new old' python3 bench.py"
