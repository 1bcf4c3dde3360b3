#!/bin/bash
# Round-6 GPU check 4: forward row-sum-by-MFMA A/B, fp32 (ours vs the reference's eager fp32) on one
# box + its step trace, TP-2 emulated collectives at 153 GB/s, one- vs two-chunk kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "200|t_att6|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'test_attention and 6'" \
  "400|ab_fwd6|bash tools/ab_env.sh DPFS_ATTN_IMPL '0 6,0 0 6,0'" \
  "200|bench_fp32|python -u bench.py --fp32 --model reference --seq-len 1000 --steps 10 --warmup 3" \
  "200|bench_fp32_ref|python -u bench.py --fp32 --model reference --seq-len 1000 --impl reference --steps 10 --warmup 3" \
  "300|prof_fp32|BENCH_ARGS='--fp32 --model reference --seq-len 1000' bash tools/prof_step.sh r6fp32b" \
  "300|tpsim_emul153|python -u tools/tp_sim.py --tp 2 --configs sp:1,sp:2 --steps 5 --emulate-comm 153" \
  "300|tpsim_emul8|python -u tools/tp_sim.py --tp 8 --configs sp:1,sp:2 --steps 5 --emulate-comm 153" \
  "300|prof_c1|bash tools/prof_tpsim.sh tp2c1 2 sp:1" \
  "300|prof_c2|bash tools/prof_tpsim.sh tp2c2 2 sp:2"
