#!/bin/bash
# Round-6 GPU check 3: fp32 fixes + split-K, CE bookkeeping, GEMM beside a collective stand-in,
# planner at TP 2/4/8, bench, stagger A/B, TP floors with emulated collectives, fp32 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|t_k|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'f32 or ce_finalize or emb_sort or beside_collective'" \
  "300|t_fp32|python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fp32_gpu.py" \
  "400|t_mem|python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_memory_tp_gpu.py tests/test_memory_gpu.py" \
  "200|bench|python -u bench.py" \
  "240|bench_fp32|python -u bench.py --fp32 --model reference --seq-len 1000 --steps 10 --warmup 3" \
  "400|ab_stagger|python -u tools/ab_attr.py --rounds 2 '' 'ext:attn_stagger(1)' 'ext:attn_stagger(2)' -- --steps 20" \
  "300|tpsim_noop|python -u tools/tp_sim.py --tp 2 --configs sp:1,sp:2 --steps 5" \
  "300|tpsim_emul|python -u tools/tp_sim.py --tp 2 --configs sp:1,sp:2 --steps 5 --emulate-comm 64"
