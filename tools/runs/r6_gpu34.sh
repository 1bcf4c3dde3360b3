#!/bin/bash
# Round-6 GPU check 34: end-of-round full-depth model runs on one GPU (GPT-2 large, LLaMA-2-7B
# shape, 13B shape at seq 8192 with planner-chosen recompute) and the TP 2 / 4 / 8 per-rank
# compute floors (tools/tp_sim.py, SP, one and two chunks) after the attention bias-partials fix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "400|m_large|python3 -u bench.py --model gpt2-large --batch-per-gpu 16 --steps 4 --warmup 2" \
  "400|m_7b|python3 -u bench.py --model llama2-7b --seq-len 4096 --batch-per-gpu 2 --steps 3 --warmup 2" \
  "500|m_13b|python3 -u bench.py --model llama-13b --seq-len 8192 --batch-per-gpu 1 --steps 3 --warmup 2" \
  "300|tp2|python3 -u tools/tp_sim.py --tp 2 --configs sp:1,sp:2 --steps 5" \
  "300|tp4|python3 -u tools/tp_sim.py --tp 4 --configs sp:1,sp:2 --steps 5" \
  "300|tp8|python3 -u tools/tp_sim.py --tp 8 --configs sp:1,sp:2 --steps 5"
