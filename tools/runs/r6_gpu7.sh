#!/bin/bash
# Round-6 GPU check 7: HIP-graph train step (bitwise test + bench A/B); TP 2 / 8 chunk counts
# under emulated collectives (1 / 2 / 4 chunks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "240|t_graph|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py -k graph_train_step" \
  "400|ab_graph|bash tools/ab_env.sh DPFS_GRAPH 'off on off on'" \
  "400|tpsim2_c4|python -u tools/tp_sim.py --tp 2 --configs sp:1,sp:2,sp:4 --steps 5 --emulate-comm 153" \
  "400|tpsim2_noemu|python -u tools/tp_sim.py --tp 2 --configs sp:1,sp:2,sp:4 --steps 5" \
  "400|tpsim8_c4|python -u tools/tp_sim.py --tp 8 --configs sp:1,sp:2,sp:4 --steps 5 --emulate-comm 153"
