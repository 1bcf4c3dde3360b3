#!/bin/bash
# Round-6 GPU check 8: is the TP-2 emulated-collective slowdown the CUs the collective holds, or
# the schedule's dependencies?  Same modelled durations with 1 / 8 / 32 stand-in workgroups.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "300|tpsim2_b1|python -u tools/tp_sim.py --tp 2 --configs sp:1,sp:2,sp:4 --steps 5 --emulate-comm 153 --comm-blocks 1" \
  "300|tpsim2_b8|python -u tools/tp_sim.py --tp 2 --configs sp:2,sp:4 --steps 5 --emulate-comm 153 --comm-blocks 8" \
  "300|tpsim2_b64|python -u tools/tp_sim.py --tp 2 --configs sp:2 --steps 5 --emulate-comm 153 --comm-blocks 64"
