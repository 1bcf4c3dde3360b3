#!/bin/bash
# Round-6 GPU check 47: TN GEMMs alone with the 32x32x16 loop's barrier-row hook 0 / 1 / 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh "300|tnbr|python3 tools/tn_br_probe.py"
