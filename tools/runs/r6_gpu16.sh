#!/bin/bash
# Round-6 GPU check 16: stray kernel call sites; TP-2 collective/compute overlap under emulated collectives.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "200|stray16c|python -u tools/find_stray_kernels.py" \
  "200|stray32c|python -u tools/find_stray_kernels.py --fp32" \
  "300|ovl2c2|bash tools/prof_tpsim_emul.sh tp2c2 2 sp:2 153" \
  "300|ovl2c1|bash tools/prof_tpsim_emul.sh tp2c1 2 sp:1 153"
