#!/bin/bash
# Round-6 GPU check 31: PMC of the training step's kernels after the attention bias-partials fix
# (MFMA busy, instruction mix per MFMA), bench.py with 2 timed steps after 2 warmup steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
SETA="A SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh \
  "300|pmc_step|PMC_SETS='$SETA' bash tools/pmc_run.sh pmc_step python3 $PWD/bench.py --steps 2 --warmup 2 && python3 tools/pmc_summary.py gpurun_out/pmc_step > gpurun_out/pmcsum_step.txt"
cp gpurun_out/pmc_step/A.log gpurun_out/pmc_step_A.log 2>/dev/null; rm -rf gpurun_out/pmc_step
