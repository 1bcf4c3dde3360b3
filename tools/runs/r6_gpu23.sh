#!/bin/bash
# Round-6 GPU check 23: end-of-round PMC of the attention kernels (GPT-2 small layer shape, impl 4
# forward / backward) -- MFMA busy and instruction mix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
SETA="A SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh \
  "200|pmc_af|PMC_SETS='$SETA' bash tools/pmc_run.sh pmc_af python3 tools/attn_probe.py --impl 4 --iters 5 && python3 tools/pmc_summary.py gpurun_out/pmc_af > gpurun_out/pmcsum_af.txt" \
  "200|pmc_ab|PMC_SETS='$SETA' bash tools/pmc_run.sh pmc_ab python3 tools/attn_probe.py --impl 4 --iters 5 --bwd && python3 tools/pmc_summary.py gpurun_out/pmc_ab > gpurun_out/pmcsum_ab.txt"
rm -rf gpurun_out/pmc_af gpurun_out/pmc_ab
