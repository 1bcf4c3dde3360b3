#!/bin/bash
# PMC counter passes (one rocprofv3 run per set) of the attention kernels via tools/attn_probe.py.
# Usage: bash tools/pmc_attn_fwd.sh <outdir> [attn_probe args...]   (e.g. --impl 4 --iters 5 [--bwd])
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$1; shift
PMC_SETS="A SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE;B SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA;C SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC" \
  bash $R/tools/pmc_run.sh $OUT python3 $R/tools/attn_probe.py "$@"
