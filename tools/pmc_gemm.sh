#!/bin/bash
# PMC counters for the GEMM kernels (v2 vs v3) on one shape; run on the GPU box via gpurun.
# Usage: bash tools/pmc_gemm.sh [probe args...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ARGS=${*:-"--layout nt --M 32768 --N 4096 --K 768 --impl 2 --iters 5"}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters.txt 2>&1
SETS=${PMC_SETS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT;SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS"}
IFS=';' read -ra SETARR <<< "$SETS"
for set in "${SETARR[@]}"; do
  name=$(echo $set | cut -d' ' -f1)
  timeout -k 10 180 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$name -o run -- \
    python3 $R/tools/gemm_probe.py $ARGS > $R/gpurun_out/pmc/$name.log 2>&1
  rc=$?
  echo "pmc set $name rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
