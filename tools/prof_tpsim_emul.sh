#!/bin/bash
# Collective / compute overlap of tools/tp_sim.py --emulate-comm (one config) under rocprofv3:
#   tools/prof_tpsim_emul.sh TAG TP CONFIG GBPS -> gpurun_out/ovl_TAG.txt
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag=$1; tp=$2; cfg=$3; gbps=$4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $R/gpurun_out/pe_$tag -o run -- python3 $R/tools/tp_sim.py --tp $tp --configs $cfg --steps 5 --emulate-comm $gbps > $R/gpurun_out/pe_$tag.log 2>&1 || exit $?
python3 $R/tools/comm_overlap.py $R/gpurun_out/pe_$tag/run_results.db --skip 3 --steps 3 > $R/gpurun_out/ovl_$tag.txt 2>&1
rm -rf $R/gpurun_out/pe_$tag
cat $R/gpurun_out/ovl_$tag.txt
