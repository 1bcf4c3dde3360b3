#!/bin/bash
# Kernel summary of tools/tp_sim.py (one config) under rocprofv3 (kernel trace only):
#   tools/prof_tpsim.sh TAG TP CONFIG  -> gpurun_out/sum_TAG.txt  (timed steps: after the 2nd Adam)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag=$1; tp=$2; cfg=$3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_$tag -o run -- python3 $R/tools/tp_sim.py --tp $tp --configs $cfg --steps 5 > $R/gpurun_out/p_$tag.log 2>&1 || exit $?
python3 $R/tools/prof_summary.py $R/gpurun_out/p_$tag/run_results.db --after adam_k --skip 2 --steps 6 --top 60 > $R/gpurun_out/sum_$tag.txt 2>&1
rm -rf $R/gpurun_out/p_$tag
head -25 $R/gpurun_out/sum_$tag.txt
