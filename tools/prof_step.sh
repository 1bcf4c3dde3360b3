#!/bin/bash
# Timed-step kernel summary of bench.py (GPT-2 small TP 1) on the GPU box: rocprofv3 kernel trace,
# tools/prof_summary.py over the 10 timed steps, database deleted on the box (gpurun_out stays small).
R=${GRAFT_REPO_ROOT}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_head -o run -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/p_head.log 2>&1 || exit $?
python3 $R/tools/prof_summary.py $R/gpurun_out/p_head/run_results.db --after adam_k --skip 5 --steps 10 --top 45 > $R/gpurun_out/sum_head.txt 2>&1
rm -rf $R/gpurun_out/p_head
