#!/bin/bash
# Timed-step kernel summary of the headline bench under rocprofv3 (kernel trace only):
#   tools/prof_step.sh TAG [VAR=value ...]   -> gpurun_out/sum_TAG.txt (+ p_TAG.log)
# (BENCH_ARGS="--fp32 --model reference ...": extra bench.py arguments)
# The rocpd database is deleted on the box; only the summary comes back.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_$tag -o run -- python3 $R/bench.py --steps 10 --warmup 5 ${BENCH_ARGS:-} > $R/gpurun_out/p_$tag.log 2>&1 || exit $?
python3 $R/tools/prof_summary.py $R/gpurun_out/p_$tag/run_results.db --after adam_k --skip 5 --steps 10 --top 60 \
    ${DPFS_PROF_SEQ:+--sequence "$DPFS_PROF_SEQ"} > $R/gpurun_out/sum_$tag.txt 2>&1
python3 $R/tools/gap_analysis.py $R/gpurun_out/p_$tag/run_results.db --last-ms 150 --top 12 >> $R/gpurun_out/sum_$tag.txt 2>&1
rm -rf $R/gpurun_out/p_$tag
head -30 $R/gpurun_out/sum_$tag.txt
