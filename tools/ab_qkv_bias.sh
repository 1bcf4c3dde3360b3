#!/bin/bash
# A/B of the fused QKV bias gradient on one box: timed-step kernel summaries only (the rocpd
# databases are deleted on the box).
R=${GRAFT_REPO_ROOT}
cd /tmp && export TMPDIR=/tmp
for tag in on off on2; do
  [ "$tag" = off ] && export DPFS_QKV_BIAS_IN_ATTN=0 || export DPFS_QKV_BIAS_IN_ATTN=1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p_$tag -o run -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/p_$tag.log 2>&1 || exit $?
  python3 $R/tools/prof_summary.py $R/gpurun_out/p_$tag/run_results.db --after adam_k --skip 5 --steps 10 --top 60 > $R/gpurun_out/sum_$tag.txt 2>&1
  rm -rf $R/gpurun_out/p_$tag
done
