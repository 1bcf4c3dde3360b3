#!/bin/bash
# The driver's 8-GPU bench protocol at FULL size (GPT-2 small, 12 layers, seq 1024, 32 seq per
# GPU, 20 timed + 5 warmup steps), rehearsed with all 8 ranks on ONE MI355X: gloo bootstrap, the
# `auto` TP transport decision on the xGMI kernels (built, validated, timed per size class), the
# DP knee, the engine trial, the tp2dp4 headline and the extra pure tp8 layout.  Prints the one
# JSON line plus the wall time of the whole protocol (< 400 s).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-8}
export MASTER_ADDR=127.0.0.1 DPFS_BACKEND=gloo DPFS_TP_COMM=auto DPFS_TP_COMM_AUTO_ANY_BACKEND=1 \
       HSA_ENABLE_IPC_MODE_LEGACY=0
t0=$(date +%s)
timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$N --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus $N > gpurun_out/rehearsal_full_n$N.log 2>&1
rc=$?
t1=$(date +%s)
grep '^{' gpurun_out/rehearsal_full_n$N.log | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); d['rehearsal_wall_s'] = $t1 - $t0; print(json.dumps(d))
" > gpurun_out/rehearsal_full_n$N.jsonl
echo "rc=$rc wall=$((t1 - t0)) s"
tail -3 gpurun_out/rehearsal_full_n$N.log
exit $rc
