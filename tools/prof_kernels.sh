#!/bin/bash
# Per-kernel times of one command: rocprofv3 --kernel-trace --stats, summary into gpurun_out/<name>.
# Usage: bash tools/prof_kernels.sh <name> python3 tools/xxx.py args...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NAME=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$NAME -o run -- "$@" > $R/gpurun_out/$NAME.log 2>&1
rc=$?
f=$(find $R/gpurun_out/$NAME -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:25]:
    print('%10.1f us avg %6s calls  %s'%(float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:110]))
" > $R/gpurun_out/$NAME.txt
exit $rc
