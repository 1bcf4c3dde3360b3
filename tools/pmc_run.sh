#!/bin/bash
# Collect PMC counter sets (semicolon-separated in PMC_SETS) for one probe command.
# Usage: PMC_SETS="A B C;D E" bash tools/pmc_run.sh <outdir-name> python3 tools/xxx_probe.py args...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NAME=$1; shift
PROG=$1; shift
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$NAME
IFS=';' read -ra SETARR <<< "$PMC_SETS"
for set in "${SETARR[@]}"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 180 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/$NAME/$tag -o run -- \
    $PROG "$@" > $R/gpurun_out/$NAME/$tag.log 2>&1
  rc=$?
  echo "pmc set $tag rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
