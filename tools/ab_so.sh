#!/bin/bash
# Same-box interleaved A/B of two builds of the extension:
#   tools/ab_so.sh "new old new old" <command...>
# abold/<label>_C.so is copied over the in-tree _C*.so before each run of <command> (its own
# process, under a time limit, with AB_LABEL=<label> in its environment); the first label's
# build is put back at the end.  Stops at the first run that does not exit 0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
labels=$1; shift
so=$(ls distributed_pytorch_from_scratch_amd/_C.cpython-*.so)
first=${labels%% *}
mkdir -p gpurun_out
for lab in $labels; do
  cp "abold/${lab}_C.so" "$so" || exit 3
  echo "--- [$lab] $*"
  AB_LABEL=$lab timeout -k 10 300 "$@" || { rc=$?; cp "abold/${first}_C.so" "$so"; echo "run [$lab] rc=$rc"; exit $rc; }
done
cp "abold/${first}_C.so" "$so"
