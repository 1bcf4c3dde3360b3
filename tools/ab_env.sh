#!/bin/bash
# Same-box interleaved A/B of one environment switch on the headline bench:
#   tools/ab_env.sh VAR "v1 v2 v1 v2" [bench args...]
# Each run is its own process under a time limit; prints one line per run (value, ms/step).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
var=$1; vals=$2; shift 2
mkdir -p gpurun_out
for v in $vals; do
  out=$(env "$var=$v" timeout -k 10 200 python bench.py "$@" 2>gpurun_out/ab_err.log | grep '^{') || { echo "run $var=$v failed"; tail -5 gpurun_out/ab_err.log; exit 1; }
  python - "$var=$v" "$out" <<'PY'
import json, sys
d = json.loads(sys.argv[2])
print(f"{sys.argv[1]:>32}  {d['ms_per_step']:8.3f} ms/step  {d['value']:>12,.0f} tok/s  loss {d.get('final_loss')}")
PY
done
