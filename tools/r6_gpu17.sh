#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r6_final.sh
