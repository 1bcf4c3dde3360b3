#!/bin/bash
# Round-6 GPU check 45: the rebuilt bounds-assert extension (_C_kassert, current sources): its
# training-step + decode test, plus smoke() on the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "400|kassert|python3 -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -k kernel_assert" \
  "200|smoke|python3 -u -c 'import __graft_entry__ as g; g.smoke()'"
