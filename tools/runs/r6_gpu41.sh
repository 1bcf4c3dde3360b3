#!/bin/bash
# Round-6 GPU check 41: barrier row 2 as the GEMM default -- bitwise vs BR 0 on the step's NN / NT
# shapes, the GEMM + model GPU tests, and the step A/B against BR 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_steps.sh \
  "200|bitwise|python3 -c \"
import torch
from distributed_pytorch_from_scratch_amd.ops import _ext
C = _ext.require()
torch.manual_seed(0)
for (M, N, K) in [(32768, 768, 2304), (32768, 768, 4096), (32768, 2048, 768), (32768, 2304, 768), (4096, 1000, 512)]:
    a = torch.randn(M, K, device='cuda').bfloat16(); b = torch.randn(K, N, device='cuda').bfloat16(); bt = b.t().contiguous()
    outs = {}
    for br in (0, 2):
        C.gemm4_br(br)
        outs[br] = (C.gemm_nn(a, b), C.gemm_nt(a, bt), C.gemm_nn(a, b, variant=2), C.gemm_nt(a, bt, variant=1))
    print(M, N, K, 'bitwise BR2 == BR0:', all(torch.equal(x, y) for x, y in zip(outs[0], outs[2])), flush=True)
C.gemm4_br(2)
\"" \
  "500|tests|python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k 'gemm or model or train or bitwise or reproducib'" \
  "900|ab|python3 tools/ab_attr.py --rounds 4 '' 'ext:gemm4_br(0)' -- --steps 20"
