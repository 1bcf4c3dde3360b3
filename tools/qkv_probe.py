import torch, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from distributed_pytorch_from_scratch_amd.ops import _ext
from tools.bench_kernels import timeit
C = _ext.require()
M, N, K = 32768, 2304, 768
x = torch.randn(M, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
b = torch.randn(N, device="cuda")
pos = torch.arange(1024, device="cuda").repeat(32)
tab = torch.randn(1024, 64, device="cuda")
res = timeit({"plain": lambda: C.gemm_nt(x, w, b), "rope": lambda: C.gemm_nt(x, w, b, pos, tab, 24, 64),
              "blas": lambda: torch.nn.functional.linear(x, w, b.bfloat16())}, iters=20, rounds=5)
for k, v in res.items():
    print(k, round(v, 4), "ms", round(2 * M * N * K / v / 1e9, 1), "TF")
