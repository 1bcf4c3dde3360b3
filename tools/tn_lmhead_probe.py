import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from distributed_pytorch_from_scratch_amd.ops import _ext
C = _ext.require()
M = 32768
dy = torch.randn(M, 50304, device="cuda").bfloat16()
x = torch.randn(M, 768, device="cuda").bfloat16()
out = torch.empty(50304, 768, device="cuda")
def t(fn, it=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it
print("plan splits", C.gemm_tn_splits(50304, 768, M) if hasattr(C, "gemm_tn_splits") else "?")
for cfg in (0, 1):
    for S in (1, 2, 3, 4, 5, 6):
        C.gemm_force(cfg, S)
        print(f"cfg {cfg} S {S}: {t(lambda: C.gemm_tn(dy, x)):.4f} ms", flush=True)
C.gemm_force(-1, 0)
print(f"auto: {t(lambda: C.gemm_tn(dy, x)):.4f} ms")
