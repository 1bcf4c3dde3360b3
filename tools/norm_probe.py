import sys, os, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from distributed_pytorch_from_scratch_amd.ops import _ext
from tools.bench_kernels import timeit
C=_ext.require()
M,D=32768,768
y=torch.randn(M,D,device="cuda").bfloat16(); r=torch.randn(M,D,device="cuda").bfloat16(); b=torch.randn(D,device="cuda"); w=torch.rand(D,device="cuda")
def unf():
    x=C.bias_residual(y,b,r); C.rmsnorm_fwd(x,w,1e-5)
def fus():
    C.add_rmsnorm_fwd(y,b,r,w,1e-5)
t=timeit({"unfused":unf,"fused":fus},iters=50)
print({k: round(v*1000,1) for k,v in t.items()}, "us")
