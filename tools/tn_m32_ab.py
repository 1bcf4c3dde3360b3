"""A/B of the TN (weight-gradient) main loop: 32x32x16 (gemm4_k M32) vs 16x16x32, GPT-2-small
step shapes, interleaved, ms per call (HIP events, 20 reps after warmup)."""
import torch
from distributed_pytorch_from_scratch_amd.ops import _ext

C = _ext.require()
import sys
SHAPES = [("qkv", 2304, 768, 32768), ("wo", 768, 768, 32768), ("gateup", 4096, 768, 32768),
          ("down", 768, 2048, 32768), ("lmhead", 50304, 768, 32768)]
if "--llama7b" in sys.argv:   # LLaMA-2-7B shape, seq 4096 x batch 2 = 8192 tokens
    SHAPES = [("qkv", 12288, 4096, 8192), ("wo", 4096, 4096, 8192), ("gateup", 22016, 4096, 8192),
              ("down", 4096, 11008, 8192), ("lmhead", 32000, 4096, 8192)]


def t(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


tot = {0: 0.0, 1: 0.0}
for name, M, N, K in SHAPES:
    a = torch.randn(K, M, device="cuda").bfloat16()
    b = torch.randn(K, N, device="cuda").bfloat16()
    out = torch.empty(M, N, device="cuda")
    res = {0: [], 1: []}
    for rep in range(3):
        for v in (1, 0):
            C.gemm4_m32(v)
            res[v].append(t(lambda: C.gemm_tn(a, b, out, False)))
    C.gemm4_m32(1)
    r0, r1 = min(res[0]), min(res[1])
    tot[0] += r0
    tot[1] += r1
    fl = 2.0 * M * N * K
    print(f"{name:7s} {M}x{N}x{K}  16x16x32 {r0:.4f} ms ({fl / r0 / 1e9:.0f} TF)   32x32x16 {r1:.4f} ms "
          f"({fl / r1 / 1e9:.0f} TF)   {r0 / r1:.3f}x", flush=True)
print(f"sum: 16x16x32 {tot[0]:.4f} ms, 32x32x16 {tot[1]:.4f} ms")
