"""Is an fp8 GEMM path available on this torch / ROCm build for gfx950, and what does it buy?

Times torch._scaled_mm (hipBLASLt fp8, OCP e4m3fn / e5m2 operands, per-tensor scales, bf16
output) against the bf16 GEMM on the GPT-2-small projection shapes, and checks its error
against an fp32 product of the same quantised operands.

    python tools/fp8_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import timeit  # noqa: E402


def q(t, dtype):
    amax = t.abs().amax().float().clamp(min=1e-12)
    scale = torch.finfo(dtype).max / amax
    return (t.float() * scale).to(dtype), (1.0 / scale).reshape(())


def main():
    dev = "cuda"
    print("torch", torch.__version__, "fp8 types:", torch.float8_e4m3fn, torch.float8_e5m2, flush=True)
    shapes = [(32768, 2304, 768), (32768, 768, 768), (32768, 4096, 768), (32768, 768, 2048),
              (32768, 50304, 768), (32768, 768, 4096)]
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        try:
            a8, sa = q(a, torch.float8_e4m3fn)
            w8, sw = q(w, torch.float8_e4m3fn)
            y8 = torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sw, out_dtype=torch.bfloat16)
        except Exception as e:   # not supported on this build
            print(f"{M}x{N}x{K}: _scaled_mm failed: {type(e).__name__}: {e}", flush=True)
            return
        ref = (a8.float() * sa) @ (w8.float() * sw).t()
        err = ((y8.float() - ref).norm() / ref.norm()).item()
        fns = {"bf16": lambda: a @ w.t(),
               "fp8": lambda: torch._scaled_mm(a8, w8.t(), scale_a=sa, scale_b=sw, out_dtype=torch.bfloat16)}
        t = timeit(fns, iters=10)
        fl = 2 * M * N * K
        print(f"{M}x{N}x{K}: bf16 {t['bf16'] * 1e3:.1f} us ({fl / t['bf16'] / 1e9:.0f} TF), fp8 {t['fp8'] * 1e3:.1f} us "
              f"({fl / t['fp8'] / 1e9:.0f} TF), rel err vs fp32 of the quantised operands {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
