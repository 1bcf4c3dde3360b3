"""Run one GEMM layout/shape repeatedly with a chosen implementation (for rocprofv3 PMC runs).

    python tools/gemm_probe.py --layout nt --M 32768 --N 4096 --K 768 --impl 2 --sched 0 2 4 --iters 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="nt", choices=["nt", "nn", "tn"])
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--impl", type=int, nargs="+", default=[2])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sched", type=int, nargs="+", default=[-1])
    ap.add_argument("--cfg", type=int, nargs="+", default=[-1])
    ap.add_argument("--blas", action="store_true", help="also time hipBLASLt (torch) on the same layout")
    ap.add_argument("--v4", type=int, default=None, help="kernel variant for impl 3 (0 v4, 1 / 2 v4 256 / 192 wide, 3 v3)")
    ap.add_argument("--sched4", type=int, default=None, help="v4 schedule (gemm4_sched)")
    ap.add_argument("--check", action="store_true", help="relative error of each implementation vs fp32 torch")
    a = ap.parse_args()
    C = _ext.require()
    var = a.v4 or 0
    if a.sched4 is not None:
        C.gemm4_sched(a.sched4)
    M, N, K = a.M, a.N, a.K
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    fn = {"nt": lambda: C.gemm_nt(x, w, None, variant=var), "nn": lambda: C.gemm_nn(dy, w, variant=var),
          "tn": lambda: C.gemm_tn(dy, x, variant=0 if var != 3 else 3)}[a.layout]
    ref = {"nt": lambda: x.float() @ w.float().t(), "nn": lambda: dy.float() @ w.float(),
           "tn": lambda: dy.float().t() @ x.float()}[a.layout]() if a.check else None
    for impl, sched, cfg in [(i, sc, cf) for i in a.impl for sc in (a.sched if i >= 2 else [0]) for cf in a.cfg]:
        C.gemm_set_impl(impl)
        C.gemm_v2_sched(sched)
        C.gemm_force(cfg, 0)
        if ref is not None:
            out = fn().float()
            err = ((out - ref).norm() / ref.norm()).item()
            print(f"impl {impl} sched {sched} cfg {cfg} {a.layout} {M}x{N}x{K}: rel err {err:.2e}", flush=True)
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.iters
        print(f"impl {impl} sched {sched} cfg {cfg} {a.layout} {M}x{N}x{K}: {ms:.4f} ms {2.0 * M * N * K / ms / 1e9:.1f} TF", flush=True)
    C.gemm_set_impl(3)
    C.gemm_v2_sched(-1)
    C.gemm_force(-1, 0)
    if a.blas:
        bfn = {"nt": lambda: torch.nn.functional.linear(x, w), "nn": lambda: torch.matmul(dy, w),
               "tn": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)}[a.layout]
        for _ in range(a.iters):
            bfn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            bfn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.iters
        print(f"hipBLASLt {a.layout} {M}x{N}x{K}: {ms:.4f} ms {2.0 * M * N * K / ms / 1e9:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
