"""Time hipBLASLt algorithms through our binding (ops lt_run) in-process, for one GEMM shape.

    python tools/lt_probe.py --layout 2 --M 2304 --N 768 --K 32768 [--accumulate] [--algos 0 5 13]

Prints per-algorithm ms (event-timed, back-to-back reps) next to our kernel and torch's path,
to separate kernel time from binding overhead (run under rocprofv3 --kernel-trace --stats to
see the kernels themselves).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402


def ms(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", type=int, default=2)
    ap.add_argument("--M", type=int, default=2304)
    ap.add_argument("--N", type=int, default=768)
    ap.add_argument("--K", type=int, default=32768)
    ap.add_argument("--accumulate", action="store_true")
    ap.add_argument("--algos", type=int, nargs="*", default=None)
    a = ap.parse_args()
    C = _ext.require()
    M, N, K, L = a.M, a.N, a.K, a.layout
    dev = "cuda"
    if L == 0:
        x, w = torch.randn(M, K, device=dev).bfloat16(), torch.randn(N, K, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ours = lambda: C.gemm_nt(x, w, None, out=out)  # noqa: E731
        blas = lambda: torch.mm(x, w.t(), out=out)  # noqa: E731
    elif L == 1:
        x, w = torch.randn(M, K, device=dev).bfloat16(), torch.randn(K, N, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ours = lambda: C.gemm_nn(x, w, out=out)  # noqa: E731
        blas = lambda: torch.matmul(x, w, out=out)  # noqa: E731
    else:
        x, w = torch.randn(K, M, device=dev).bfloat16(), torch.randn(K, N, device=dev).bfloat16()
        out = torch.zeros(M, N, device=dev, dtype=torch.float32)
        ours = lambda: C.gemm_tn(x, w, out, a.accumulate)  # noqa: E731
        blas = lambda: torch.mm(x.t(), w, out_dtype=torch.float32, out=out)  # noqa: E731
    n = C.lt_algos(L, M, N, K, False)
    print(f"layout {L} {M}x{N}x{K} accumulate={a.accumulate}: {n} algorithms", flush=True)
    print(f"  ours  {ms(ours):.4f} ms", flush=True)
    print(f"  torch {ms(blas):.4f} ms", flush=True)
    for i in (a.algos if a.algos is not None else range(n)):
        t = ms(lambda: C.lt_run(L, x, w, out, None, i, a.accumulate))
        print(f"  lt{i:<3d} {t:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
