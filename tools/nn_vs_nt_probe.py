"""Data-gradient GEMMs dX = dY W (NN: W row-major [K, N], the B operand MN-major) against the same
product in the NT layout on a pre-transposed weight (W^T row-major [N, K], both operands
K-contiguous), GPT-2-small shapes, every tile-width variant, interleaved.  Answers whether
keeping a transposed bf16 weight shadow for the dgrads would pay.

    python tools/nn_vs_nt_probe.py [--rounds 5 --iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

# (name, M tokens, N = d_in of the weight, K = d_out): dX[M, N] = dY[M, K] W[K, N]
SHAPES = [("qkv", 32768, 768, 2304), ("wo", 32768, 768, 768), ("gateup", 32768, 768, 4096),
          ("down", 32768, 2048, 768), ("lmhead", 32768, 768, 50304)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", nargs="*", default=None)
    a = ap.parse_args()
    C = _ext.require()
    for name, M, N, K in SHAPES:
        if a.shapes and name not in a.shapes:
            continue
        dy = (torch.randn(M, K, device="cuda") / 4).bfloat16()
        w = (torch.randn(K, N, device="cuda") / 4).bfloat16()
        wt = w.t().contiguous()
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(10):
            w.t().contiguous()
        t1 = torch.cuda.Event(enable_timing=True)
        t1.record()
        torch.cuda.synchronize()
        ref = C.gemm_nn(dy, w)
        arms = {}
        for v in (0, 1, 2):
            arms[f"nn v{v}"] = (lambda v=v: C.gemm_nn(dy, w, variant=v))
            arms[f"nt v{v}"] = (lambda v=v: C.gemm_nt(dy, wt, variant=v))
        err = (C.gemm_nt(dy, wt).float() - ref.float()).abs().max().item()
        r = timeit(arms, iters=a.iters, rounds=a.rounds)
        fl = 2.0 * M * N * K
        best_nn = min(v for k, v in r.items() if k.startswith("nn"))
        best_nt = min(v for k, v in r.items() if k.startswith("nt"))
        print(f"{name} M{M} N{N} K{K}: max|nt - nn| {err:.3e}; transpose of W {t0.elapsed_time(t1) / 10:.4f} ms; "
              + "  ".join(f"{k} {v:.4f}" for k, v in r.items())
              + f"  -> best nn {best_nn:.4f} ({fl / best_nn / 1e9:.0f} TF)  best nt {best_nt:.4f} ({fl / best_nt / 1e9:.0f} TF)",
              flush=True)


if __name__ == "__main__":
    main()
