"""TN (weight-gradient) GEMMs of the GPT-2-small step, c[M, N] = a[K, M]^T b[K, N] with K = 32768
tokens, timed with the 32x32x16 main loop's barrier-row hook at 0 / 1 / 2 (interleaved, median).

    python tools/tn_br_probe.py [--rounds 7 --iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402

SHAPES = [("qkv", 2304, 768), ("wo", 768, 768), ("gateup", 4096, 768), ("down", 768, 2048), ("lmhead", 50304, 768)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    C = _ext.require()
    K = 32768
    for name, M, N in SHAPES:
        x = (torch.randn(K, M, device="cuda") / 4).bfloat16()
        y = (torch.randn(K, N, device="cuda") / 4).bfloat16()

        def mk(br):
            def f():
                C.gemm4_br_tn(br)
                return C.gemm_tn(x, y)
            return f
        r = timeit({br: mk(br) for br in (0, 1, 2)}, iters=a.iters, rounds=a.rounds)
        C.gemm4_br_tn(0)
        print(f"tn {name} {M}x{N}x{K}: " + "  ".join(f"br{k} {v:.4f} ms" for k, v in r.items()), flush=True)


if __name__ == "__main__":
    main()
