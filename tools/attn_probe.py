"""Run the attention kernels repeatedly with chosen implementations (for rocprofv3 PMC runs).

    python tools/attn_probe.py --B 32 --T 1024 --H 12 --hd 64 --impl 1 2 --iters 10 [--bwd]
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--hd", type=int, default=64)
    ap.add_argument("--impl", type=int, nargs="+", default=[2])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bwd", action="store_true")
    a = ap.parse_args()
    C = _ext.require()
    B, T, H, hd = a.B, a.T, a.H, a.hd
    qkv = torch.randn(B * T, 3 * H * hd, device="cuda").bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    scale = 1 / math.sqrt(hd)
    o, lse = C.attn_fwd(q, k, v, scale, True)
    do = torch.randn_like(o)
    d = torch.empty_like(qkv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    fl = 4.0 * B * H * T * T * hd / 2 * (2.5 if a.bwd else 1.0)
    from tools.bench_kernels import timeit

    def mk(impl):
        def g():
            C.attn_set_impl(impl)
            C.attn_set_bwd_impl(impl if a.bwd else 2)
            if a.bwd:
                C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv)
            else:
                C.attn_fwd(q, k, v, scale, True)
        return g
    if not a.bwd:   # forward outputs of every implementation against impl 1
        C.attn_set_impl(1)
        o1, l1 = C.attn_fwd(q, k, v, scale, True)
        for impl in a.impl:
            C.attn_set_impl(impl)
            oi, li = C.attn_fwd(q, k, v, scale, True)
            print(f"impl {impl} vs 1: max|dO| {(oi.float() - o1.float()).abs().max().item():.3e} "
                  f"max|dLSE| {(li - l1).abs().max().item():.3e}", flush=True)
    res = timeit({impl: mk(impl) for impl in a.impl}, iters=a.iters, rounds=5)  # interleaved, median
    for impl, ms in res.items():
        print(f"impl {impl} {'bwd' if a.bwd else 'fwd'}: {ms:.4f} ms {fl / ms / 1e9:.1f} TF", flush=True)
    C.attn_set_impl(1)
    C.attn_set_bwd_impl(2)


if __name__ == "__main__":
    main()
