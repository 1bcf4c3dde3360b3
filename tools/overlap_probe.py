"""Does running a layer's weight-gradient GEMMs on a second stream, concurrently with the
input-gradient GEMMs / attention backward of the main stream, beat running them in sequence?

    python tools/overlap_probe.py [--tokens 32768]

GPT-2-small layer shapes at batch 32 x 1024 (TP 1): per backward segment the main-stream op
(dgrad NN GEMM or attention backward) and the independent wgrad TN GEMM; prints serial vs
two-stream time for each pair and for the whole layer sequence.
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext, gemm_select as GS  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    a = ap.parse_args()
    k = _ext.require()
    M, d, F, H, hd, T = a.tokens, 768, 2048, 12, 64, 1024
    B = M // T
    r = lambda *s: torch.randn(*s, device="cuda").bfloat16()
    gq, sw, wd = r(M, d), r(M, F), r(d, F)
    dgu, h2, wgu = r(M, 2 * F), r(M, d), r(2 * F, d)
    g2, o, wo = r(M, d), r(M, d), r(d, d)
    dqkv, h1, wqkv = r(M, 3 * d), r(M, d), r(3 * d, d)
    qkv = r(M, 3 * d)
    q, kk, v = (qkv[:, i * d:(i + 1) * d].view(B, T, H, hd) for i in range(3))
    ao, lse = k.attn_fwd(q, kk, v, 1 / math.sqrt(hd), True)
    dq_, dk_, dv_ = (dqkv[:, i * d:(i + 1) * d].view(B, T, H, hd) for i in range(3))
    acc = {n: torch.zeros(s, device="cuda") for n, s in (("wd", (d, F)), ("wgu", (2 * F, d)), ("wo", (d, d)),
                                                        ("wqkv", (3 * d, d)))}
    side = torch.cuda.Stream()
    pairs = {
        "down   nn(M,F<-d) | tn(d x F)": (lambda: GS.gemm_nn(k, gq, wd), lambda: GS.gemm_tn(k, gq, sw, acc["wd"], True)),
        "gateup nn(M,d<-2F) | tn(2F x d)": (lambda: GS.gemm_nn(k, dgu, wgu), lambda: GS.gemm_tn(k, dgu, h2, acc["wgu"], True)),
        "wo     nn(M,d<-d) | tn(d x d)": (lambda: GS.gemm_nn(k, g2, wo), lambda: GS.gemm_tn(k, g2, o, acc["wo"], True)),
        "attn_bwd | tn(d x d) [wo]": (lambda: k.attn_bwd(g2.view(B, T, H, hd), q, kk, v, ao, lse, 1 / math.sqrt(hd), True,
                                                         dq_, dk_, dv_), lambda: GS.gemm_tn(k, g2, o, acc["wo"], True)),
        "qkv    nn(M,d<-3d) | tn(3d x d)": (lambda: GS.gemm_nn(k, dqkv, wqkv), lambda: GS.gemm_tn(k, dqkv, h1, acc["wqkv"], True)),
    }

    def serial(f, g):
        def run():
            f()
            g()
        return run

    def overlap(f, g):
        def run():
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                g()
            f()
            torch.cuda.current_stream().wait_stream(side)
        return run

    fns = {}
    for name, (f, g) in pairs.items():
        fns[name + " :: main only"] = f
        fns[name + " :: side only"] = g
        fns[name + " :: serial"] = serial(f, g)
        fns[name + " :: two streams"] = overlap(f, g)

    def layer(two):
        def run():
            for f, g in pairs.values():
                if two:
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        g()
                    f()
                else:
                    f()
                    g()
            torch.cuda.current_stream().wait_stream(side)
        return run
    fns["whole layer :: serial"] = layer(False)
    fns["whole layer :: two streams"] = layer(True)
    res = timeit(fns, iters=20, rounds=5)
    for name, ms in res.items():
        print(f"{name:55s} {ms * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
