"""Time the lm_head forward GEMM + CE statistics + in-place CE backward over all tokens at once
vs in token chunks (a chunk's logits stay in the 256 MB Infinity Cache between the three passes).

    python tools/ce_chunk_probe.py --M 32768 --V 50304 --d 768 --chunks 0 8192 4096 2048 1024
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--V", type=int, default=50304)
    ap.add_argument("--valid", type=int, default=50257)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--chunks", type=int, nargs="+", default=[0, 8192, 4096, 2048, 1024])
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    C = _ext.require()
    M, V, d = a.M, a.V, a.d
    dev = "cuda"
    hf = torch.randn(M, d, device=dev).bfloat16()
    W = (torch.randn(V, d, device=dev) * 0.02).bfloat16()
    bias = torch.randn(V, device=dev).bfloat16() * 0.01
    tgt = torch.randint(0, a.valid, (M,), device=dev)
    gs = torch.full((M,), 1.0 / M, device=dev)
    buf = torch.empty(M, V, device=dev, dtype=torch.bfloat16)
    db = torch.empty(V, device=dev)

    def run(chunk):
        c = chunk or M
        for s in range(0, M, c):
            e = min(M, s + c)
            lg = buf[s:e]
            torch.addmm(bias, hf[s:e], W.t(), out=lg)
            st = C.ce_fwd_stats(lg, tgt[s:e], 0, a.valid)
            lse = st[:, 0] + torch.log(st[:, 1])
            C.ce_bwd(lg, tgt[s:e], lse, gs[s:e], 0, a.valid, lg, db)

    for chunk in a.chunks:
        run(chunk)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.iters):
            run(chunk)
        ev[1].record()
        torch.cuda.synchronize()
        print(f"chunk {chunk or M}: {ev[0].elapsed_time(ev[1]) / a.iters:.3f} ms (GEMM + stats + CE bwd)", flush=True)
    # the three passes separately at full size
    for name, fn in (("gemm", lambda: torch.addmm(bias, hf, W.t(), out=buf)),
                     ("stats", lambda: C.ce_fwd_stats(buf, tgt, 0, a.valid)),
                     ("bwd", lambda: C.ce_bwd(buf, tgt, torch.zeros(M, device=dev), gs, 0, a.valid, buf, db))):
        fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.iters):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        print(f"  {name}: {ev[0].elapsed_time(ev[1]) / a.iters:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
