"""Fused Adam (csrc/kernels/adam.hip) on the GPT-2-small parameter set (124M fp32 params in the
model's tensor shapes, bf16 shadows for the 2-D ones): time per step and the achieved HBM
bytes/s (30 B per parameter: fp32 param / m / v read + written, fp32 grad read, bf16 shadow
written).

    python tools/adam_probe.py [--rounds 5] [--iters 20]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C = _ext.require()
    from distributed_pytorch_from_scratch_amd.models import get_preset, Transformer
    from distributed_pytorch_from_scratch_amd.ops.optim import FusedAdam
    args = get_preset("gpt2-small")
    m = Transformer.from_args(args).cuda()
    for p in m.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    opt = FusedAdam(m.parameters(), lr=3e-4)
    opt.step()
    n = sum(p.numel() for p in m.parameters())
    ts = {1: []}
    for rd in range(a.rounds):
        for u in (1,):
            opt.step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                opt.step()
            e1.record()
            e1.synchronize()
            ts[u].append(e0.elapsed_time(e1) / a.iters)
    for u, v in ts.items():
        med = statistics.median(v)
        print(f"fused adam: {med:.4f} ms (min {min(v):.4f})  {30 * n / med / 1e9:.2f} TB/s over {n / 1e6:.1f}M params")


if __name__ == "__main__":
    main()
