"""Attention kernels timed alone vs in step-like context (GPT-2-small layer shape).

The step trace prices the backward at ~0.37 ms per layer, back-to-back timing at ~0.28 ms.
Arms (each call bracketed by its own events, median over --n calls):
  hot        back-to-back calls (the operands stay in the 256 MiB infinity cache / L2)
  hot_rope   + inverse RoPE and the QKV bias gradient, as the training step calls it
  rope_only / bias_only  one of the two
  cold       a 1 GiB memset before each call (infinity cache / L2 flushed)
  after_gemm a bf16 GEMM (~1 ms) before each call (chip under MFMA load, as between the step's GEMMs)

    python tools/attn_ctx_probe.py [--fwd]
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
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--fwd", action="store_true")
    ap.add_argument("--impls", type=int, nargs="*", default=[],
                    help="backward implementations to compare as the step calls them (RoPE + bias), e.g. 4 6 7 9")
    a = ap.parse_args()
    C = _ext.require()
    B, T, H, hd = 32, 1024, 12, 64
    qkv = torch.randn(B * T, 3 * H * hd, device="cuda").bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    scale = 1 / math.sqrt(hd)
    o, lse = C.attn_fwd(q, k, v, scale, True)
    do = torch.randn_like(o)
    d = torch.empty_like(qkv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    pos = torch.arange(T, device="cuda").repeat(B).contiguous()
    inv = 1.0 / (10000 ** (torch.arange(0, hd, 2, device="cuda").float() / hd))
    ang = torch.arange(T, device="cuda").float()[:, None] * inv[None]
    tab = torch.cat([ang.cos(), ang.sin()], 1).contiguous()
    db = torch.empty(3 * H * hd, device="cuda")
    flush = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    ga = torch.randn(8192, 8192, device="cuda").bfloat16()
    gb = torch.randn(8192, 8192, device="cuda").bfloat16()

    def bwd(rope=False, bias=None):
        bias = rope if bias is None else bias
        C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv, pos if rope else None, tab if rope else None,
                   db if bias else None)

    def fwd():
        C.attn_fwd(q, k, v, scale, True)

    op = fwd if a.fwd else bwd
    if a.impls:   # implementation comparison only: every arm with RoPE + bias, as the step calls it
        arms = {f"impl{i}": (None, (lambda i=i: C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv, pos, tab, db,
                                                              impl=i))) for i in a.impls}
    else:
        arms = {}
    arms = arms or {
        "hot": (None, op),
        "hot_rope": (None, (lambda: bwd(True)) if not a.fwd else op),
        "rope_only": (None, (lambda: bwd(True, False)) if not a.fwd else op),
        "bias_only": (None, (lambda: bwd(False, True)) if not a.fwd else op),
        "cold": (lambda: flush.zero_(), op),
        "after_gemm": (lambda: torch.mm(ga, gb), op),
        "cold_rope": (lambda: flush.zero_(), (lambda: bwd(True)) if not a.fwd else op),
    }
    res = {k_: [] for k_ in arms}
    for _ in range(2):
        for pre, f in arms.values():
            if pre:
                pre()
            f()
    torch.cuda.synchronize()
    for i in range(a.n):
        for name, (pre, f) in arms.items():
            if pre:
                pre()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            f()
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e))
    for name, v_ in res.items():
        v_.sort()
        print(f"{'fwd' if a.fwd else 'bwd'} {name:>11}: median {v_[len(v_) // 2]:.4f} ms  min {v_[0]:.4f}  "
              f"max {v_[-1]:.4f}", flush=True)


if __name__ == "__main__":
    main()
