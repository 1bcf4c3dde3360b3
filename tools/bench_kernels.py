"""Micro-benchmarks of the hot kernels at the headline (GPT-2 small) shapes.

Times each hand-written kernel against the vendor path of the same op in the same process
(interleaved rounds, median; guide §5.4 rule 24) on random data:
  * GEMM NT / NN / TN  vs torch.matmul (hipBLASLt)
  * causal attention fwd (+bwd) vs torch SDPA
Prints one JSON line per case.  Usage: python tools/bench_kernels.py [--tp N] [--tokens M]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402


def timeit(fns, iters=20, rounds=5):
    """Interleaved timing, median over rounds.  One untimed pass over every arm first, and the
    arm order rotates per round: the arm timed first in a round read ~2.5 % slow
    (profiles/r4_kernel_experiments.txt item 18)."""
    res = {k: [] for k in fns}
    keys = list(fns)
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    for rd in range(rounds):
        for k in keys[rd % len(keys):] + keys[:rd % len(keys)]:
            f = fns[k]
            f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                f()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) / iters)
    return {k: sorted(v)[len(v) // 2] for k, v in res.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--ffn", type=int, default=2048)
    ap.add_argument("--vocab", type=int, default=50304)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    C = _ext.require()
    dev = "cuda"
    M, d, f, V, n = a.tokens, a.d, a.ffn, a.vocab, a.tp
    hl = max(1, math.ceil(a.heads / n))
    hd = d // a.heads
    shapes = {
        "qkv": (M, 3 * hl * hd, d), "wo": (M, d, hl * hd), "gate_up": (M, 2 * f // n, d),
        "down": (M, d, f // n), "lm_head": (M, V // n, d),
    }
    if not a.only or "gemm" in a.only:
        for name, (m, nn_, k) in shapes.items():
            x = torch.randn(m, k, device=dev).bfloat16()
            w = torch.randn(nn_, k, device=dev).bfloat16()
            dy = torch.randn(m, nn_, device=dev).bfloat16()
            fl = 2.0 * m * nn_ * k
            def old(f, impl=1):
                def g():
                    C.gemm_set_impl(impl)
                    f()
                    C.gemm_set_impl(3)
                return g
            t = timeit({
                "nt": lambda: C.gemm_nt(x, w, None), "nt_ref": lambda: x @ w.t(),
                "nt_v1": old(lambda: C.gemm_nt(x, w, None)), "nn_v1": old(lambda: C.gemm_nn(dy, w)),
                "tn_v1": old(lambda: C.gemm_tn(dy, x)),
                "nn": lambda: C.gemm_nn(dy, w), "nn_ref": lambda: dy @ w,
                "tn": lambda: C.gemm_tn(dy, x), "tn_ref": lambda: dy.t() @ x,
            })
            out = {"case": f"gemm_{name}", "M": m, "N": nn_, "K": k}
            for key, ms in t.items():
                out[key + "_ms"] = round(ms, 4)
                out[key + "_tflops"] = round(fl / ms / 1e9, 1)
            print(json.dumps(out), flush=True)
    if not a.only or "attn" in a.only:
        B = max(1, M // a.seq)
        T = a.seq
        qkv = torch.randn(B * T, 3 * hl * hd, device=dev).bfloat16()
        q, k, v = (qkv[:, i * hl * hd:(i + 1) * hl * hd].view(B, T, hl, hd) for i in range(3))
        scale = 1 / math.sqrt(hd)
        o, lse = C.attn_fwd(q, k, v, scale, True)
        do = torch.randn_like(o)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = (dqkv[:, i * hl * hd:(i + 1) * hl * hd].view(B, T, hl, hd) for i in range(3))
        qt, kt, vt = (t.transpose(1, 2).contiguous().requires_grad_(True) for t in (q, k, v))
        F = torch.nn.functional

        def ref_fb():
            out = F.scaled_dot_product_attention(qt, kt, vt, is_causal=True)
            out.backward(do.transpose(1, 2))

        t = timeit({
            "fwd": lambda: C.attn_fwd(q, k, v, scale, True),
            "fwd_r1": lambda: C.attn_fwd(q, k, v, scale, True, impl=1),
            "fwd_ref": lambda: F.scaled_dot_product_attention(qt.detach(), kt.detach(), vt.detach(), is_causal=True),
            "bwd": lambda: C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv),
            "fwdbwd_ref": ref_fb,
        }, iters=10)
        fl = 4.0 * B * hl * T * T * hd / 2
        out = {"case": "attention", "B": B, "T": T, "H": hl, "hd": hd}
        for key, ms in t.items():
            mult = 1 if key.startswith("fwd") and "bwd" not in key else (2.5 if key == "bwd" else 3.5)
            out[key + "_ms"] = round(ms, 4)
            out[key + "_tflops"] = round(mult * fl / ms / 1e9, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
