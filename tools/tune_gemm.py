"""Sweep GEMM implementations / tile configs / K-splits per (layout, shape) on the GPU.

Prints one JSON line per (shape, layout) with the time of every variant, so the static
selection heuristics in csrc/kernels/gemm.hip can be set from measurements.
"""
import argparse, json, math, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext
from tools.bench_kernels import timeit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--tokens-per-tp", type=int, default=16384)
    ap.add_argument("--layouts", nargs="+", default=["nt", "nn", "tn"])
    ap.add_argument("--gemms", nargs="+", default=["qkv", "wo", "gate_up", "down", "lm_head"])
    a = ap.parse_args()
    C = _ext.require()
    d, f, V, H = 768, 2048, 50304, 12
    hd = d // H
    for n in a.tp:
        M = a.tokens_per_tp * n
        hl = math.ceil(H / n)
        shapes = {"qkv": (M, 3 * hl * hd, d), "wo": (M, d, hl * hd), "gate_up": (M, 2 * f // n, d),
                  "down": (M, d, f // n), "lm_head": (M, V // n, d)}
        for name, (m, nn_, k) in shapes.items():
            x = torch.randn(m, k, device="cuda").bfloat16()
            w = torch.randn(nn_, k, device="cuda").bfloat16()
            dy = torch.randn(m, nn_, device="cuda").bfloat16()
            ops = {"nt": lambda: C.gemm_nt(x, w, None), "nn": lambda: C.gemm_nn(dy, w),
                   "tn": lambda: C.gemm_tn(dy, x)}
            flops = 2.0 * m * nn_ * k
            if name not in a.gemms:
                continue
            for lay, fn in ops.items():
                if lay not in a.layouts:
                    continue
                variants = {}
                out_elems = nn_ * k if lay == "tn" else m * nn_
                if out_elems * 4 * (32 if lay == "tn" else 4) > 24e9:  # split-K slabs beyond ~24 GB
                    continue
                def mk(impl, cfg, sp):
                    def g():
                        C.gemm_set_impl(impl); C.gemm_force(cfg, sp)
                        fn()
                        C.gemm_set_impl(3); C.gemm_force(-1, 0)
                    return g
                variants["v1"] = mk(1, -1, 0)
                variants["auto"] = mk(2, -1, 0)
                for cfg in (0, 1):
                    for sp in ((1, 2, 4) if lay != "tn" else (1, 2, 4, 8, 16, 32)):
                        variants[f"c{cfg}s{sp}"] = mk(2, cfg, sp)
                t = timeit(variants, iters=10, rounds=3)
                best = min(t, key=t.get)
                print(json.dumps({"tp": n, "gemm": name, "layout": lay, "M": m, "N": nn_, "K": k, "best": best,
                                  "best_tflops": round(flops / t[best] / 1e9, 1),
                                  "auto_tflops": round(flops / t["auto"] / 1e9, 1),
                                  "ms": {kk: round(v, 4) for kk, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
