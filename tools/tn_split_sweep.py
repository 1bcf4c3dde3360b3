"""TN (weight-gradient) GEMM: time every (tile config, K-split) on the engine's wgrad shapes.

    python tools/tn_split_sweep.py [--tokens 131072] [--shapes 384x768 768x128 ...]

Shape MxN = weight-gradient output (out_features x in_features), K = tokens.  Prints one JSON
line per shape: the automatic plan's time and the best forced (cfg, splits).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--shapes", nargs="+", default=["384x768", "768x128", "512x768", "768x256"])
    ap.add_argument("--splits", type=int, nargs="+", default=[4, 8, 12, 16, 21, 24, 32, 42, 48, 64])
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    C = _ext.require()
    K = a.tokens

    def t(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / a.iters

    for sh in a.shapes:
        M, N = map(int, sh.split("x"))
        dy = torch.randn(K, M, device="cuda").bfloat16()
        x = torch.randn(K, N, device="cuda").bfloat16()
        acc = torch.zeros(M, N, device="cuda")
        res = {}
        C.gemm_force(-1, 0)
        res["auto"] = t(lambda: C.gemm_tn(dy, x, acc, True))
        for cfg in (0, 1):
            for S in a.splits:
                C.gemm_force(cfg, S)
                res[f"c{cfg}s{S}"] = t(lambda: C.gemm_tn(dy, x, acc, True))
        C.gemm_force(-1, 0)
        best = min((k for k in res if k.startswith("c")), key=res.get)
        fl = 2.0 * M * N * K
        print(json.dumps({"M": M, "N": N, "K": K, "auto_ms": round(res["auto"], 4),
                          "auto_tflops": round(fl / res["auto"] / 1e9, 1), "best": best,
                          "best_ms": round(res[best], 4), "best_tflops": round(fl / res[best] / 1e9, 1),
                          "all": {k: round(v, 4) for k, v in res.items() if k.startswith("c")}}), flush=True)


if __name__ == "__main__":
    main()
