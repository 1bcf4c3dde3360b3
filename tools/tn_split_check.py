"""Forced K-split counts vs the planner's choice for the TN weight-gradient GEMMs of the GPT-2
small TP 1 step (M = 32768 tokens): prints each shape's best forced (cfg, S) next to auto.

    python tools/tn_split_check.py
"""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402

C = _ext.require()
K = 32768


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for M, N in ((2304, 768), (768, 768), (4096, 768), (768, 2048), (50304, 768)):
    dy = torch.randn(K, M, device="cuda").bfloat16()
    x = torch.randn(K, N, device="cuda").bfloat16()
    res = []
    for cfg in (0, 1):
        for S in range(1, 17):
            C.gemm_force(cfg, S)
            res.append((t(lambda: C.gemm_tn(dy, x)), cfg, S))
    C.gemm_force(-1, 0)
    auto = t(lambda: C.gemm_tn(dy, x))
    best = min(res)
    print(f"tn {M}x{N}x{K}: auto {auto:.4f} ms (S={C.gemm_tn_splits(M, N, K) if hasattr(C, 'gemm_tn_splits') else '?'}), "
          f"best forced {best[0]:.4f} ms at cfg {best[1]} S {best[2]}", flush=True)
