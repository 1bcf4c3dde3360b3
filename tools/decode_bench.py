"""Greedy decode throughput: HIP-graph-replayed decode step vs the eager step vs the
reference's full recompute per token (test.py:144-150), one GPU.

    python tools/decode_bench.py [--model gpt2-small] [--batch 1 8] [--prompt 128] [--new 256]

Prints one JSON line per (batch, mode): ms per generated token (per step of the batch) and
tokens/s (batch x steps / time).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--recompute-new", type=int, default=32, help="tokens for the full-recompute baseline")
    a = ap.parse_args()
    import torch
    from distributed_pytorch_from_scratch_amd.models import get_preset, Transformer
    from distributed_pytorch_from_scratch_amd.models.generation import generate
    from distributed_pytorch_from_scratch_amd.utils.dist import init_dist_env
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29591")
    init_dist_env(rank=0, tp_size=1, world_size=1)
    args = get_preset(a.model)
    m = Transformer.from_args(args).cuda()
    m.reset_parameters()
    m.eval()
    for B in a.batch:
        prompt = torch.randint(0, args.vocab_size, (B, a.prompt), device="cuda")
        for mode in ("graph", "eager"):
            os.environ["DPFS_DECODE_GRAPH"] = "1" if mode == "graph" else "0"
            generate(m, prompt, max_new_tokens=a.new)           # warm-up: GEMM choices, graph capture
                                                                #   (reused by the same-shape call)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            generate(m, prompt, max_new_tokens=a.new)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"model": a.model, "batch": B, "mode": mode, "prompt": a.prompt, "new": a.new,
                              "ms_per_step": round(1000 * dt / a.new, 3),
                              "tokens_per_s": round(B * a.new / dt, 1)}), flush=True)
        # reference formulation: every token re-runs the whole prefix (no cache)
        seq = prompt
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.inference_mode():
            for _ in range(a.recompute_new):
                T = seq.size(1)
                logits = m(seq, torch.arange(T, device="cuda").repeat(B, 1))[:, -1]
                seq = torch.cat([seq, logits.argmax(-1, keepdim=True)], 1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"model": a.model, "batch": B, "mode": "full-recompute", "prompt": a.prompt,
                          "new": a.recompute_new, "ms_per_step": round(1000 * dt / a.recompute_new, 3),
                          "tokens_per_s": round(B * a.recompute_new / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
