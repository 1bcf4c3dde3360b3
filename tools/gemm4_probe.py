"""GEMM v4 (csrc/kernels/gemm4.hip) vs v3 (gemm.hip gemmp_k) vs hipBLASLt on the GPT-2-small
step shapes: correctness against fp32 torch, then interleaved timing rounds in one process
(CDNA guide rule 24: variants x rounds, median and min reported).

    python tools/gemm4_probe.py [--rounds 7] [--iters 10] [--layouts nt nn tn] [--check-only]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_from_scratch_amd.ops import _ext  # noqa: E402

T = 32768
SHAPES = {
    # (M, N, K) of C[M,N] = A . B  (names: the GPT-2-small projection they serve)
    "nt": [("qkv", T, 2304, 768), ("wo", T, 768, 768), ("gateup", T, 4096, 768), ("down", T, 768, 2048),
           ("lmhead", T, 50304, 768)],
    "nn": [("qkv", T, 768, 2304), ("wo", T, 768, 768), ("gateup", T, 768, 4096), ("down", T, 2048, 768),
           ("lmhead", T, 768, 50304)],
    "tn": [("qkv", 2304, 768, T), ("wo", 768, 768, T), ("gateup", 4096, 768, T), ("down", 768, 2048, T),
           ("lmhead", 50304, 768, T)],
}
# square shapes (--big): the main loop's rate where prologue / epilogue costs are amortised
BIG = {l: [("sq4k", 4096, 4096, 4096), ("sq8k", 8192, 8192, 8192)] for l in ("nt", "nn", "tn")}
# per-call kernel variant of the next `ours` call (0 = v4 at its own width, 1 / 2 = v4 256 / 192
# wide, 3 = v3): an argument of the kernel entry points, set here per arm
VAR = [0]


def set_variant(mask_or_v4: int, bn: int = 0):
    VAR[0] = 3 if not mask_or_v4 else {0: 0, 256: 1, 192: 2}[bn]


def operands(layout, M, N, K, gen, bias=False):
    r = lambda *s: torch.randn(*s, device="cuda", generator=gen).bfloat16()
    if layout == "nt":
        a, b = r(M, K), r(N, K)
        bv = torch.randn(N, device="cuda", generator=gen) if bias else None
        bb = bv.bfloat16() if bias else None
        return a, b, (lambda C: C.gemm_nt(a, b, bv, variant=VAR[0])), (lambda: torch.nn.functional.linear(a, b, bb)), \
            (lambda: a.float() @ b.float().t() + (bv if bias else 0))
    if layout == "nn":
        a, b = r(M, K), r(K, N)
        return a, b, (lambda C: C.gemm_nn(a, b, variant=VAR[0])), (lambda: torch.matmul(a, b)), (lambda: a.float() @ b.float())
    a, b = r(K, M), r(K, N)
    return a, b, (lambda C: C.gemm_tn(a, b, variant=0 if VAR[0] != 3 else 3)), (lambda: torch.mm(a.t(), b, out_dtype=torch.float32)), \
        (lambda: a.float().t() @ b.float())


def timed(fn, iters):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


_FLUSH = []


def timed_cold(fn, iters):
    """Per-call time with the caches flushed before every call (a 512 MB write evicts the L2s and
    the Infinity Cache), as in the training step where the operands come from HBM."""
    if not _FLUSH:
        _FLUSH.append(torch.empty(128 * 1024 * 1024, dtype=torch.float32, device="cuda"))
    fn()
    tot = 0.0
    for _ in range(iters):
        _FLUSH[0].fill_(1.0)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        tot += s.elapsed_time(e)
    return tot / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--layouts", nargs="+", default=["nt", "nn", "tn"])
    ap.add_argument("--shapes", nargs="+", default=None, help="subset of names (qkv wo gateup down lmhead)")
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--scheds", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--no-blas", action="store_true")
    ap.add_argument("--bias", action="store_true", help="NT with an fp32 bias (the projections that carry one)")
    ap.add_argument("--bn", type=int, nargs="*", default=[],
                    help="extra arms: the last --scheds variant with the v4 tile width forced (256 / 192)")
    ap.add_argument("--splits", type=int, nargs="*", default=[],
                    help="extra arms (TN): the last --scheds variant with the K-split count forced (gemm_force)")
    ap.add_argument("--group-m", type=int, nargs="*", default=[],
                    help="extra arms: the last --scheds variant with this item-order group size")
    ap.add_argument("--diag", action="store_true",
                    help="NT / TN (32x32x16): DIAG build's per-wave cycle split (step waits / bodies / epilogues), s_memtime")
    ap.add_argument("--ablate", type=int, nargs="*", default=[],
                    help="extra v4 arms with timing-only ablations (bits: 1 no stores, 2 zero operands, 4 no DMA wait, 8 no step barrier)")
    ap.add_argument("--cold", action="store_true", help="flush the caches before every timed call")
    ap.add_argument("--big", action="store_true", help="also the 4096^3 / 8192^3 square shapes")
    ap.add_argument("--sk", action="store_true", help="NT / NN: also the stream-K kernel (variant 8) where it applies")
    ap.add_argument("--custom", type=int, nargs=3, action="append", default=[], metavar=("M", "N", "K"),
                    help="extra shape(s) of every --layouts layout (name 'cM_N_K')")
    ap.add_argument("--br", type=int, nargs="*", default=[],
                    help="extra arms: the last --scheds variant with BR rows of MFMAs before each step's barrier")
    a = ap.parse_args()
    if a.cold:
        global timed
        timed = timed_cold
    C = _ext.require()
    gen = torch.Generator(device="cuda").manual_seed(0)
    for layout in a.layouts:
        for name, M, N, K in SHAPES[layout] + (BIG[layout] if a.big else []) + \
                [(f"c{m}_{n}_{k}", m, n, k) for m, n, k in a.custom]:
            if a.shapes and name not in a.shapes and not name.startswith("c"):
                continue
            _, _, ours, blas, ref = operands(layout, M, N, K, gen, a.bias)
            want = ref() if M * N <= 50304 * 768 * 2 else None
            res = {}
            for tag, mask, sc, bn in [(f"v4s{sc}", 7, sc, 0) for sc in a.scheds] + \
                    [(f"bn{b}", 7, a.scheds[-1], b) for b in a.bn] + [("v3", 0, 0, 0)]:
                set_variant(mask, bn)
                C.gemm4_sched(sc)
                if want is not None:
                    out = ours(C).float()
                    res[tag] = ((out - want).norm() / want.norm()).item()
            for x in a.ablate:   # the non-destructive switches (64 = W8 epilogue stores) are checked too
                if want is not None and not (x & 15):
                    set_variant(1)
                    C.gemm4_ablate(x)
                    out = ours(C).float()
                    C.gemm4_ablate(0)
                    res[f"abl{x}"] = ((out - want).norm() / want.norm()).item()
                    C.gemm4_ablate(x)
                    o2 = ours(C)
                    C.gemm4_ablate(0)
                    res[f"abl{x}_bitwise_vs_default"] = float(torch.equal(o2, ours(C)))
            for br in a.br:                   # the BR variants: bit-identical to BR 0
                if want is not None:
                    set_variant(1)
                    C.gemm4_sched(a.scheds[-1])
                    C.gemm4_br(br)
                    o = ours(C)
                    C.gemm4_br(0)
                    res[f"br{br}_bitwise_vs_default"] = float(torch.equal(o, ours(C)))
            set_variant(1)
            del want
            flops = 2.0 * M * N * K
            print(f"{layout} {name} {M}x{N}x{K}: rel err " + " ".join(f"{k} {v:.2e}" for k, v in res.items()),
                  flush=True)
            if a.check_only:
                continue
            for dmode in ((16, 17, 32) if a.diag and layout in ("nt", "tn") else ()):
                d = torch.zeros(256 * 4 * 4, dtype=torch.int64, device="cuda")
                C.gemm4_diag(d)
                set_variant(1)
                C.gemm4_ablate(dmode)
                ours(C)
                torch.cuda.synchronize()
                d.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ours(C)
                e1.record()
                e1.synchronize()
                wall_ms = e0.elapsed_time(e1)
                C.gemm4_ablate(0)
                C.gemm4_diag(torch.empty(0))
                v = d.view(-1, 4).double()
                v = v[v[:, 3] > 0]
                if v.shape[0] == 0:   # the DIAG build covers the 256-wide FAST NT kernel only
                    print(f"{layout} {name} DIAG: no 256-wide launch for this shape", flush=True)
                    continue
                tiles = ((M + 255) // 256) * ((N + 255) // 256)
                if layout == "tn":   # items = tiles x K-splits
                    tiles *= max(1, C.gemm_tn_splits(M, N, K)) if hasattr(C, "gemm_tn_splits") else 1
                per = tiles / (v.shape[0] / 4)
                tot = v[:, :3].sum(1)
                clk = (v[:, :3].sum(1).max().item()) / (wall_ms * 1e-3) / 1e9   # longest wave's cycles / wall
                tagd = {16: "", 17: "(no stores)", 32: "(no DMA issued)"}[dmode]
                print(f"{layout} {name} DIAG{tagd} wall {wall_ms:.4f} ms, clock >= {clk:.2f} GHz; per wave (s_memtime ticks, mean over {v.shape[0]} waves, {per:.1f} tiles "
                      f"per WG): wait {v[:, 0].mean():.0f}  body {v[:, 1].mean():.0f}  epilogue {v[:, 2].mean():.0f}  "
                      f"-> per tile wait {v[:, 0].mean() / per:.0f} body {v[:, 1].mean() / per:.0f} "
                      f"epi {v[:, 2].mean() / per:.0f}; shares wait {(v[:, 0] / tot).mean():.3f} "
                      f"epi {(v[:, 2] / tot).mean():.3f}", flush=True)
            arms = [f"v4s{sc}" for sc in a.scheds] + [f"br{x}" for x in a.br] + [f"gm{g}" for g in a.group_m] + [f"bn{b}" for b in a.bn] + [f"sp{x}" for x in a.splits] + \
                [f"abl{x}" for x in a.ablate] + ["v3"] + \
                (["sk"] if a.sk and layout in ("nt", "nn") and C.gemm_sk_applies(M, N, K) else []) + \
                ([] if a.no_blas else ["blas"])
            ts = {k: [] for k in arms}
            for rd in range(a.rounds):
                # (the arm order rotates per round: the first-timed arm of a round reads slow)
                for k in arms[rd % len(arms):] + arms[:rd % len(arms)]:
                    if k.startswith("v4s"):
                        set_variant(1)
                        C.gemm4_sched(int(k[3:]))
                        ts[k].append(timed(lambda: ours(C), a.iters))
                    elif k.startswith("br"):
                        set_variant(1)
                        C.gemm4_sched(a.scheds[-1])
                        C.gemm4_br(int(k[2:]))
                        ts[k].append(timed(lambda: ours(C), a.iters))
                        C.gemm4_br(0)
                    elif k.startswith("sp"):
                        set_variant(1)
                        C.gemm4_sched(a.scheds[-1])
                        C.gemm_force(-1, int(k[2:]))
                        ts[k].append(timed(lambda: ours(C), a.iters))
                        C.gemm_force(-1, 0)
                    elif k.startswith("bn"):
                        set_variant(1)
                        C.gemm4_sched(a.scheds[-1])
                        set_variant(1, int(k[2:]))
                        ts[k].append(timed(lambda: ours(C), a.iters))
                        set_variant(1)
                    elif k.startswith("gm"):
                        set_variant(1)
                        C.gemm4_sched(a.scheds[-1])
                        C.gemm4_group_m(int(k[2:]))
                        ts[k].append(timed(lambda: ours(C), a.iters))
                        C.gemm4_group_m(4)
                    elif k.startswith("abl"):
                        set_variant(1)
                        C.gemm4_sched(a.scheds[-1])
                        C.gemm4_ablate(int(k[3:]))
                        ts[k].append(timed(lambda: ours(C), a.iters))
                        C.gemm4_ablate(0)
                    elif k == "sk":
                        VAR[0] = 8
                        ts[k].append(timed(lambda: ours(C), a.iters))
                        set_variant(1)
                    elif k == "v3":
                        set_variant(0)
                        ts[k].append(timed(lambda: ours(C), a.iters))
                    else:
                        ts[k].append(timed(blas, a.iters))
            set_variant(1)
            C.gemm4_sched(a.scheds[-1])
            line = "   ".join(f"{k} {statistics.median(v):.4f} ms (min {min(v):.4f}) "
                               f"{flops / statistics.median(v) / 1e9:.0f} TF" for k, v in ts.items())
            print(f"{layout} {name} {M}x{N}x{K}: {line}", flush=True)


if __name__ == "__main__":
    main()
