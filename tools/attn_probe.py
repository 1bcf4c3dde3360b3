"""Run the attention kernels repeatedly with chosen implementations (for rocprofv3 PMC runs).

    python tools/attn_probe.py --B 32 --T 1024 --H 12 --hd 64 --impl 1 4 --iters 10 [--bwd]
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
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--hd", type=int, default=64)
    ap.add_argument("--impl", type=int, nargs="+", default=[4])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--diag", action="store_true",
                    help="forward v3 DIAG build (impl 5): per-wave s_memtime split wait / QK+max / exp+pack / PV")
    ap.add_argument("--ab", default=None, help="name of a temporary int kernel switch of _C to A/B (forward or --bwd)")
    ap.add_argument("--ab-vals", type=int, nargs="+", default=[0, 1])
    a = ap.parse_args()
    C = _ext.require()
    B, T, H, hd = a.B, a.T, a.H, a.hd
    qkv = torch.randn(B * T, 3 * H * hd, device="cuda").bfloat16()
    q, k, v = (qkv[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    scale = 1 / math.sqrt(hd)
    o, lse = C.attn_fwd(q, k, v, scale, True)
    do = torch.randn_like(o)
    d = torch.empty_like(qkv)
    dq, dk, dv = (d[:, i * H * hd:(i + 1) * H * hd].view(B, T, H, hd) for i in range(3))
    fl = 4.0 * B * H * T * T * hd / 2 * (2.5 if a.bwd else 1.0)
    from tools.bench_kernels import timeit

    def mk(impl):
        def g():
            if a.bwd:
                C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv, impl=impl)
            else:
                C.attn_fwd(q, k, v, scale, True, impl=impl)
        return g
    if not a.bwd:   # forward outputs of every implementation against impl 1
        o1, l1 = C.attn_fwd(q, k, v, scale, True, impl=1)
        for impl in a.impl:
            oi, li = C.attn_fwd(q, k, v, scale, True, impl=impl)
            print(f"impl {impl} vs 1: max|dO| {(oi.float() - o1.float()).abs().max().item():.3e} "
                  f"max|dLSE| {(li - l1).abs().max().item():.3e}", flush=True)
    if a.diag and not a.bwd:
        grid = ((T + 127) // 128) * B * H
        d = torch.zeros(grid * 40, dtype=torch.int64, device="cuda")
        C.attn_diag(d)
        C.attn_fwd(q, k, v, scale, True, impl=5)
        torch.cuda.synchronize()
        C.attn_diag(torch.empty(0))
        torch.save(d.cpu(), os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "attn_diag.pt"))
        w10 = d.view(-1, 10).double()
        w10 = w10[w10[:, 7] > 0]                # (rows of the buffer past the grid stay zero)
        pro = w10[:, 8]
        w8 = w10[:, :8]
        print(f"DIAG per wave, block prologues {pro.mean():.0f} ticks, epilogues {w10[:, 9].mean():.0f} ticks", flush=True)
        w = w8[:, :4]
        life = w8[:, 5] - w8[:, 4]
        span = (w8[:, 5].max() - w8[:, 4].min()).item()
        rt = w8[:, 7] - w8[:, 6]
        rspan = (w8[:, 7].max() - w8[:, 6].min()).item()
        print(f"DIAG realtime (100 MHz): kernel span {rspan / 100:.1f} us, wave life mean {rt.mean() / 100:.2f} us; "
              f"s_memtime ticks per us {(life / rt).mean() * 100:.0f}; sum of wave lives / (span x 12 waves x 256 CUs) "
              f"{rt.sum().item() / rspan / (256 * 12) * 100:.1f}%", flush=True)
        ev = torch.cat([torch.stack([w8[:, 6], torch.ones_like(rt)], 1), torch.stack([w8[:, 7], -torch.ones_like(rt)], 1)])
        ev = ev[ev[:, 0].argsort()]
        conc = ev[:, 1].cumsum(0)
        tq = [(w8[:, 6].min() + f * rspan).item() for f in (0.1, 0.25, 0.5, 0.75, 0.9)]
        cq = [conc[(ev[:, 0] <= x).nonzero().max()].item() for x in tq]
        print(f"DIAG resident waves: max {conc.max().item():.0f}; at 10/25/50/75/90% of the span {cq}", flush=True)
        print(f"DIAG kernel span {span:.0f} ticks; wave life mean {life.mean():.0f} (loop share "
              f"{(w.sum(1) / life).mean() * 100:.1f}%), sum of wave lives / (span x resident waves) "
              f"{life.sum().item() / span / (256 * 12) * 100:.1f}%", flush=True)
        tot = w.sum(1)
        names = ["wait+barrier", "QK+mask+max", "exp+pack", "PV"]
        print("DIAG per wave (s_memtime ticks): " + "  ".join(
            f"{n} {w[:, i].mean():.0f} ({(w[:, i] / tot).mean() * 100:.1f}%)" for i, n in enumerate(names)), flush=True)
        heavy = w[tot > tot.quantile(0.9)]
        print("DIAG heaviest 10% waves: " + "  ".join(f"{n} {heavy[:, i].mean():.0f}" for i, n in enumerate(names)),
              flush=True)
    if a.diag and a.bwd:
        items = (B * H + 7) // 8 * 8 * (((T + 127) // 128 + 1) // 2)
        d = torch.zeros(items * 4 * 10, dtype=torch.int64, device="cuda")
        C.attn_diag(d)
        C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv, impl=5)
        torch.cuda.synchronize()
        C.attn_diag(torch.empty(0))
        w = d.view(-1, 10).double()
        w = w[w[:, 9] > 0]
        life = w[:, 9] - w[:, 8]
        names = ["wait+barrier", "S,dP+exp0", "exp1+mask+dS+pack", "dO^T+dV", "Q^T+dK", "epilogue", "prologue"]
        nt = w[:, 7]
        print(f"DIAG dK/dV: {w.shape[0]} waves, wave life mean {life.mean():.0f} ticks, tiles per wave "
              f"{nt.mean():.2f}, per tile: " + "  ".join(f"{n} {(w[:, i] / nt).mean():.0f}" for i, n in
                                                        enumerate(names[:5])), flush=True)
        print("DIAG dK/dV per wave (ticks, share of life): " + "  ".join(
            f"{n} {w[:, i].mean():.0f} ({(w[:, i] / life).mean() * 100:.1f}%)" for i, n in enumerate(names)),
            flush=True)
    if a.ab and not a.bwd:   # a forward build switch, interleaved, bitwise check
        sw = getattr(C, a.ab)

        def mkf(x):
            def g():
                sw(x)
                return C.attn_fwd(q, k, v, scale, True, impl=4)
            return g
        o0, l0 = mkf(a.ab_vals[0])()
        for x in a.ab_vals[1:]:
            o1, l1 = mkf(x)()
            print(f"{a.ab} {x} vs {a.ab_vals[0]} bitwise equal: {torch.equal(o0, o1) and torch.equal(l0, l1)}", flush=True)
        r = timeit({f"{a.ab}={x}": mkf(x) for x in a.ab_vals}, iters=a.iters, rounds=7)
        for kk, ms in r.items():
            print(f"fwd {kk}: {ms:.4f} ms {fl / ms / 1e9:.1f} TF", flush=True)
        sw(a.ab_vals[0])
    if a.ab and a.bwd:   # a dK/dV v3 build switch (C.<name>(0 / 1)), interleaved, bitwise check
        sw = getattr(C, a.ab)

        def mkab(x):
            def g():
                sw(x)
                C.attn_bwd(do, q, k, v, o, lse, scale, True, dq, dk, dv, impl=4)
            return g
        vals = a.ab_vals
        mkab(vals[0])()
        ref = [t.clone() for t in (dq, dk, dv)]
        for x in vals[1:]:
            mkab(x)()
            print(f"{a.ab} {x} vs {vals[0]} bitwise equal: " +
                  str(all(torch.equal(u, w) for u, w in zip(ref, (dq, dk, dv)))), flush=True)
        r = timeit({f"{a.ab}={x}": mkab(x) for x in vals}, iters=a.iters, rounds=7)
        for kk, ms in r.items():
            print(f"bwd {kk}: {ms:.4f} ms {fl / ms / 1e9:.1f} TF", flush=True)
        sw(a.ab_vals[0])
    res = timeit({impl: mk(impl) for impl in a.impl}, iters=a.iters, rounds=5)  # interleaved, median
    for impl, ms in res.items():
        print(f"impl {impl} {'bwd' if a.bwd else 'fwd'}: {ms:.4f} ms {fl / ms / 1e9:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
