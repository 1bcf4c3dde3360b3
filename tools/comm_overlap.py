"""Overlap of the (emulated) TP collectives with compute in a rocprofv3 kernel trace of
``tools/tp_sim.py --emulate-comm`` (rocpd ``*_results.db``): per step, the union of the
collective stand-ins' intervals (``occupy_k``), of the compute kernels' intervals, their
overlap, the time only a collective runs (compute waiting on it) split into the forward / the
backward (at the cross-entropy kernel), and the longest such stretches with their neighbours.

    python tools/comm_overlap.py run_results.db [--skip 2] [--steps 3]
"""
from __future__ import annotations

import argparse
import re
import sqlite3


def _union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _len(iv):
    return sum(e - s for s, e in iv)


def _minus(a, b):
    """intervals of a not covered by b (both unions)"""
    out, j = [], 0
    for s, e in a:
        cur = s
        while j < len(b) and b[j][1] <= cur:
            j += 1
        k = j
        while k < len(b) and b[k][0] < e:
            if b[k][0] > cur:
                out.append([cur, b[k][0]])
            cur = max(cur, b[k][1])
            k += 1
        if cur < e:
            out.append([cur, e])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--skip", type=int, default=2, help="Adam launches to skip (warmup steps)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    con = sqlite3.connect(a.path)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    k0 = "start" if "start" in cols else "start_ns"
    k1 = "end" if "end" in cols else "end_ns"
    rows = sorted(con.execute(f"select {k0}, {k1}, name from kernels"))
    adam = [r for r in rows if "adam_k" in r[2]]
    if len(adam) < a.skip + a.steps:
        print(f"only {len(adam)} Adam launches")
        return
    tot = {"step": 0, "comm": 0, "comp": 0, "comm_only_fwd": 0, "comm_only_bwd": 0, "idle": 0}
    stretches = []
    for si in range(a.steps):
        t0, t1 = adam[a.skip + si - 1][1] if a.skip + si > 0 else rows[0][0], adam[a.skip + si][1]
        win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
        comm = _union([[s, e] for s, e, n in win if "occupy_k" in n])
        comp = _union([[s, e] for s, e, n in win if "occupy_k" not in n])
        ce = [s for s, e, n in win if "ce_stats" in n or "ce_fused" in n]
        t_ce = min(ce) if ce else t1
        only = _minus(comm, comp)
        idle = _minus(_minus([[t0, t1]], comp), comm)
        tot["step"] += t1 - t0
        tot["comm"] += _len(comm)
        tot["comp"] += _len(comp)
        tot["idle"] += _len(idle)
        tot["comm_only_fwd"] += sum(min(e, t_ce) - s for s, e in only if s < t_ce)
        tot["comm_only_bwd"] += sum(e - max(s, t_ce) for s, e in only if e > t_ce)
        for s, e in only:
            before = max((r for r in win if r[1] <= s and "occupy_k" not in r[2]), key=lambda r: r[1], default=None)
            after = min((r for r in win if r[0] >= e and "occupy_k" not in r[2]), key=lambda r: r[0], default=None)
            stretches.append((e - s, "fwd" if s < t_ce else "bwd", before[2] if before else "-", after[2] if after else "-"))
    n = a.steps
    print(f"per step (mean of {n}): step {tot['step'] / n / 1e6:.2f} ms; compute busy {tot['comp'] / n / 1e6:.2f} ms; "
          f"collectives busy {tot['comm'] / n / 1e6:.2f} ms; collective-only (compute waiting) forward "
          f"{tot['comm_only_fwd'] / n / 1e6:.2f} ms, backward {tot['comm_only_bwd'] / n / 1e6:.2f} ms; idle {tot['idle'] / n / 1e6:.2f} ms")
    short = lambda x: re.sub(r"\(.*$", "", x)[:60]
    print("longest collective-only stretches:")
    for d, ph, b, af in sorted(stretches, reverse=True)[: a.top]:
        print(f"  {d / 1e3:8.1f} us  {ph}  after {short(b)}  ->  {short(af)}")


if __name__ == "__main__":
    main()
