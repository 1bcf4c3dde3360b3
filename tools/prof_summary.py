"""Summarise a rocprofv3 kernel trace (rocpd SQLite ``*_results.db`` or ``*kernel_stats.csv``).

    python tools/prof_summary.py gpurun_out/prof4/run_results.db [--steps 8] [--top 40] [--csv out.csv]

Groups dispatches by kernel name (template arguments shortened), prints total / per-step time,
call counts and share of GPU time.  ``--steps`` divides totals by the number of training steps
the profiled run executed (warmup + timed) to give ms/step per kernel.  ``--after adam_k
--skip 5`` (rocpd database only) keeps the dispatches that start after the 5th dispatch whose
name contains ``adam_k`` -- i.e. the timed steps of ``bench.py --warmup 5`` -- and also
reports the first-to-last dispatch span.
"""
from __future__ import annotations

import argparse
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def _short(name: str, width: int = 90) -> str:
    name = re.sub(r"\(.*\)$", "", name)          # drop the parameter list
    name = re.sub(r"\s+", " ", name)
    return name if len(name) <= width else name[: width - 3] + "..."


def load(path: str, after: str = None, skip: int = 0, span=None):
    rows = defaultdict(lambda: [0.0, 0])
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        recs = list(con.execute("select name, start, end from kernels order by start"))
        t0 = None
        if after:
            marks = [st for name, st, _ in recs if after in name]
            if len(marks) < skip:
                raise SystemExit(f"only {len(marks)} dispatches match {after!r} (need {skip})")
            t0 = marks[skip - 1] if skip > 0 else None
        first = last = None
        for name, st, en in recs:
            if t0 is not None and st <= t0:
                continue
            first = st if first is None else first
            last = en if last is None else max(last, en)
            r = rows[_short(name)]
            r[0] += (en - st) / 1e6
            r[1] += 1
        if span is not None and first is not None:
            span.append((last - first) / 1e6)
    else:
        with open(path) as f:
            for rec in csv.DictReader(f):
                if "Kernel_Name" in rec:          # *kernel_trace.csv: one row per dispatch
                    r = rows[_short(rec["Kernel_Name"])]
                    r[0] += (int(rec["End_Timestamp"]) - int(rec["Start_Timestamp"])) / 1e6
                    r[1] += 1
                    continue
                r = rows[_short(rec["Name"])]      # *kernel_stats.csv: one row per kernel
                r[0] += float(rec["TotalDurationNs"]) / 1e6
                r[1] += int(rec["Calls"])
    return rows


def sequence(path: str, pattern: str, step_mark: str = None):
    """The dispatches of the last step (after the last ``step_mark`` dispatch but one) whose name
    contains ``pattern``: order, us, grid columns (whatever the rocpd view calls them)."""
    con = sqlite3.connect(path)
    cur = con.execute("select * from kernels order by start")
    cols = [d[0] for d in cur.description]
    recs = cur.fetchall()
    ix = {c: i for i, c in enumerate(cols)}
    gcols = [c for c in cols if "grid" in c.lower() or "workgroup" in c.lower()]
    marks = [i for i, r in enumerate(recs) if step_mark and step_mark in r[ix["name"]]]
    lo = marks[-2] + 1 if len(marks) >= 2 else 0
    hi = marks[-1] + 1 if marks else len(recs)
    print(f"# last step's dispatches matching {pattern!r} (columns: {', '.join(gcols)})")
    for k, r in enumerate(recs[lo:hi]):
        if pattern in r[ix["name"]]:
            print(f"{k:5d} {(r[ix['end']] - r[ix['start']]) / 1e3:9.1f} us  "
                  + " ".join(str(r[ix[c]]) for c in gcols) + "  " + _short(r[ix["name"]], 70))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--after", default=None, help="keep dispatches after the --skip'th one containing this")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--sequence", default=None, metavar="PATTERN",
                    help="(rocpd database) also list the last step's dispatches whose name contains "
                         "PATTERN, in order, with duration and grid size")
    a = ap.parse_args(argv)
    if a.sequence and a.path.endswith(".db"):
        sequence(a.path, a.sequence, a.after)
    span = []
    rows = load(a.path, a.after, a.skip, span)
    tot = sum(v[0] for v in rows.values())
    items = sorted(rows.items(), key=lambda kv: -kv[1][0])
    print(f"total GPU kernel time {tot:.2f} ms over {a.steps} step(s) = {tot / a.steps:.2f} ms/step")
    if span:
        print(f"first-to-last dispatch {span[0]:.2f} ms = {span[0] / a.steps:.2f} ms/step")
    print(f"{'ms/step':>9} {'calls/step':>10} {'us/call':>9} {'share':>6}  kernel")
    for name, (ms, n) in items[: a.top]:
        print(f"{ms / a.steps:9.3f} {n / a.steps:10.1f} {1e3 * ms / max(1, n):9.1f} {100 * ms / tot:5.1f}%  {name}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "ms_per_step", "calls_per_step", "us_per_call", "share_pct"])
            for name, (ms, n) in items:
                w.writerow([name, f"{ms / a.steps:.4f}", f"{n / a.steps:.2f}", f"{1e3 * ms / max(1, n):.2f}",
                            f"{100 * ms / tot:.2f}"])
    return 0


if __name__ == "__main__":
    sys.exit(main())
