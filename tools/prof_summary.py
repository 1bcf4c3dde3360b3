"""Summarise a rocprofv3 kernel trace (rocpd SQLite ``*_results.db`` or ``*kernel_stats.csv``).

    python tools/prof_summary.py gpurun_out/prof4/run_results.db [--steps 8] [--top 40] [--csv out.csv]

Groups dispatches by kernel name (template arguments shortened), prints total / per-step time,
call counts and share of GPU time.  ``--steps`` divides totals by the number of training steps
the profiled run executed (warmup + timed) to give ms/step per kernel.
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


def load(path: str):
    rows = defaultdict(lambda: [0.0, 0])
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        for name, dur in con.execute("select name, duration from kernels"):
            r = rows[_short(name)]
            r[0] += dur / 1e6
            r[1] += 1
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


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default=None)
    a = ap.parse_args(argv)
    rows = load(a.path)
    tot = sum(v[0] for v in rows.values())
    items = sorted(rows.items(), key=lambda kv: -kv[1][0])
    print(f"total GPU kernel time {tot:.2f} ms over {a.steps} step(s) = {tot / a.steps:.2f} ms/step")
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
