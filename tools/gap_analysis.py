"""Idle gaps on the GPU timeline of a rocprofv3 kernel trace (rocpd SQLite ``*_results.db``).

    python tools/gap_analysis.py gpurun_out/prof/run_results.db [--last-ms 200] [--top 15]

Over the last ``--last-ms`` of the trace: span, busy time (union of kernel intervals, so
concurrent streams are not double counted), idle time, and the largest gaps with the kernels
on either side — where a step waits on the host, a sync or an allocation instead of the GPU.
"""
from __future__ import annotations

import argparse
import re
import sqlite3


def _short(name: str, width: int = 60) -> str:
    name = re.sub(r"\(.*\)$", "", name)
    return name if len(name) <= width else name[: width - 3] + "..."


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last-ms", type=float, default=200.0)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--host", action="store_true", help="trace has --hip-trace regions: explain gaps")
    a = ap.parse_args(argv)
    con = sqlite3.connect(a.path)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    k0 = "start" if "start" in cols else "start_ns"
    k1 = "end" if "end" in cols else "end_ns"
    rows = sorted(con.execute(f"select {k0}, {k1}, name from kernels"))
    if not rows:
        print("no kernels")
        return
    t_end = max(r[1] for r in rows)
    t_lo = t_end - a.last_ms * 1e6
    rows = [r for r in rows if r[1] > t_lo]
    span = (t_end - max(t_lo, rows[0][0])) / 1e6
    busy, gaps = 0.0, []
    cur_s, cur_e, prev_name = rows[0][0], rows[0][1], rows[0][2]
    for s, e, n in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(((s - cur_e) / 1e3, prev_name, n))
            cur_s, cur_e = s, e
        elif e > cur_e:
            cur_e = e
        prev_name = n if e >= cur_e else prev_name
    busy += cur_e - cur_s
    busy /= 1e6
    idle = sum(g[0] for g in gaps) / 1e3
    print(f"window {span:.2f} ms: busy {busy:.2f} ms, idle {idle:.2f} ms ({100 * idle / span:.1f} %), "
          f"{len(gaps)} gaps")
    small = sum(g[0] for g in gaps if g[0] < 20) / 1e3
    print(f"gaps < 20 us: {small:.2f} ms total (launch seams); larger: {idle - small:.2f} ms")
    for us, before, after in sorted(gaps, reverse=True)[: a.top]:
        print(f"{us:9.1f} us  after {_short(before)}  ->  {_short(after)}")
    if a.host:
        host_view(a.path, a.last_ms)



def host_view(path: str, last_ms: float = 150.0, top: int = 6):
    """For the largest gaps of a trace that also holds ``--hip-trace`` regions: when the host
    issued the kernel that ended each gap, and the host calls in the 1.5 ms before it."""
    con = sqlite3.connect(path)
    kcols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    if "corr_id" not in kcols:
        print("kernels view has no corr_id")
        return
    rows = sorted(con.execute("select start, end, name, corr_id from kernels"))
    t_end = max(r[1] for r in rows)
    rows = [r for r in rows if r[1] > t_end - last_ms * 1e6]
    gaps, cur_e = [], rows[0][1]
    for i in range(1, len(rows)):
        if rows[i][0] > cur_e:
            gaps.append((rows[i][0] - cur_e, i))
        cur_e = max(cur_e, rows[i][1])
    for g, i in sorted(gaps, reverse=True)[:top]:
        s, e, name, corr = rows[i]
        launch = con.execute("select name, start, end from regions where corr_id = ?", (corr,)).fetchone()
        print(f"--- gap {g / 1e3:.1f} us before {_short(name)}")
        if launch:
            print(f"    launched by {launch[0]} at {(launch[1] - s) / 1e3:+.1f} us vs kernel start")
            prev = con.execute("select name, start, end from regions where start < ? and start > ? "
                               "order by start", (launch[1], launch[1] - 1.5e6)).fetchall()
            for n, ps, pe in prev[-12:]:
                print(f"      {(ps - launch[1]) / 1e3:+9.1f} us  {(pe - ps) / 1e3:8.1f} us  {n}")


if __name__ == "__main__":
    main()
