"""Longest host API calls in a rocprofv3 trace (``--hip-trace`` rocpd SQLite ``*_results.db``).

    python tools/api_blocking.py gpurun_out/prof/run_results.db [--top 25] [--last-ms 200]

Prints the views in the database, then the longest HIP runtime calls in the last ``--last-ms``
of the trace: a call that blocks the host (synchronous copy, device sync, hipMalloc / hipFree
on a busy device) is where the GPU runs dry.
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--last-ms", type=float, default=200.0)
    a = ap.parse_args()
    con = sqlite3.connect(a.path)
    names = [r[0] for r in con.execute("select name from sqlite_master where type in ('view','table')")]
    print("views:", [n for n in names if not n.startswith("rocpd_")][:40])
    view = "regions" if "regions" in names else None
    if view is None:
        print("no regions view")
        return
    cols = [r[1] for r in con.execute(f"pragma table_info({view})")]
    print("columns:", cols)
    s, e = ("start", "end") if "start" in cols else ("start_ns", "end_ns")
    t_end = con.execute(f"select max({e}) from {view}").fetchone()[0]
    lo = t_end - a.last_ms * 1e6
    rows = con.execute(f"select name, {s}, {e} from {view} where {e} > ? order by ({e} - {s}) desc limit ?",
                       (lo, a.top)).fetchall()
    for name, st, en in rows:
        print(f"{(en - st) / 1e3:10.1f} us  at {(st - lo) / 1e6:8.2f} ms  {name}")
    agg = con.execute(f"select name, count(*), sum({e} - {s}) from {view} where {e} > ? group by name "
                      f"order by sum({e} - {s}) desc limit 15", (lo,)).fetchall()
    print("-- totals in window --")
    for name, n, tot in agg:
        print(f"{tot / 1e6:9.2f} ms {n:7d} calls  {name}")


if __name__ == "__main__":
    main()
