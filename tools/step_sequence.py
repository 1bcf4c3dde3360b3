"""Dispatch sequence of one training step from a rocprofv3 rocpd database: every kernel of the
step in launch order with its duration and grid, so per-call times map onto the step's GEMM
shapes / layers (the kernel-name summary of tools/prof_summary.py cannot tell the QKV from the
down projection when they share a template instance).

    python tools/step_sequence.py gpurun_out/p_x/run_results.db --after adam_k --skip 5 [--steps 1]
"""
from __future__ import annotations

import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after", default="adam_k")
    ap.add_argument("--skip", type=int, default=5)
    ap.add_argument("--steps", type=int, default=1, help="number of steps to list (each ends at an adam_k)")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [d[1] for d in con.execute("pragma table_info(kernels)")]
    grid = [c for c in cols if re.fullmatch(r"grid_size(_[xyz])?", c)]
    wg = [c for c in cols if re.fullmatch(r"workgroup_size(_[xyz])?", c)]
    sel = ", ".join(["name", "start", "end"] + grid + wg)
    recs = list(con.execute(f"select {sel} from kernels order by start"))
    marks = [i for i, r in enumerate(recs) if a.after in r[0]]
    i0 = marks[a.skip - 1] + 1
    i1 = marks[a.skip - 1 + a.steps] + 1
    print(f"# columns: grid {grid} workgroup {wg}")
    t_prev = None
    for i, r in enumerate(recs[i0:i1]):
        name = re.sub(r"\(.*\)$", "", r[0])
        name = re.sub(r"^void ", "", name)
        name = re.sub(r"dpfs::(g4::)?", "", name)
        gap = (r[1] - t_prev) / 1e3 if t_prev is not None else 0.0
        t_prev = r[2]
        print(f"{i:4d} {(r[2] - r[1]) / 1e3:9.1f} us  gap {gap:7.1f}  grid {tuple(r[3:3 + len(grid)])} "
              f"wg {tuple(r[3 + len(grid):])}  {name[:110]}")


if __name__ == "__main__":
    main()
