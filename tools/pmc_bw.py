"""HBM bytes per kernel from a FETCH_SIZE / WRITE_SIZE rocprofv3 pass (tools/pmc_run.sh with
PMC_SETS="FETCH_SIZE;WRITE_SIZE"): per kernel name, dispatches, MB fetched / written per call
(FETCH_SIZE and WRITE_SIZE are KiB), mean duration under the counter pass and the implied TB/s.

    python tools/pmc_bw.py gpurun_out/pmc_bw [--top 25] [--after adam_k --skip 1]
"""
import argparse
import collections
import csv
import os
import re


def load(path, counter, after=None, skip=0):
    """Per kernel [KiB, calls, ns]; with ``after`` only dispatches that follow the ``skip``-th
    dispatch whose name contains it (e.g. the steps after the first Adam: selection timing
    and warmup excluded)."""
    per = collections.defaultdict(lambda: [0.0, 0, 0.0])   # name -> [KiB, calls, ns]
    rows = sorted((r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter),
                  key=lambda r: int(r["Dispatch_Id"]))
    if after:
        seen, start = 0, len(rows)
        for i, r in enumerate(rows):
            if after in r["Kernel_Name"]:
                seen += 1
                if seen == skip:
                    start = i + 1
                    break
        rows = rows[start:]
    for r in rows:
        name = re.sub(r"\(.*\)$", "", r["Kernel_Name"])[:80]
        e = per[name]
        e[0] += float(r["Counter_Value"])
        e[1] += 1
        e[2] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--after", default="adam_k")
    ap.add_argument("--skip", type=int, default=1)
    a = ap.parse_args()
    f = load(os.path.join(a.root, "FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE", a.after, a.skip)
    w = load(os.path.join(a.root, "WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE", a.after, a.skip)
    rows = []
    for name, (kib, n, ns) in f.items():
        wk = w.get(name, [0.0, 1, 0.0])
        fmb, wmb = kib / n / 1024, wk[0] / max(wk[1], 1) / 1024
        us = ns / n / 1000
        rows.append((ns, name, n, fmb, wmb, us, (fmb + wmb) / 1e6 / (us / 1e6) if us else 0.0))
    print(f"{'calls':>6} {'MB rd/call':>11} {'MB wr/call':>11} {'us/call':>9} {'TB/s':>6}  kernel")
    for ns, name, n, fmb, wmb, us, tbs in sorted(rows, reverse=True)[: a.top]:
        print(f"{n:6d} {fmb:11.1f} {wmb:11.1f} {us:9.1f} {tbs:6.2f}  {name}")


if __name__ == "__main__":
    main()
