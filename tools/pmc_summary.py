"""Average rocprofv3 PMC counters per kernel over dispatches: python tools/pmc_summary.py gpurun_out/pmc"""
import collections
import csv
import glob
import os
import sys


def main(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    for k, v in agg.items():
        if not any(x in k for x in ("dpfs", "gemm", "attn", "Cijk")):
            continue
        print(k)
        for c, x in sorted(v.items()):
            print(f"   {c:40s} {x / len(disp[k][c]):16.0f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
