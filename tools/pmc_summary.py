"""Average rocprofv3 PMC counters per kernel over dispatches: python tools/pmc_summary.py gpurun_out/pmc"""
import collections
import csv
import glob
import os
import sys


def derived(c):
    """MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), and the
    instruction mix per MFMA (VALU excludes the MFMAs themselves)."""
    out = []
    g, m = c.get("GRBM_GUI_ACTIVE"), c.get("SQ_INSTS_MFMA")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        out.append(f"MFMA busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g / 8) * 100:5.1f}%")
    if m:
        if "SQ_INSTS_SALU" in c:
            out.append(f"SALU/MFMA {c['SQ_INSTS_SALU'] / m:.2f}")
        if "SQ_INSTS_VALU" in c:
            out.append(f"VALU(non-MFMA)/MFMA {(c['SQ_INSTS_VALU'] - m) / m:.2f}")
        if "SQ_INSTS_LDS" in c:
            out.append(f"LDS/MFMA {c['SQ_INSTS_LDS'] / m:.3f}")
    return "  ".join(out)


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
        avg = {c: x / len(disp[k][c]) for c, x in v.items()}
        print(f"{k:60s} {derived(avg)}")
        for c, x in sorted(avg.items()):
            print(f"   {c:40s} {x:16.0f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
