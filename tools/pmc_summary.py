"""Summarise rocprofv3 --pmc CSVs (one sub-directory per counter set) per GEMM kernel.

Usage: python tools/pmc_summary.py gpurun_out/pmc3 [--match gemm_]
Counters are summed over dispatches of the same kernel and template signature (shape groups are kept
apart by grid size); derived ratios: wait share of wave cycles, MFMA busy per SIMD vs GRBM_GUI_ACTIVE/XCD.
"""
import argparse
import collections
import csv
import glob
import os
import re


def short(name):
    m = re.search(r"(gemm_\w+?)<(.*?)>\(", name) or re.search(r"(\w+)", name)
    return m.group(0)[:70] if m else name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="gemm")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    ndisp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(a.dir, "*", "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if a.match not in r["Kernel_Name"] and "Cijk" not in r["Kernel_Name"]:
                    continue
                key = (short(r["Kernel_Name"]), r["Grid_Size"])
                tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
                ndisp[key].add((f, r["Dispatch_Id"]))
    for key, c in sorted(tot.items()):
        wc = c.get("SQ_WAVE_CYCLES", 0)
        print(f"{key[0]}  grid={key[1]}")
        for k in sorted(c):
            print(f"    {k:28s} {c[k]:.4g}")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in c:
                    print(f"    {k + ' / WAVE_CYCLES':28s} {c[k] / wc:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            # MFMA busy is summed over SIMDs (1024); GRBM_GUI_ACTIVE over 8 XCDs
            print(f"    {'MFMA busy per SIMD':28s} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (c['GRBM_GUI_ACTIVE'] / 8):.3f}")


if __name__ == "__main__":
    main()
