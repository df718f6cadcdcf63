"""Clock and MFMA-pipe occupancy per dispatch from rocprofv3 --pmc counter CSVs (which carry each dispatch's start /
end timestamps): effective clock = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs) / duration
(MI355X_MICROARCH.md 'DVFS give-back'), and MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs against the cycles of
that clock (and against 2.4 GHz, the figure that ignores the clock the chip holds under load).

Usage: python tools/clock_pmc.py <dir with *counter_collection.csv (searched recursively)> <kernel name pattern>"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    root, pat = sys.argv[1], sys.argv[2]
    rows = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat not in r.get("Kernel_Name", ""):
                continue
            key = (f, r["Dispatch_Id"])
            d = rows[key]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    print(f"\n{pat} ({root}): {len(rows)} dispatches\n")
    print("| dispatch | us | clock GHz | MFMA busy at that clock | MFMA busy at 2.4 GHz |")
    print("|---|---|---|---|---|")
    clks, busy = [], []
    for (f, did), d in sorted(rows.items(), key=lambda kv: int(kv[0][1])):
        if "GRBM_GUI_ACTIVE" not in d or d["ns"] <= 0:
            continue
        ghz = d["GRBM_GUI_ACTIVE"] / 8 / d["ns"]
        mf = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024
        b_clk = mf / (d["ns"] * ghz) if ghz > 0 else 0.0
        b_24 = mf / (d["ns"] * 2.4)
        clks.append(ghz)
        busy.append(b_clk)
        print(f"| {did} | {d['ns'] / 1e3:.1f} | {ghz:.3f} | {b_clk:.3f} | {b_24:.3f} |")
    if clks:
        print(f"\nmedian clock {statistics.median(clks):.3f} GHz, median MFMA busy at that clock "
              f"{statistics.median(busy):.3f}")


if __name__ == "__main__":
    main()
