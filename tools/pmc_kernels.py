"""Per-kernel summary of rocprofv3 --pmc passes over one program (directories <root>/p<pass>/.../
*counter_collection.csv): each counter averaged per dispatch of every kernel whose name contains one of the given
patterns, plus the derived wait share of wave cycles, VALU instructions per MFMA, LDS bank-conflict cycles per LDS
cycle and MFMA-busy cycles per SIMD and active cycle (1024 SIMDs).

Usage: python tools/pmc_kernels.py <root> <pattern> [<pattern> ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    root, pats = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in sorted(glob.glob(os.path.join(root, "p*"))):
        if not os.path.isdir(d):
            continue
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                for p in pats:
                    if p in name:
                        per[p][r["Counter_Name"]] += float(r["Counter_Value"])
                        disp[p][os.path.basename(d)].add(r.get("Dispatch_Id", ""))
    print("| kernel | counter | per dispatch |\n|---|---|---|")
    for p in pats:
        if p not in per:
            continue
        n = max(len(v) for v in disp[p].values())
        avg = {k: v / max(n, 1) for k, v in per[p].items()}
        for k in sorted(avg):
            print(f"| {p} | {k} | {avg[k]:.4g} |")
        if avg.get("SQ_WAVE_CYCLES"):
            print(f"| {p} | wait_any / wave_cycles | {avg.get('SQ_WAIT_ANY', 0) / avg['SQ_WAVE_CYCLES']:.3f} |")
        if avg.get("SQ_INSTS_MFMA"):
            print(f"| {p} | VALU per MFMA | {avg.get('SQ_INSTS_VALU', 0) / avg['SQ_INSTS_MFMA']:.2f} |")
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            print(f"| {p} | LDS bank-conflict cycles / LDS cycles | "
                  f"{avg.get('SQ_LDS_BANK_CONFLICT', 0) / avg['SQ_LDS_IDX_ACTIVE']:.3f} |")
        if avg.get("GRBM_GUI_ACTIVE") and avg.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            print(f"| {p} | MFMA busy per SIMD cycle | "
                  f"{avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] * 1024):.3f} |")


if __name__ == "__main__":
    main()
