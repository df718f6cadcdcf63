"""Per-op summary of rocprofv3 --pmc passes over tools/kernel_probe.py (scripts/gpu_pmc_r03s.sh layout:
<dir>/p<pass>_<op>/.../*counter_collection.csv): each counter averaged per dispatch of the op's kernel, plus
the derived wait share of wave cycles, VALU instructions per MFMA and MFMA-busy cycles per SIMD and active cycle.

Usage: python tools/pmc_ops.py gpurun_out/pmc_r03s"""
import collections
import csv
import glob
import os
import sys

KERNELS = {"attn": "flash_attn_fwd_x6", "qkv": "gemm_4w_kernel<14", "norm": "rmsnorm_f32", "colsum": "attn_colsum_h3",
           "gateup": "gemm_4w_kernel<13", "down": "gemm_4w_kernel<10"}


def main():
    root = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sorted(glob.glob(os.path.join(root, "p*_*"))):
        if not os.path.isdir(d):
            continue
        op = os.path.basename(d).split("_", 1)[1]
        pat = KERNELS.get(op, op)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pat not in r.get("Kernel_Name", ""):
                    continue
                per[op][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[(op, os.path.basename(d))].add(r.get("Dispatch_Id", ""))
    print("| op | counter | per dispatch |\n|---|---|---|")
    for op, cs in per.items():
        n = max(len(v) for k, v in disp.items() if k[0] == op)
        avg = {k: v / max(n, 1) for k, v in cs.items()}
        for k in sorted(avg):
            print(f"| {op} | {k} | {avg[k]:.4g} |")
        if avg.get("SQ_WAVE_CYCLES"):
            print(f"| {op} | wait_any / wave_cycles | {avg.get('SQ_WAIT_ANY', 0) / avg['SQ_WAVE_CYCLES']:.3f} |")
        if avg.get("SQ_INSTS_MFMA"):
            print(f"| {op} | VALU per MFMA | {avg.get('SQ_INSTS_VALU', 0) / avg['SQ_INSTS_MFMA']:.2f} |")
        if avg.get("GRBM_GUI_ACTIVE") and avg.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs
            print(f"| {op} | MFMA busy per SIMD cycle | "
                  f"{avg['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (avg['GRBM_GUI_ACTIVE'] / 8):.3f} |")


if __name__ == "__main__":
    main()
