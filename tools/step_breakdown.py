#!/usr/bin/env python
"""Per-kernel time of the steady-state bench step from rocprofv3 kernel traces (``--kernel-trace`` CSV): the last
``--mb`` micro-batches before the final one (delimited by the LM-head LSE GEMM, one per micro-batch), per kernel family
per micro-batch, for one or more traces side by side (e.g. an A/B pair from one box).

Usage: ``python tools/step_breakdown.py a/run_kernel_trace.csv [b/run_kernel_trace.csv ...] [--mb 8]``."""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def family(name: str) -> str:
    n = name.split("(")[0].replace("void ", "")
    return n[:60]


def breakdown(path: str, mb: int) -> tuple[dict, dict, float, float]:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    lse = [i for i, r in enumerate(rows) if "gemm_4w_kernel<15" in r["Kernel_Name"]]
    a, b = lse[-mb - 1], lse[-1]
    t, n = defaultdict(float), defaultdict(int)
    for r in rows[a + 1:b + 1]:
        f = family(r["Kernel_Name"])
        t[f] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / mb
        n[f] += 1
    span = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3 / mb
    return t, n, sum(t.values()), span


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--mb", type=int, default=8)
    a = ap.parse_args()
    res = [breakdown(p, a.mb) for p in a.traces]
    fams = sorted({f for t, _, _, _ in res for f in t}, key=lambda f: -max(r[0].get(f, 0.0) for r in res))
    print(f"# Steady-state step per micro-batch (last {a.mb} micro-batches), us\n")
    print("| kernel | " + " | ".join(f"{p} (calls/mb)" for p in a.traces) + " |")
    print("|---|" + "---|" * len(res))
    for f in fams:
        if max(r[0].get(f, 0.0) for r in res) < 5.0:
            continue
        print(f"| `{f}` | " + " | ".join(f"{r[0].get(f, 0.0):.1f} ({r[1].get(f, 0) / a.mb:g})" for r in res) + " |")
    print("| **kernels** | " + " | ".join(f"**{r[2]:.1f}**" for r in res) + " |")
    print("| **wall (LSE to LSE)** | " + " | ".join(f"**{r[3]:.1f}**" for r in res) + " |")


if __name__ == "__main__":
    main()
