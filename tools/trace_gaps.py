"""Idle time between kernels in a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

Usage: python tools/trace_gaps.py <run_kernel_trace.csv> [--max-gap-us 500] [--top 25]

Sorts the dispatches by start time, merges overlapping ones and reports, for the stretches of back-to-back GPU work
(gaps shorter than --max-gap-us: longer ones are host synchronisation / Python between steps, excluded), the busy time
(union of kernel intervals), the idle time between kernels and the kernel pairs (previous -> next) that the idle time
falls between.  This is the launch / dependency overhead of a graph-replayed step that the per-kernel statistics do
not show."""
import argparse
import collections
import csv


def short(name: str, n: int = 60) -> str:
    name = name.split("(")[0]
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--max-gap-us", type=float, default=500.0)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--last-ms", type=float, default=0.0, help="only the dispatches of the trace's last N ms")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if args.last_ms > 0:
        t_end = max(e for _, e, _ in ev)
        ev = [x for x in ev if x[0] >= t_end - args.last_ms * 1e6]
    busy = idle = 0
    span0 = None
    pairs = collections.Counter()
    pair_n = collections.Counter()
    cur_end, cur_name = None, None
    for s, e, name in ev:
        if cur_end is None:
            cur_end, cur_name, span0 = e, name, s
            busy += e - s
            continue
        gap = s - cur_end
        if gap > args.max_gap_us * 1e3:
            cur_end, cur_name = e, name
            busy += e - s
            continue
        if gap > 0:
            idle += gap
            key = (short(cur_name), short(name))
            pairs[key] += gap
            pair_n[key] += 1
            busy += e - s
        else:
            busy += max(0, e - cur_end)
        if e > cur_end:
            cur_end, cur_name = e, name
    tot = busy + idle
    print(f"dispatches {len(ev)}; busy {busy / 1e6:.3f} ms, idle between kernels {idle / 1e6:.3f} ms "
          f"({100.0 * idle / max(tot, 1):.2f} % of {tot / 1e6:.3f} ms back-to-back GPU time)")
    print(f"\n| previous kernel | next kernel | gaps | total us | avg us |\n|---|---|---|---|---|")
    for (a, b), g in pairs.most_common(args.top):
        print(f"| `{a}` | `{b}` | {pair_n[(a, b)]} | {g / 1e3:.1f} | {g / 1e3 / pair_n[(a, b)]:.2f} |")


if __name__ == "__main__":
    main()
