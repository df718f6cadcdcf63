"""rocprofv3 --kernel-trace --stats CSV -> markdown table (profiles/*.md).

Usage: python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv "title" [note]"""
import csv
import sys


def main():
    path, title = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    if note:
        print(note + "\n")
    print(f"Total kernel time {tot / 1e6:.2f} ms.\n")
    print("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        name = r["Name"].replace("|", "/")
        name = name if len(name) <= 90 else name[:87] + "..."
        print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main()
