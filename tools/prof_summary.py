"""rocprofv3 kernel statistics -> markdown table (profiles/*.md).

Usage: python tools/prof_summary.py <run_kernel_stats.csv | run_results.db> "title" [note]
Accepts the CSV of ``--stats --output-format csv`` or the rocpd SQLite database rocprofv3 writes by default."""
import csv
import sqlite3
import sys


def rows_of(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        out = []
        for name, calls, tot, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            # the rocpd top_kernels view reports microseconds
            out.append({"Name": name, "Calls": calls, "TotalDurationNs": 1e3 * tot, "AverageNs": 1e3 * avg,
                        "Percentage": pct})
        return out
    return list(csv.DictReader(open(path)))


def main():
    path, title = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = rows_of(path)
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
