"""Summarise a rocprofv3 run (kernel-trace .db or kernel_stats.csv) into a markdown table.

usage: python tools/prof_summary.py <rocprof output dir> [steps]  > profiles/<name>.md
"""
import csv
import glob
import os
import sqlite3
import sys


def rows_from_db(path):
    con = sqlite3.connect(path)
    return con.execute("select name, count(*), avg(end-start), sum(end-start), min(end-start), max(end-start) "
                       "from kernels group by name order by sum(end-start) desc").fetchall()


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["AverageNs"]), float(r["TotalDurationNs"]),
                        float(r["MinNs"]), float(r["MaxNs"])))
    return sorted(out, key=lambda r: -r[3])


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    rows = rows_from_csv(csvs[0]) if csvs else rows_from_db(dbs[0])
    tot = sum(r[3] for r in rows)
    print(f"source: {os.path.relpath(csvs[0] if csvs else dbs[0])}\n")
    print("| kernel | calls | avg us | min us | max us | total ms | % |" + (" per step us |" if steps else ""))
    print("|---|---|---|---|---|---|---|" + ("---|" if steps else ""))
    for n, c, a, s, mn, mx in rows[:30]:
        name = n.replace("|", "/")[:90]
        extra = f" {s / 1e3 / steps:.1f} |" if steps else ""
        print(f"| `{name}` | {c} | {a / 1e3:.2f} | {mn / 1e3:.2f} | {mx / 1e3:.2f} | {s / 1e6:.3f} | {100 * s / tot:.1f} |{extra}")


if __name__ == "__main__":
    main()
