"""Per-kernel summary (calls, avg / total µs) from a rocprofv3 results database.

    python tools/prof_summary.py gpurun_out/prof/run_results.db [--csv out.csv] [--top 40]
"""
import argparse
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, count(*), avg(duration), sum(duration), min(duration), max(duration) "
                          "from kernels group by name order by 4 desc"))
    total = sum(r[3] for r in rows)
    for r in rows[:a.top]:
        print(f"{r[1]:6d} {r[2] / 1e3:9.2f} {r[3] / 1e3:10.1f}  {r[0][:100]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for r in rows:
                w.writerow([r[0], r[1], r[3], r[2], round(100.0 * r[3] / total, 4), r[4], r[5]])


if __name__ == "__main__":
    main()
