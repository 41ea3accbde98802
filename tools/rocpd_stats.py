"""Kernel statistics (rocprofv3 --stats layout: Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs) from a rocprofv3 rocpd SQLite database (the default output format of
rocprofv3 on ROCm 7 when --output-format is not given)."""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--out", default="-")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                          "max(end - start) from kernels group by name order by sum(end - start) desc"))
    total = sum(r[2] for r in rows) or 1
    f = sys.stdout if a.out == "-" else open(a.out, "w", newline="")
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, calls, tot, avg, mn, mx in rows:
        w.writerow([name, calls, tot, round(avg, 3), round(100.0 * tot / total, 2), mn, mx])


if __name__ == "__main__":
    main()
