#!/usr/bin/env python3
"""rocprofv3 SQLite output (*_results.db) -> the --stats kernel summary as CSV.

usage: python scripts/prof_db_stats.py <results.db> [out.csv]
Columns follow rocprofv3's kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs).
"""
import csv
import sqlite3
import sys


def main(db, out=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                     "max(end - start) from kernels group by name order by sum(end - start) desc"
                     ).fetchall()
    tot = sum(r[2] for r in rows) or 1
    f = open(out, "w", newline="") if out else sys.stdout
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, calls, total, avg, mn, mx in rows:
        w.writerow([name, calls, total, round(avg, 1), round(100.0 * total / tot, 2), mn, mx])


if __name__ == "__main__":
    main(*sys.argv[1:3])
