#!/usr/bin/env python3
"""rocprofv3 rocpd database (results.db) -> kernel stats CSV (name, calls, total_us, avg_us, pct),
the same columns as rocprofv3's --stats kernel_stats.csv.  Usage: rocpd_stats.py DB [OUT.csv]"""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = list(db.execute("select name, total_calls, total_duration, average, percentage "
                           "from top_kernels order by total_duration desc"))
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], "%.3f" % r[2], "%.3f" % r[3], "%.3f" % r[4]])


if __name__ == "__main__":
    main()
