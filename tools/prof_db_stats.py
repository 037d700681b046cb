#!/usr/bin/env python3
"""Kernel statistics CSV from a rocprofv3 results database (`-o run` without a csv format):
    python tools/prof_db_stats.py <run_results.db> > <name>_kernel_stats.csv
Columns follow rocprofv3's kernel_stats.csv: Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs (durations from the kernel dispatch records)."""
import csv
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "SELECT S.display_name, COUNT(*), SUM(K.end - K.start), MIN(K.end - K.start), "
        "MAX(K.end - K.start) FROM rocpd_kernel_dispatch K JOIN rocpd_info_kernel_symbol S "
        "ON S.id = K.kernel_id GROUP BY S.display_name ORDER BY SUM(K.end - K.start) DESC").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, mn, mx in rows:
        w.writerow([name, n, tot, round(tot / n, 1), round(100.0 * tot / total, 3), mn, mx])


if __name__ == "__main__":
    main(sys.argv[1])
