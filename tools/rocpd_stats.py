#!/usr/bin/env python3
"""Kernel statistics (the columns of rocprofv3 --stats' kernel_stats.csv) from a rocprofv3
results database (the default rocpd output format of ROCm 7).

  python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/<name>_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys


def main():
    db = sys.argv[1]
    con = sqlite3.connect(db)
    rows = {}
    for name, start, end in con.execute("select name, start, end from kernels"):
        rows.setdefault(name, []).append(end - start)
    total = sum(sum(v) for v in rows.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(d), sum(d), round(sum(d) / len(d), 3), round(100.0 * sum(d) / total, 4), min(d), max(d),
                    round(statistics.pstdev(d), 3)])


if __name__ == "__main__":
    main()
