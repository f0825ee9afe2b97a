#!/usr/bin/env python3
"""Kernel statistics CSV from a rocprofv3 results database (the `--kernel-trace --stats` run writes
`<name>_results.db`; this prints the columns of rocprofv3's kernel_stats.csv from its `kernels` view):

    python profiles/db_stats.py gpurun_out/<tag>/prof/run_results.db > profiles/r02/c3_kernel_stats_<tag>.csv
"""
import csv
import sqlite3
import statistics
import sys


def main(path):
    con = sqlite3.connect(path)
    per = {}
    for name, dur in con.execute("select name, duration from kernels"):
        per.setdefault(name, []).append(int(dur))
    total = sum(sum(v) for v in per.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name if len(name) < 200 else name[:200] + "...", len(v), sum(v), sum(v) / len(v),
                    round(100.0 * sum(v) / total, 2), min(v), max(v),
                    statistics.pstdev(v) if len(v) > 1 else 0.0])


if __name__ == "__main__":
    main(sys.argv[1])
