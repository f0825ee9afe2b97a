#!/usr/bin/env python3
"""Kernel statistics of a rocprofv3 run that wrote its default SQLite database (run_results.db),
in the column layout of rocprofv3's own --stats CSV (kernel_stats.csv):

    python tools/rocpd_stats.py gpurun_out/r06u/prof_c3/run_results.db > profiles/r06/c3_kernel_stats_r06u.csv

Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev -- over every dispatch in
the database's `kernels` view, sorted by total duration.
"""
import csv
import math
import sqlite3
import sys
from collections import defaultdict


def main(path):
    con = sqlite3.connect(path)
    durs = defaultdict(list)
    for name, d in con.execute("select name, duration from kernels"):
        durs[name].append(float(d))
    total = sum(sum(v) for v in durs.values()) or 1.0
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        n, s = len(v), sum(v)
        mean = s / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        w.writerow([name, n, int(s), mean, round(100 * s / total, 2), int(min(v)), int(max(v)), sd])


if __name__ == "__main__":
    main(sys.argv[1])
