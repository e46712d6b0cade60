"""Kernel statistics (rocprofv3 --stats CSV layout) from a rocprofv3 results database, for the
runs where this rocprofv3 writes only the rocpd SQLite file.

usage: python tools/rocpd_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    dur = defaultdict(list)
    for name, d in c.execute("select name, duration from kernels"):
        dur[name].append(int(d))
    total = sum(sum(v) for v in dur.values())
    rows = sorted(dur.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, v in rows:
            w.writerow([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / total, 2), min(v), max(v),
                        statistics.pstdev(v)])


if __name__ == "__main__":
    main()
