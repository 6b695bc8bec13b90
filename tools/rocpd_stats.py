"""Condense a rocprofv3 SQLite (rocpd) result into the kernel-stats CSV kept under profiles/:
name, calls, total_ns, average_ns, percentage (the --stats summary of the same run).

    python tools/rocpd_stats.py gpurun_out/<tag>/prof/run_results.db > profiles/<name>.csv
"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, calls, total, avg, pct in c.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, round(total, 1), round(avg, 1), round(pct, 3)])


if __name__ == "__main__":
    main(sys.argv[1])
