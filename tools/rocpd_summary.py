"""Kernel summary (name, calls, total/avg microseconds, %) of a rocprofv3 SQLite
output (`rocprofv3 --kernel-trace --stats -d DIR -o NAME`, default format),
as CSV like rocprofv3's kernel_stats.csv.

    python tools/rocpd_summary.py gpurun_out/x/prof/ao_results.db > profiles/...csv
"""
import csv
import sqlite3
import sys


def main(path, limit=12):
    con = sqlite3.connect(path)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for name, calls, total, avg, pct in con.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels limit ?", (limit,)):
        w.writerow([name if len(name) < 200 else name[:197] + "...", calls, round(total, 1), round(avg, 1),
                    round(pct, 3)])


if __name__ == "__main__":
    main(sys.argv[1])
