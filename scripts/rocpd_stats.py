"""Kernel statistics (name, calls, total/avg ns, %) from a rocprofv3 SQLite
result (`rocprofv3 --kernel-trace --stats` without --output-format csv) as a
CSV like rocprofv3's kernel_stats.csv.  Usage: rocpd_stats.py DB OUT.csv"""
import csv
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    return name if len(name) < 160 else name[:157] + "..."


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage "
                     "from top_kernels").fetchall()  # durations in us
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, calls, tot, avg, pct in rows:
            w.writerow([short(name), calls, f"{tot * 1e3:.0f}",
                        f"{avg * 1e3:.0f}", f"{pct:.2f}"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
