#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace` on this image): rocpd_stats.py DB [--per KERNEL]
prints total/avg duration per kernel name; --per divides the totals by the
call count of KERNEL (e.g. one launch per batch) and writes a CSV with -o."""
import argparse
import csv
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--per", default=None)
ap.add_argument("-o", default=None)
a = ap.parse_args()
c = sqlite3.connect(a.db)
tot = defaultdict(float)
cnt = defaultdict(int)
t0, t1 = None, None
for name, start, end in c.execute("select name, start, end from kernels"):
    tot[name] += (end - start) / 1e6
    cnt[name] += 1
    t0 = start if t0 is None else min(t0, start)
    t1 = end if t1 is None else max(t1, end)
div = 1.0
if a.per:
    m = [k for k in cnt if a.per in k]
    div = float(cnt[m[0]]) if m else 1.0
rows = sorted(tot, key=lambda k: -tot[k])
print(f"kernel time {sum(tot.values()) / div:.2f} ms per unit ({div:.0f} units)")
for k in rows[:30]:
    print(f"{tot[k] / div:9.3f} ms {cnt[k] / div:8.1f} calls {tot[k] / cnt[k] * 1e3:9.1f} us  {k[:100]}")
if a.o:
    with open(a.o, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "PerUnitMs"])
        for k in rows:
            w.writerow([k, cnt[k], int(tot[k] * 1e6), int(tot[k] / cnt[k] * 1e6), tot[k] / div])
