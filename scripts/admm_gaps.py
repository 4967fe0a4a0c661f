#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of an ADMM batch from a rocprofv3
kernel trace (diagnostic): python scripts/admm_gaps.py trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
prev_end, prev_name = None, None
gaps = []
busy = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    if prev_end is not None and s > prev_end:
        gaps.append((s - prev_end, prev_name, r["Kernel_Name"][:60], (s - t0) / 1e6))
    prev_end = max(prev_end or 0, e)
    prev_name = r["Kernel_Name"][:60]
span = prev_end - t0
print(f"span {span/1e6:.1f} ms, kernel busy {busy/1e6:.1f} ms, idle {sum(g[0] for g in gaps)/1e6:.1f} ms")
gaps.sort(reverse=True)
for g in gaps[:25]:
    print(f"{g[0]/1e3:9.1f} us at {g[3]:9.2f} ms  after {g[1]}  before {g[2]}")
