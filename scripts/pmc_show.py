#!/usr/bin/env python3
"""Print per-dispatch averages of the counter CSVs a gpu_pmc_*.sh run left."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmck"
for f in sorted(glob.glob(f"{d}/pass_*.csv")):
    rows = list(csv.DictReader(open(f)))
    if not rows:
        print(f, "(no rows)")
        continue
    agg = collections.defaultdict(list)
    for r in rows:
        agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(f, "VGPR", rows[0]["VGPR_Count"], "grid", rows[0]["Grid_Size"])
    for (k, c), v in sorted(agg.items()):
        print(f"  {k:42s} {c:28s} n={len(v):3d} avg={sum(v) / len(v):.4g}")
