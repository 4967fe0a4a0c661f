#!/usr/bin/env python3
"""Per-phase SQ instruction split of the fused auction kernel from the stop-build
counter passes (scripts/auction_phase_pmc.sh): pass_k.csv is the build that
returns after phase k (pass_0 = the whole kernel). Prints per-swarm counts of
each phase as differences of consecutive stops.
Usage: python scripts/phase_split.py DIR [B]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
NAMES = {1: "load + neighbourhoods", 2: "alignment read-back", 3: "prices", 4: "START bids",
         5: "CBAA rounds", 0: "adoption + hand-off + fused control"}
ORDER = [1, 2, 3, 4, 5, 0]
CNT = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES"]
tot = {}
for k in ORDER:
    f = os.path.join(d, f"pass_{k}.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "auction_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    tot[k] = {c: (sum(v) / len(v) / B if v else float("nan")) for c, v in agg.items()}
print(f"per swarm (B = {B}), cumulative counts of the stop-k builds -> per-phase differences")
print(f"{'phase':40s}" + "".join(f"{c[8:]:>14s}" for c in CNT))
prev = {c: 0.0 for c in CNT}
for k in ORDER:
    if k not in tot:
        continue
    row = {c: tot[k].get(c, float("nan")) - prev[c] for c in CNT}
    print(f"{NAMES[k]:40s}" + "".join(f"{row[c]:14.0f}" for c in CNT))
    prev = {c: tot[k].get(c, float("nan")) for c in CNT}
if 0 in tot:
    print(f"{'whole kernel':40s}" + "".join(f"{tot[0].get(c, float('nan')):14.0f}" for c in CNT))
