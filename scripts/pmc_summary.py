#!/usr/bin/env python3
"""Summarise the two rocprofv3 PMC passes (scripts/gpu_pmc.sh) into
profiles/<round>_pmc_traffic.json: HBM bytes per launch per kernel.

FETCH_SIZE / WRITE_SIZE are KiB (TCC_EA0 request counters x 64 B / 1024).
gfx950 tallies a wide coalesced read at half its bytes
(MI355X_MICROARCH.md "HBM [CDNA4]"), so hbm_bytes = 2*FETCH + WRITE; the
uncorrected figure is kept beside it.

Usage: python scripts/pmc_summary.py gpurun_out/pmc profiles/r1_pmc_traffic.json
"""
import collections
import csv
import json
import os
import sys


def main(src, dst):
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                     "`python3 bench.py --steps 2 --warmup 1 --no-cpu`",
           "correction": "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB x 1024); gfx950 "
                         "FETCH_SIZE counts wide coalesced reads at 1/2",
           "kernels": {}}
    vals = collections.defaultdict(dict)
    for C in ("FETCH_SIZE", "WRITE_SIZE"):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(src, C + ".csv"))):
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]) * 1024.0)
        for k, v in acc.items():
            vals[k][C] = sum(v) / len(v)
            vals[k]["launches"] = len(v)
    bench = json.load(open(os.path.join(src, "bench_FETCH_SIZE.json")))
    out["config"] = {"n": bench["config"]["n"], "B_per_gpu": bench["config"]["B_per_gpu"],
                     "workload": bench["config"]["workload"]}
    for k, v in vals.items():
        out["kernels"][k] = {"fetch_bytes_raw": v["FETCH_SIZE"], "write_bytes": v["WRITE_SIZE"],
                             "hbm_bytes": 2 * v["FETCH_SIZE"] + v["WRITE_SIZE"],
                             "launches_sampled": v["launches"]}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
