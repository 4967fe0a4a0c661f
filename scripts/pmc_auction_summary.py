#!/usr/bin/env python3
"""Summarise the SQ counter passes of scripts/gpu_pmc_auction.sh into
profiles/<round>_pmc_auction.json: per-dispatch instruction counts of the
auction kernel and its issue utilisation.

Issue model (MI355X_MICROARCH.md; cdna_hip_programming.md "CU = 4 x SIMD-32"):
per CU and cycle at most one scalar instruction, two wave64 vector
instructions (four SIMD-32 units, 2 cycles each) and one LDS instruction
issue. frac = instructions / (kernel time x clock x 256 CUs x that rate),
with the kernel's mean duration from the kernel-trace pass of the same
command (trace.csv; else the call time of out_1.txt) and the 2.4 GHz peak clock: a lower bound on the busy fraction
when the chip clocks lower. SQ_*_CYCLES counters count quad-cycles (x4).
VALU is reported as VALU-active as well: SQ_ACTIVE_INST_VALU x 4 / (kernel
cycles x 256 CUs x 4 SIMDs) -- an fp64 VALU op holds its SIMD for several
cycles, so the instruction-count model under-reads a fp64-heavy kernel.

Usage: python scripts/pmc_auction_summary.py gpurun_out/pmca profiles/r2_pmc_auction.json
"""
import collections
import csv
import glob
import json
import os
import re
import sys

CLOCK_HZ = 2.4e9
CUS = 256
RATE = {"SQ_INSTS_SALU": 1.0, "SQ_INSTS_VALU": 2.0, "SQ_INSTS_LDS": 1.0}


def main(src, dst):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, "pass_*.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    txt = open(os.path.join(src, "out_1.txt")).read()
    m = re.search(r"(?:auction-only|solve) B=(\d+) n=(\d+): ([0-9.]+) ms", txt)
    B, n, ms = int(m.group(1)), int(m.group(2)), float(m.group(3))
    out = {"source": "rocprofv3 --pmc (two passes of SQ counters, counters only) of "
                     "`python3 scripts/auction_only.py` (scripts/gpu_pmc_auction.sh)",
           "model": "frac = insts / (kernel_ms x 2.4 GHz x 256 CUs x issue rate per CU-cycle: "
                    "SALU 1, VALU 2 (wave64 on 4 x SIMD-32), LDS 1); *_CYCLES are quad-cycles; "
                    "valu_active = SQ_ACTIVE_INST_VALU x 4 / (kernel cycles x 256 CUs x 4 SIMDs)",
           "config": {"n": n, "B_per_gpu": B, "kernel_ms": ms},
           "kernels": {}}
    # the kernel's own duration from the kernel-trace pass (trace.csv), when
    # present; otherwise the whole solve call's time (an upper bound)
    kdur = collections.defaultdict(list)
    tp = os.path.join(src, "trace.csv")
    if os.path.exists(tp):
        for r in csv.DictReader(open(tp)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            kdur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    for k, cv in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cv.items()}
        kms = sum(kdur[k]) / len(kdur[k]) if kdur.get(k) else ms
        cyc = kms * 1e-3 * CLOCK_HZ * CUS
        e = {"kernel_ms": kms, "call_ms": ms,
             "kernel_ms_source": "trace.csv (kernel-trace pass)" if kdur.get(k) else "call time",
             "per_dispatch": avg,
             "per_swarm": {c: avg[c] / B for c in ("SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS")
                           if c in avg}}
        for c, rate in RATE.items():
            if c in avg:
                e[c.replace("SQ_INSTS_", "").lower() + "_issue_frac"] = avg[c] / (cyc * rate)
        if "SQ_ACTIVE_INST_VALU" in avg:
            e["valu_active"] = avg["SQ_ACTIVE_INST_VALU"] * 4.0 / (cyc * 4.0)
        if "SQ_WAVE_CYCLES" in avg and "SQ_WAIT_ANY" in avg:
            e["wait_any_share"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
        if "SQ_WAVE_CYCLES" in avg and "SQ_ACTIVE_INST_ANY" in avg:
            e["active_inst_share"] = avg["SQ_ACTIVE_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_ACTIVE_INST_LDS" in avg and avg["SQ_ACTIVE_INST_LDS"]:
            e["lds_bank_conflict_per_active_lds"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_ACTIVE_INST_LDS"]
        out["kernels"][k] = e
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
