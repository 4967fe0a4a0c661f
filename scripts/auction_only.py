"""Runs the auction kernel alone (do_control=0) on the bench workload, for
PMC/ISA studies: python scripts/auction_only.py [--B 8192] [--reps 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aclswarm_amd import engine, workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=8192)
ap.add_argument("--n", type=int, default=100)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--L", type=float, default=None, help="generator area (default: the bench config's)")
ap.add_argument("--complete", action="store_true", help="complete formation graphs (config C2)")
ap.add_argument("--control", action="store_true", help="run the control kernels too")
ap.add_argument("--crowd", type=float, default=None,
                help="scale positions about each swarm's centre (bench.py's ca_probe: 0.3)")
ap.add_argument("--hist", action="store_true", help="print the eff_rounds histogram")
ap.add_argument("--margin", action="store_true",
                help="track the decision margin (default: skip_margin, the bench headline's kernel)")
a = ap.parse_args()
dev = torch.device("cuda:0")
gen = torch.Generator(device=dev)
gen.manual_seed(1)
w = workload.simform_workload(a.B, a.n, gen, dev, L=a.L, complete=a.complete)
if a.crowd is not None:
    cen = w["q"][:, :, :2].mean(dim=1, keepdim=True)
    w["q"][:, :, :2] = cen + a.crowd * (w["q"][:, :, :2] - cen)
T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"],
                              w["planes"])
engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"], do_control=a.control, margin=a.margin)  # warm
torch.cuda.synchronize()
ms = []
for _ in range(a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"], do_control=a.control,
                       margin=a.margin)
    e1.record()
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
st = engine.status_to_numpy(out["status"])
print(("solve" if a.control else "auction-only") + " B=%d n=%d: %.3f ms (min of %d), %.0f swarms/s; eff_rounds sum %d, valid %d" % (
    a.B, a.n, min(ms), a.reps, a.B / min(ms) * 1e3, int(st["eff_rounds"].sum()),
    int((st["flags"] & 1).sum())))
if a.hist:
    import numpy as np
    er = st["eff_rounds"].astype(np.int64)
    h = np.bincount(er)
    print("eff_rounds histogram (rounds: swarms):",
          {int(k): int(v) for k, v in enumerate(h) if v})
    print("eff_rounds mean %.2f, p50 %d, p90 %d, p99 %d, max %d" % (
        er.mean(), np.percentile(er, 50), np.percentile(er, 90), np.percentile(er, 99), er.max()))
