"""acl_tile_gains alone on the bench's C3 formation table (PMC / timing of
the setup kernel): python scripts/tile_only.py [--B 65536] [--reps 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aclswarm_amd import engine, workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=65536)
ap.add_argument("--n", type=int, default=100)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda:0")
gen = torch.Generator(device=dev)
gen.manual_seed(1)
w = workload.simform_workload(a.B, a.n, gen, dev)
T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"], w["planes"])
T.tile_gains()
torch.cuda.synchronize()
ms = []
for _ in range(a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    T.tile_gains()
    e1.record()
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
nbytes = 2 * w["gains"].numel() * 8
print("tile_gains F=%d n=%d: %.3f ms (min of %d), %.1f GB moved (read + write), %.0f GB/s" % (
    a.B, a.n, min(ms), a.reps, nbytes / 1e9, nbytes / (min(ms) * 1e-3) / 1e9))
