#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of the auction kernel, on the bench
workload, through the library's internal hook acl_internal_set_stamps.

Stamp layout per swarm (csrc/control_params.h, kStampStride = 32 u64):
  0..6   s_memtime at the end of each auction phase (the XCD's shader clock:
         only differences within one workgroup are used)
  7      s_memtime at the end of the fused control phase (0 if the swarm had
         per-vehicle rows and left its control to gain_kernel)
  8, 9   s_memrealtime (the 100 MHz clock every XCD shares) at the swarm's
         start and end: the kernel span and the mean resident swarms
  16..   section counters of the -DACL_AUCTION_PROF / ACL_WIDE_PROF /
         ACL_CA_PROF builds"""
import argparse
import ctypes as ct
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aclswarm_amd import _lib as L  # noqa: E402
from aclswarm_amd import engine, workload  # noqa: E402

NAMES = ["load+nbhd", "align", "prices", "cbaa", "adopt", "handoff"]

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=65536)
ap.add_argument("--n", type=int, default=100)
ap.add_argument("--formations", type=int, default=0)
ap.add_argument("--L", type=float, default=None)
ap.add_argument("--crowd", type=float, default=None,
                help="scale positions about each swarm's centre (collision avoidance active)")
ap.add_argument("--margin", action="store_true",
                help="track the decision margin (default: skip_margin, the bench headline's kernel)")
ap.add_argument("--no-control", action="store_true",
                help="auction only (the PROF build's CBAA section counters are not overwritten "
                     "by the collision-avoidance kernel's)")
args = ap.parse_args()
dev = torch.device("cuda:0")
gen = torch.Generator(device=dev)
gen.manual_seed(1)
w = workload.simform_workload(args.B, args.n, gen, dev, F=(args.formations or None), L=args.L)
if args.n > 128:
    NAMES[:] = ["load+nbhd", "align", "prices", "cbaa", "adopt", "handoff"]
T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"],
                              w["planes"])
if args.crowd:
    c = w["q"][:, :, :2].mean(dim=1, keepdim=True)
    w["q"][:, :, :2] = c + args.crowd * (w["q"][:, :, :2] - c)
lib = L.lib()
lib.acl_internal_set_stamps.argtypes = [ct.c_void_p]
SS, RT0, RT1, SEC = 32, 8, 9, 16  # csrc/control_params.h kStamp*
st = torch.zeros((args.B, SS), dtype=torch.int64, device=dev)
ctl = not args.no_control
engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"], do_control=ctl, margin=args.margin)  # warm
torch.cuda.synchronize()
lib.acl_internal_set_stamps(ct.c_void_p(st.data_ptr()))
engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"], do_control=ctl, margin=args.margin)
torch.cuda.synchronize()
lib.acl_internal_set_stamps(ct.c_void_p(0))
s = st.cpu().numpy().astype(np.float64)
d = np.diff(s[:, :7], axis=1)
tot = d.sum(1)
print(f"per-swarm cycles: mean {tot.mean():.0f}  median {np.median(tot):.0f}")
for k, nm in enumerate(NAMES):
    print(f"  {nm:16s} mean {d[:, k].mean():10.0f}  share {d[:, k].sum() / tot.sum() * 100:5.1f}%")
# fused control phase (slot 7): its cycles and its share of the life of the
# swarms that ran it (same-workgroup s_memtime differences only)
fz = s[:, 7] > 0
if fz.any():
    g = s[fz, 7] - s[fz, 6]
    life = s[fz, 7] - s[fz, 0]
    print(f"  control (fused)  mean {g.mean():10.0f}  share of swarm life "
          f"{g.sum() / life.sum() * 100:5.1f}%  ({int(fz.sum())} of {args.B} swarms fused)")
# kernel span and residency from the shared 100 MHz clock (slots 8, 9)
ok = (s[:, RT0] > 0) & (s[:, RT1] > 0)
if ok.any():
    r0, r1 = s[ok, RT0], s[ok, RT1]
    span = r1.max() - r0.min()
    print(f"  span {span / 100:.1f} us (100 MHz clock); mean resident swarms "
          f"{(r1 - r0).sum() / span:.1f}; swarm life mean {(r1 - r0).mean() / 100:.2f} us")
    e = s[ok, 7] if fz[ok].all() else s[ok, 6]
    c = s[ok, 0]
    print(f"  shader clock over the swarm lives: {((e - c) / (r1 - r0)).mean() * 100:.0f} MHz")
# CBAA column-step sections (a -DACL_AUCTION_PROF=1 build): cycles summed
# over a swarm's waves, and the counts of evaluated columns, walks and scans
sec = st.cpu().numpy()[:, SEC:SEC + 9].astype(np.uint64)
# (n <= 128: ca_pair_kernel writes no stamps, so the slots are the CBAA's
# with collision avoidance on as well)
if args.n <= 128 and sec[:, :8].any():
    SN = ["level 0", "levels", "margin bound", "runner-up walk", "exact scan", "write-back",
          "selects+barrier", "column barrier"]
    tot8 = sec[:, :8].astype(np.float64).sum()
    for k, nm in enumerate(SN):
        x = sec[:, k].astype(np.float64)
        print(f"  cbaa {nm:16s} wave-cycles/swarm {x.mean():10.0f}  share {x.sum() / tot8 * 100:5.1f}%")
    cnt = sec[:, 8]
    f12 = lambda sh, w=12: ((cnt >> np.uint64(sh)) & np.uint64((1 << w) - 1)).astype(np.float64)
    if os.environ.get("ACL_PROF_OLDPACK"):  # libraries before round 4: 21-bit fields
        cols, walks, scans = f12(0, 21), f12(21, 21), f12(42, 21)
        sels = selx = np.zeros_like(cols)
    else:
        cols, walks, scans, sels, selx = f12(0), f12(12), f12(24), f12(36), f12(48)
    print(f"  per swarm: columns evaluated {cols.mean():.1f}, runner-up walks {walks.mean():.1f}, "
          f"exact scans {scans.mean():.1f}, re-selects {sels.mean():.1f}, "
          f"select margin evaluations (per 64-task chunk) {selx.mean():.1f}")
# wide CBAA sections (a -DACL_WIDE_PROF=1 build, n > 128): wave-cycles summed
# over the swarm's 16 waves
if args.n > 128 and sec[:, :4].any():
    WN = ["column updates", "exact scans", "re-selects", "round barriers"]
    for k, nm in enumerate(WN):
        x = sec[:, k].astype(np.float64)
        print(f"  wide {nm:16s} wave-cycles/swarm {x.mean():12.0f}")
    cnt = sec[:, 4]
    m21 = np.uint64((1 << 21) - 1)
    print(f"  per swarm: columns {(cnt & m21).astype(float).mean():.1f}, exact scans "
          f"{((cnt >> np.uint64(21)) & m21).astype(float).mean():.1f}, re-selects "
          f"{(cnt >> np.uint64(42)).astype(float).mean():.1f}, rounds {sec[:, 5].astype(float).mean():.1f}")
    for k, nm in enumerate(["T load + keys", "levels", "write-back"]):
        print(f"    column {nm:14s} wave-cycles/swarm {sec[:, 6 + k].astype(np.float64).mean():12.0f}")
    spc = st.cpu().numpy()[:, SEC + 9].astype(np.uint64)
    if spc.any():
        g = lambda sh: ((spc >> np.uint64(sh)) & m21).astype(float).mean()
        print(f"  column updates per swarm: sparse {g(0):.1f}, dense {g(21):.1f}, "
              f"sparse -> dense {g(42):.1f}")
# collision avoidance (a -DACL_CA_PROF=1 build, --crowd, n > 128): ca_kernel
# wave-cycles (ca_pair_kernel, n <= 128, has no such counters)
if args.crowd and not args.no_control and args.n > 128:
    x = st.cpu().numpy()[:, SEC + 8:SEC + 12].astype(np.float64)
    cnt = x[:, 3].sum()
    print(f"  ca close vehicles {cnt:.0f} ({cnt / args.B:.1f} per swarm)")
    for k, nm in enumerate(["sector build", "resolve", "other (q, loop)"]):
        print(f"  ca {nm:16s} wave-cycles per close vehicle {x[:, k].sum() / max(cnt, 1):10.0f}")
