#!/usr/bin/env python3
"""Closed-loop episode benchmark (acl_episode_batch).

B swarms of n = 100 vehicles (config C3 shape: noncomplete formations, a
unique formation per swarm, ADMM-structured gain records) flown for `steps`
control periods of 10 ms: auto-auctions every 120 steps (1.2 s), DistCntrl +
Safety + makeSafeTraj every step, supervisor ticks every 2 steps. Reports
swarm-steps/s (one swarm advanced one control period) with the state
resident in HBM, per-kernel times from HIP events are not used here (the
step is a sequence of small launches; rocprofv3 --stats gives the split).
The CPU baseline runs oracle/episode_oracle.py's loop on a bounded sample.

--assignment both: the reference's CBAA-vs-centralized comparison
(coordination_ros.cpp:330-343, /operator/central_assignment): the same swarms
flown once with the distributed auction and once with the operator's
Hungarian assignment at every auto-auction (acl_episode_params_t::assignment),
and the episode outcomes of each (converged / gridlocked swarms and their
steps, collision-avoidance vehicle-steps, auction events) in one line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from aclswarm_amd import _lib as L  # noqa: E402
from aclswarm_amd import engine, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16384)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-tile-gains", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="also time the chunk of `steps` captured once as a HIP graph and "
                         "replayed (the per-step launches without host launch overhead)")
    ap.add_argument("--reps", type=int, default=3, help="graph replays timed")
    ap.add_argument("--assignment", choices=("cbaa", "central", "both"), default="cbaa")
    args = ap.parse_args()
    if args.assignment == "both":
        return compare(args)
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(99)
    w = workload.simform_workload(args.B, args.n, gen, dev, F=None, complete=False, planes=5)
    T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"], w["planes"])
    if not args.no_tile_gains:
        T.tile_gains()  # formation setup: tile-ordered gain records (acl_tile_gains)
    # warm-up: a short episode (first launches, workspace)
    ep_run = L.default_episode_params()
    ep_run.assignment = L.ASSIGN_CENTRAL if args.assignment == "central" else L.ASSIGN_CBAA
    e0 = engine.Episode(T, w["fidx"], w["q"], w["vel"], w["P_in"], params=ep_run)
    e0.run(2)
    torch.cuda.synchronize()
    e = engine.Episode(T, w["fidx"], w["q"], w["vel"], w["P_in"], params=ep_run)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.run(args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    graph = None
    if args.graph:
        # the same chunk captured once on a side stream and replayed: each
        # replay advances the state by `steps` control periods with the
        # captured step numbering (auctions at the same offsets)
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        eg = engine.Episode(T, w["fidx"], w["q"], w["vel"], w["P_in"])
        with torch.cuda.stream(gs):
            eg.run(args.steps, stream=gs.cuda_stream)  # eager chunk on the capture stream
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=gs):
            eg.run(args.steps, stream=gs.cuda_stream)
        torch.cuda.synchronize()
        with torch.cuda.stream(gs):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(gs):
            for _ in range(args.reps):
                g.replay()
        torch.cuda.synchronize()
        dg = (time.perf_counter() - t0) / args.reps
        # eager launches over the same stretch of the episode as the timed
        # replays (chunks 3 .. 2 + reps): the swarms are further along there
        # (closer, more collision avoidance) than in the first chunk above
        ee = engine.Episode(T, w["fidx"], w["q"], w["vel"], w["P_in"])
        ee.run(2 * args.steps)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ee.run(args.steps)
        torch.cuda.synchronize()
        de = (time.perf_counter() - t0) / args.reps
        graph = {"value": args.B * args.steps / dg, "unit": "swarm-steps/s",
                 "ms_per_step": dg / args.steps * 1e3, "replays": args.reps,
                 "eager_same_stretch_ms_per_step": de / args.steps * 1e3,
                 "what": f"{args.steps} steps captured once as a HIP graph, replayed; "
                         "eager_same_stretch: eager launches over the same chunks of the episode"}
    st = e.status()
    ep = e.ep
    line = {
        "metric": f"closed-loop episode swarm-steps/sec (N={args.n})",
        "value": args.B * args.steps / dt, "unit": "swarm-steps/s",
        "B": args.B, "n": args.n, "steps": args.steps, "seconds": dt,
        "ms_per_step": dt / args.steps * 1e3,
        "auctions_per_swarm": int(st["n_auctions"][0] + st["n_skipped"][0]),
        "control_dt": ep.control_dt, "auction_every": ep.auction_every,
        "dtype": "f64", "data": "synthetic (simform_workload, C3 shape)",
        "graph": graph,
        "episode": {"converged": int((st["converged_step"] >= 0).sum()),
                    "gridlocked": int((st["gridlock_step"] >= 0).sum()),
                    "invalid_auctions": int(st["n_invalid"].sum()),
                    "disagree_auctions": int(st["n_disagree"].sum()),
                    "ca_vehicle_steps": int(st["n_ca_steps"].sum())},
    }
    if not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import episode_oracle as E
        epd = E.params_from_struct(ep)
        b = 0
        f = int(w["fidx"][b])
        p = w["p"][f].cpu().numpy()
        adj = w["adj"][f].cpu().numpy().astype(np.uint8)
        G = workload.dense_gains_host(w, f)
        q = w["q"][b].cpu().numpy()
        vel = w["vel"][b].cpu().numpy()
        P = w["P_in"][b].cpu().numpy().view(np.uint16)
        t0 = time.perf_counter()
        k = 0
        while True:
            E.run_episode(q, vel, P, p, adj, G, 1, epd, step0=k)
            k += 1
            if time.perf_counter() - t0 > args.cpu_budget:
                break
        tc = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": k / tc, "unit": "swarm-steps/s", "cores": 1,
                                "kind": "port",
                                "sample": f"{k} control steps of one n={args.n} swarm through "
                                          "oracle/episode_oracle.py (C restatement of "
                                          "DistCntrl/Safety/CBAA per vehicle), 1 thread"}
    print(json.dumps(line), flush=True)


def outcomes(st, steps):
    conv = st["converged_step"]
    grid = st["gridlock_step"]
    c = conv >= 0
    return {"converged": int(c.sum()),
            "converged_step_mean": float(conv[c].mean()) if c.any() else None,
            "converged_step_median": float(np.median(conv[c])) if c.any() else None,
            "gridlocked": int((grid >= 0).sum()),
            "ca_vehicle_steps": int(st["n_ca_steps"].sum()),
            "assignments_applied": int(st["n_auctions"].sum()),
            "invalid": int(st["n_invalid"].sum()), "skipped": int(st["n_skipped"].sum()),
            "disagree": int(st["n_disagree"].sum()), "steps": steps}


def compare(args):
    """CBAA vs the centralized Hungarian on the same swarms (same workload,
    same start): one JSON line with both modes' episode outcomes and rates."""
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(99)
    w = workload.simform_workload(args.B, args.n, gen, dev, F=None, complete=False, planes=5)
    T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"], w["planes"])
    if not args.no_tile_gains:
        T.tile_gains()
    res = {}
    for name, mode in (("cbaa", L.ASSIGN_CBAA), ("central", L.ASSIGN_CENTRAL)):
        ep = L.default_episode_params()
        ep.assignment = mode
        e0 = engine.Episode(T, w["fidx"], w["q"], w["vel"], w["P_in"], params=ep)
        e0.run(2)
        torch.cuda.synchronize()
        e = engine.Episode(T, w["fidx"], w["q"], w["vel"], w["P_in"], params=ep)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.run(args.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        r = outcomes(e.status(), args.steps)
        r["swarm_steps_per_s"] = args.B * args.steps / dt
        r["ms_per_step"] = dt / args.steps * 1e3
        res[name] = r
    line = {"metric": f"closed-loop episodes, CBAA vs centralized Hungarian (N={args.n})",
            "B": args.B, "n": args.n, "steps": args.steps, "control_dt": 0.01,
            "auction_every": 120, "dtype": "f64",
            "data": "synthetic (simform_workload, C3 shape: noncomplete generator formations, "
                    "a unique formation per swarm), same swarms and starts in both modes",
            "cbaa": res["cbaa"], "central": res["central"]}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
