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

--trials: batched Monte-Carlo trials (acl_trial_batch, supervisor.py over
the closed loop) at the C3 shape: B swarms of n = 100, each flying its
formation group's two formations (the reference generator's 'A' and 'B',
generate_random_formation.py:59-80) with gains designed on the device by
acl_admm_solve_batch (the reference's own ADMM design, not synthetic
blocks, so that the swarms can converge), through HOVERING -> ... ->
COMPLETE / TERMINATE with the reference's timings (supervisor.py:50-57);
reports trials/s (every trial run to its end) and the trial records'
statistics, per assignment mode.

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
    ap.add_argument("--trials", action="store_true", help="batched Monte-Carlo trials (see above)")
    ap.add_argument("--max-steps", type=int, default=70000,
                    help="trials: control steps at most (the 600 s watchdog ends every trial "
                         "by 60 000)")
    ap.add_argument("--chunk", type=int, default=2000, help="trials: steps per call")
    args = ap.parse_args()
    if args.trials:
        return trials(args)
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
    n, B = args.n, args.B
    L_side = 15.0 if n <= 20 else 40.0 * (n / 100.0) ** 0.5
    # the formations' gains from acl_admm_solve_batch (converging swarms)
    T, _, _ = admm_table(n, B, L_side, 0, dev)
    if not args.no_tile_gains:
        T.tile_gains()
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    side = 20.0 * (n / 20.0) ** 0.5
    q = workload.nonoverlapping_points(B, n, side, side, 1.0, 1.0, 1.5, gen, dev)
    w = {"fidx": (2 * torch.arange(B, device=dev)).to(torch.int32), "q": q,
         "vel": torch.zeros_like(q),
         "P_in": torch.arange(n, dtype=torch.int16, device=dev).expand(B, n).contiguous()}
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
            "data": "synthetic: the reference generator's formations (C3 shape: L=40, "
                    "noncomplete, formation 'A' of seeds 0..B-1) with gains designed by "
                    "acl_admm_solve_batch; start.sh-style starts at the identity "
                    "assignment; the same swarms and starts in both modes",
            "cbaa": res["cbaa"], "central": res["central"]}
    print(json.dumps(line), flush=True)


def admm_table(n, F, L_side, seed0, dev, chunk=1024):
    """The formation groups of F swarms ('A' and 'B' from the reference
    generator, seeds seed0 ..) with gains from acl_admm_solve_batch, as a
    5-entry-record formation table of 2F formations: swarm b flies 2b, 2b+1."""
    g = engine.generate_formation_groups(
        torch.arange(seed0, seed0 + F, dtype=torch.int64, device=dev), n, False, L_side, L_side,
        2.0, 2.0)
    if int((g["status"] != 0).sum().item()):
        raise RuntimeError("a formation did not fit the box")
    p = g["points"].reshape(2 * F, n, 3).contiguous()        # [F][2] -> 2F
    adj = g["adj"].bool().repeat_interleave(2, dim=0)         # one graph per group
    recs, E = [], adj.sum(dim=(1, 2)).to(torch.int64)
    iters = []
    t0 = time.perf_counter()
    for f0 in range(0, 2 * F, chunk):
        f1 = min(2 * F, f0 + chunk)
        G, its = engine.admm_design(p[f0:f1], adj[f0:f1].to(torch.float64))
        iters.append(its)
        ff, ii, jj = adj[f0:f1].nonzero(as_tuple=True)
        i3, j3 = 3 * ii, 3 * jj
        zeros = torch.stack([G[ff, i3, j3 + 2], G[ff, i3 + 1, j3 + 2], G[ff, i3 + 2, j3],
                             G[ff, i3 + 2, j3 + 1]])
        if bool((zeros != 0).any()) or bool(torch.signbit(zeros).any()):
            raise RuntimeError("ADMM gains without the solver.cpp:49-77 block structure")
        recs.append(torch.stack([G[ff, i3, j3], G[ff, i3, j3 + 1], G[ff, i3 + 1, j3],
                                 G[ff, i3 + 1, j3 + 1], G[ff, i3 + 2, j3 + 2]], dim=1).reshape(-1))
        del G
    torch.cuda.synchronize()
    t_admm = time.perf_counter() - t0
    goff = torch.zeros(2 * F, dtype=torch.int64, device=dev)
    goff[1:] = torch.cumsum(E, 0)[:-1]
    bits = workload.pack_bits(adj)
    T = engine.FormationTable(n, p, bits, torch.cat(recs), goff, 5)
    its = torch.cat(iters)
    return T, t_admm, {"admm_iters_max": int(its.max().item()),
                       "admm_unreliable": int((its < 0).sum().item())}


def trial_stats(tr, K):
    r = tr.records()
    st = tr.status()
    done = r["done_step"] >= 0
    comp = r["state"] == L.TRIAL_COMPLETE
    term = r["state"] == L.TRIAL_TERMINATE
    names = {L.TRIAL_HOVERING: "HOVERING", L.TRIAL_WAITING: "WAITING_ON_ASSIGNMENT",
             L.TRIAL_FLYING: "FLYING", L.TRIAL_IN_FORMATION: "IN_FORMATION",
             L.TRIAL_GRIDLOCK: "GRIDLOCK"}
    from_ = {names.get(int(s), str(int(s))): int(((r["last_state"] == s) & term).sum())
             for s in np.unique(r["last_state"][term])}
    out = {"trials": int(len(done)), "ended": int(done.sum()), "complete": int(comp.sum()),
           "terminated": int(term.sum()), "terminated_from": from_,
           "steps_to_end_mean": float(r["done_step"][done].mean()) if done.any() else None}
    if comp.any():
        out["complete_records"] = {
            "time_s_mean_per_formation": [float(x) for x in r["time"][comp].mean(axis=0)],
            "time_avoidance_s_mean_per_formation":
                [float(x) for x in r["time_avoidance"][comp].mean(axis=0)],
            "assignments_mean_per_formation":
                [float(x) for x in r["assignments"][comp].mean(axis=0)],
            "dist_m_mean_per_vehicle": float(r["dist"][comp].mean())}
    out["auctions_mean"] = float(st["n_auctions"].mean())
    out["invalid_total"] = int(st["n_invalid"].sum())
    out["disagree_total"] = int(st["n_disagree"].sum())
    return out


def trials(args):
    """Batched Monte-Carlo trials at the C3 shape (acl_trial_batch)."""
    dev = torch.device("cuda:0")
    n, B = args.n, args.B
    L_side = 15.0 if n <= 20 else 40.0 * (n / 100.0) ** 0.5
    T, t_admm, admm = admm_table(n, B, L_side, 0, dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    side = 20.0 * (n / 20.0) ** 0.5
    q = workload.nonoverlapping_points(B, n, side, side, 1.0, 1.0, 1.5, gen, dev)
    vel = torch.zeros_like(q)
    fseq = torch.arange(2 * B, dtype=torch.int32, device=dev).view(B, 2)
    modes = {"cbaa": [L.ASSIGN_CBAA], "central": [L.ASSIGN_CENTRAL],
             "both": [L.ASSIGN_CBAA, L.ASSIGN_CENTRAL]}[args.assignment]
    res = {}
    for mode in modes:
        tp = L.default_trial_params()
        tp.ep.assignment = mode
        w = engine.Trial(T, fseq[:8], q[:8], vel[:8], params=tp)  # warm-up (code objects)
        w.run(4)
        torch.cuda.synchronize()
        tr = engine.Trial(T, fseq, q, vel, params=tp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        steps = 0
        while steps < args.max_steps:
            c = min(args.chunk, args.max_steps - steps)
            tr.run(c)
            steps += c
            st = tr.status()              # (one sync per chunk)
            print(f"[trials] mode {mode}: {steps} steps, {int((st['done_step'] >= 0).sum())} "
                  f"of {B} trials ended, {time.perf_counter() - t0:.1f} s", file=sys.stderr,
                  flush=True)
            if (st["done_step"] >= 0).all():
                break
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        r = trial_stats(tr, 2)
        r.update({"value": B / dt, "unit": "trials/s", "seconds": dt, "steps_run": steps,
                  "swarm_steps_per_s": B * steps / dt, "ms_per_step": dt / steps * 1e3})
        res["central" if mode == L.ASSIGN_CENTRAL else "cbaa"] = r
    line = {"metric": f"batched Monte-Carlo trials (supervisor.py state machine, N={n})",
            "B": B, "n": n, "formations_per_trial": 2, "control_dt": 0.01,
            "timings": "supervisor.py:50-57 (hover 5 s, assignment 20 s, gridlock 90 s, trial 600 s), "
                       "form_settle_time 1.5 s, autoauction 1.2 s, tick 50 Hz",
            "dtype": "f64",
            "data": "synthetic: the reference generator's formation groups ('A', 'B'; L=40, "
                    "noncomplete, seeds 0..B-1) with gains designed by acl_admm_solve_batch; "
                    "start positions start.sh-style discs",
            "setup": {"admm_s": t_admm, **admm}, **res}
    if not args.no_cpu:
        line["cpu_baseline"] = cpu_trial_baseline(T, 0, q, args.cpu_budget)
    print(json.dumps(line), flush=True)


def cpu_trial_baseline(T, b, q, budget):
    """oracle/trial_oracle.py on one n=100 trial of the batch for `budget`
    seconds of one core: control steps per second (a trial's steps / that
    rate is its CPU time)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import trial_oracle as TO
    n = T.n
    forms = {}
    for f in (2 * b, 2 * b + 1):
        p = T.p[f].cpu().numpy()
        bits = T.adj[f].cpu().numpy().view(np.uint64)
        adj = np.zeros((n, n), np.uint8)
        for i in range(n):
            for j in range(n):
                adj[i, j] = (int(bits[i][j // 64]) >> (j % 64)) & 1
        E = int(adj.sum())
        off = int(T.gain_off[f].item())
        rec = T.gains[5 * off: 5 * off + 5 * E].view(E, 5).cpu().numpy()
        ii, jj = np.nonzero(adj)
        G = np.zeros((3 * n, 3 * n))
        for k, (r, c) in enumerate([(0, 0), (0, 1), (1, 0), (1, 1), (2, 2)]):
            G[3 * ii + r, 3 * jj + c] = rec[:, k]
        forms[f] = (p, adj, G)
    tp = TO.default_params()
    t = TO.TrialSwarm(n, [2 * b, 2 * b + 1], forms, tp)
    qq = q[b].cpu().numpy()
    vv = np.zeros_like(qq)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < budget and not t.done:
        qq, vv, _, _ = t.step(k, qq, vv)
        k += 1
    dt = time.perf_counter() - t0
    return {"value": k / dt, "unit": "swarm-steps/s", "cores": 1, "kind": "port",
            "sample": f"{k} control steps of trial 0 (n={n}) through oracle/trial_oracle.py "
                      "(C restatement of CBAA / DistCntrl / Safety per vehicle), 1 thread"}


if __name__ == "__main__":
    main()
