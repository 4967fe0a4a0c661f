#!/usr/bin/env python3
"""Headline benchmark: swarm assignment+control solves/sec (N=100 vehicles).

One step = one acl_solve_batch over B swarms (config C3: simform100
noncomplete graphs, every swarm with its own formation -- points, graph and
3x3 gain blocks with the structure admm::Solver::solve gives them, streamed
as 40-byte records per edge -- so the per-swarm gain stream dominates the bytes), i.e.
for every swarm: all vehicles' 2-D Umeyama alignment, CBAA to consensus
(bit-exact, exact fixed-point exit), adoption, one DistCntrl step,
saturation and collision avoidance. Inputs are resident in HBM before the
timed region. With --gpus N (torchrun), every rank solves its own B swarms
(weak scaling, no exchange during the solve) and the step ends with the
RCCL gather of assignments + statistics to rank 0.

Prints ONE JSON line on rank 0 (the driver's contract).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from aclswarm_amd import _lib as L  # noqa: E402
from aclswarm_amd import dist as D  # noqa: E402
from aclswarm_amd import engine, workload  # noqa: E402

METRIC = "swarm assignment+control solves/sec (N=100) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def algorithmic_bytes(w, lo, hi):
    """Bytes the solve of swarms [lo, hi) must move (each input read once,
    each output written once), split by the kernel that owns
    them. Auction kernel, per swarm: fidx 4, q 24n, P_in 2n, P_out 2n,
    status 16; per formation used: p 24n, adjacency bits 8nW. Gain kernel
    (DistCntrl + saturation + the collision test), per swarm: vel 24n,
    u 24n, u_safe 24n, ca n; per formation used: gain_off 8, gains 8 G E_f
    (G = 5 stored planes for ADMM-structured blocks, 9 for general ones).
    The collision-avoidance kernel touches only the vehicles the gain kernel
    listed (none in this workload): 0. Re-reads (the later kernels' q, p,
    adjacency, P_out, the workspace hand-off) are implementation traffic,
    not counted."""
    n = w["n"]
    W = (n + 63) // 64
    Bc = hi - lo
    used = torch.unique(w["fidx"][lo:hi])
    E = w["E"][used].sum().item()
    auction = Bc * (4 + n * (24 + 2 + 2) + 16) + used.numel() * (24 * n + 8 * n * W)
    gain = Bc * n * (24 + 24 + 24 + 1) + used.numel() * 8 + 8 * w["planes"] * E
    return auction, gain, 0, E / used.numel()


def pmc_traffic(n, B, kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/r*_pmc_traffic.json, scripts/gpu_pmc.sh + pmc_summary.py) when
    it was measured on this same configuration; else None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    for f in reversed(files):
        d = json.load(open(f))
        if d["config"]["n"] == n and d["config"]["B_per_gpu"] == B and kernel in d["kernels"]:
            return d["kernels"][kernel]["hbm_bytes"], os.path.relpath(f, ROOT)
    return None, None


def chunk_size(B):
    """acl_solve_batch launches each kernel once over all B swarms."""
    return B


def cpu_baseline(w, out, budget_s, nthreads):
    """Time the CPU restatement (oracle/, the reference's literal 2N-round
    schedule) on a bounded sample of the same swarms; also check parity of
    that sample against the GPU outputs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    n = w["n"]

    def gather(idx):
        fi = w["fidx"][idx].cpu().numpy()
        forms, inv = np.unique(fi, return_inverse=True)
        pts = w["p"][torch.from_numpy(forms).to(w["p"].device)].cpu().numpy()
        adj = w["adj"][torch.from_numpy(forms).to(w["adj"].device)].cpu().numpy().astype(np.uint8)
        G = np.stack([workload.dense_gains_host(w, int(f)) for f in forms])
        q = w["q"][idx].cpu().numpy()
        vel = w["vel"][idx].cpu().numpy()
        Pin = w["P_in"][idx].cpu().numpy().view(np.uint16)
        return inv.astype(np.int32), q, vel, pts, adj, G, Pin

    # calibrate on a few swarms, then size the sample to the time budget
    cal = torch.arange(min(2 * nthreads, w["q"].shape[0]))
    args = gather(cal)
    _, t = O.solve_batch(*args, nthreads=nthreads, early_exit=False)
    per = t / len(cal)
    S = int(max(len(cal), min(4096, budget_s / max(per, 1e-6))))
    S = min(S, w["q"].shape[0])
    idx = torch.arange(S)
    args = gather(idx)
    res, t_lit = O.solve_batch(*args, nthreads=nthreads, early_exit=False)
    res_ee, t_ee = O.solve_batch(*args, nthreads=nthreads, early_exit=True)
    # parity of the sample (GPU ran with the exact fixed-point exit)
    gP = out["P_out"][idx].cpu().numpy().view(np.uint16)
    gst = engine.status_to_numpy(out["status"][idx])
    gus = out["u_safe"][idx].cpu().numpy()
    assign_ok = bool((gP == res["P_out"]).all() and (gP == res_ee["P_out"]).all())
    status_ok = bool((gst["flags"] == res["status"]["flags"]).all()
                     and (gst["eff_rounds"] == res["status"]["eff_rounds"]).all())
    rel = np.abs(gus - res["u_safe"]) / np.maximum(np.abs(res["u_safe"]), 1.0)
    return {
        "value": S / t_lit, "unit": "solves/s", "cores": nthreads, "kind": "port",
        "sample": f"{S} of the benchmark's swarms (n={n}), CPU restatement oracle/ at -O2 "
                  f"-ffp-contract=off, reference schedule of 2N={2 * n} CBAA rounds, "
                  f"{nthreads} threads",
        "value_fixed_point_exit": S / t_ee,
        "parity_sample": {"swarms": S, "assignments_bit_exact": assign_ok,
                          "status_exact": status_ok, "u_safe_max_rel_err": float(rel.max())},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--B", type=int, default=65536, help="swarms per GPU")
    ap.add_argument("--n", type=int, default=100, help="vehicles per swarm")
    ap.add_argument("--formations", type=int, default=0,
                    help="0: every swarm has its own formation; F>0: F shared formations")
    ap.add_argument("--full-rounds", action="store_true",
                    help="run all 2N CBAA rounds instead of stopping at the fixed point")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--gain-planes", type=int, default=5, choices=(5, 9),
                    help="5: ADMM-structured gain blocks (the reference's gains); "
                         "9: general 3x3 blocks")
    ap.add_argument("--no-tile-gains", action="store_true",
                    help="pair kernel reads the row-major records instead of the "
                         "tile-ordered copy made at formation setup (acl_tile_gains)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 7919 * rank)
    t0 = time.time()
    w = workload.simform_workload(args.B, args.n, gen, dev,
                                  F=(args.formations or None), complete=False,
                                  planes=args.gain_planes, seed0=rank * args.B)
    torch.cuda.synchronize()
    t_gen = time.time() - t0
    T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"],
                              w["planes"])
    t_tile = None
    if not args.no_tile_gains and w["planes"] == 5 and args.n <= 128:
        # formation setup (once per formation table, outside the timed solves)
        t0 = time.time()
        T.tile_gains()
        torch.cuda.synchronize()
        t_tile = time.time() - t0
    B, n = args.B, args.n
    out = {
        "P_out": torch.empty((B, n), dtype=torch.int16, device=dev),
        "status": torch.empty((B, 16), dtype=torch.uint8, device=dev),
        "u": torch.empty((B, n, 3), dtype=torch.float64, device=dev),
        "u_safe": torch.empty((B, n, 3), dtype=torch.float64, device=dev),
        "ca_flag": torch.empty((B, n), dtype=torch.uint8, device=dev),
    }
    stream = torch.cuda.current_stream(dev)

    def step():
        engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"], early_exit=not args.full_rounds,
                     out=out, stream=stream.cuda_stream)
        return D.gather_results(out["P_out"], out["status"])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    lib = L.lib()
    lib.acl_internal_kernel_timing(1)   # HIP events around each launch, on its stream
    t0 = time.perf_counter()
    res = None
    for k in range(args.steps):
        evs[k][0].record(stream)
        engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"], early_exit=not args.full_rounds,
                     out=out, stream=stream.cuda_stream)
        evs[k][1].record(stream)
        res = D.gather_results(out["P_out"], out["status"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    call_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    kms = (ctypes.c_double * 3)()
    kcnt = (ctypes.c_int * 3)()
    if lib.acl_internal_kernel_times(kms, kcnt) != 0:
        raise RuntimeError("kernel timing failed")
    lib.acl_internal_kernel_timing(0)
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt_max = float(dt_t.item())
    stats = D.stats_dict(res[1], res[2])

    # algorithmic bytes per launch (the chunk every launch but the last covers)
    ch = chunk_size(B)
    nlaunch = (B + ch - 1) // ch
    a_all, g_all, s_all, e_avg = algorithmic_bytes(w, 0, B)
    c_all = g_all + s_all
    per_launch = {"auction": a_all / nlaunch, "gain": g_all / nlaunch, "ca": s_all / nlaunch}
    kern = {}
    for k, (name, sym) in enumerate((("auction", "acl_amd::solve_kernel"),
                                     ("gain", "acl_amd::gain_pair_kernel<%s>" % ("true" if t_tile is not None else "false")
                                      if w["planes"] == 5
                                      and os.environ.get("ACLSWARM_AMD_GAIN_PAIR", "1") != "0"
                                      else f"acl_amd::gain_kernel<{w['planes']}>"),
                                     ("ca", "acl_amd::ca_kernel"))):
        avg = kms[k] / max(kcnt[k], 1)
        ach = per_launch[name] / (avg * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(n, B, sym) if args.formations == 0 else (None, None)
        kern[name] = {"kernel": sym, "launches_per_step": nlaunch, "avg_launch_ms": avg,
                      "bytes_per_launch": per_launch[name], "achieved_GBs": ach,
                      "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc}
    # the roofline is an HBM roofline: its kernel is the one that carries the
    # path's HBM stream (the gain kernel, ~98% of the algorithmic bytes); the
    # auction kernel's own line in `kernels` shows it is not HBM-bound
    dom = max(kern, key=lambda k: kern[k]["bytes_per_launch"])
    pipe_ach = (a_all + c_all) / (call_ms * 1e-3) / 1e9
    line = {
        "metric": METRIC,
        "value": world * B / dt_max,
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt_max * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": "simform100_nc (config C3): noncomplete random formation graphs, "
                        + ("a unique formation (points, graph, gain blocks) per swarm"
                           if not args.formations else f"{args.formations} shared formations"),
            "formations": "the reference generator (generate_random_formation.py:59-80, "
                          "L=40, h=2, min_dist=2) after np.random.seed(s), "
                          f"s = {rank * args.B}..{rank * args.B + (args.formations or args.B) - 1}, "
                          "reproduced bit-exact on the device",
            "n": n, "B_per_gpu": B, "B_total": world * B,
            "edges_per_formation_avg": e_avg,
            "cbaa": "all 2N rounds" if args.full_rounds else "exact fixed-point exit",
            "parallelism": f"swarm-sharded x{world}",
            "gains": ("synthetic ADMM-structured blocks [a b 0; c d 0; 0 0 e] "
                      "(solver.cpp:49-77), 5-entry records = 40 B/edge" if w["planes"] == 5 else
                      "synthetic random 3x3 blocks, 9 planes = 72 B/edge"),
            "gain_layout": ("tile-ordered copy (acl_tile_gains, formation setup: %.3f s, "
                            "not timed)" % t_tile) if t_tile is not None else "row-major records",
        },
        "roofline": {
            "bound": "hbm", "achieved": kern[dom]["achieved_GBs"], "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": kern[dom]["frac"], "traffic": kern[dom]["traffic"],
            "traffic_source": kern[dom]["traffic_source"],
            "kernel": kern[dom]["kernel"], "avg_launch_ms": kern[dom]["avg_launch_ms"],
            "bytes_per_launch": kern[dom]["bytes_per_launch"],
            "note": "kernel carrying the HBM stream (most algorithmic bytes); the auction "
                    "kernel (LDS-resident CBAA) is VALU/LDS-issue bound, HBM frac in "
                    "`kernels.auction`; whole call in `pipeline`; see DESIGN.md",
            "kernels": kern,
            "pipeline": {"what": "whole acl_solve_batch call (auction, gain, ca kernels)",
                         "call_ms": call_ms, "bytes": a_all + c_all,
                         "achieved_GBs": pipe_ach, "frac": pipe_ach / HBM_PEAK_GBS},
        },
        "stats": stats,
        "gen_s": t_gen,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        nthreads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        nthreads = max(1, min(nthreads, os.cpu_count() or 1))
        line["cpu_baseline"] = cpu_baseline(w, out, args.cpu_budget, nthreads)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
