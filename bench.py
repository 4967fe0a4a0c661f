#!/usr/bin/env python3
"""Headline benchmark: swarm assignment+control solves/sec (N=100 vehicles).

One step = one acl_solve_batch over B swarms per GPU (config C3 by default:
simform100 noncomplete graphs, every swarm with its own formation -- points,
graph and 3x3 gain blocks with the structure admm::Solver::solve gives them,
streamed as 40-byte records per edge -- so the per-swarm gain stream
dominates the bytes), i.e. for every swarm: all vehicles' 2-D Umeyama
alignment, CBAA to consensus (bit-exact, exact fixed-point exit), adoption,
one DistCntrl step, saturation and collision avoidance, then the gather of
every rank's assignments + status records to rank 0 (dist.gather_results).
Inputs are resident in HBM before the timed region.

--gpus N: one process per GPU. Launched by torchrun (WORLD_SIZE set) each
rank solves its own B swarms (weak scaling, no exchange during the solve);
launched directly with N > 1, this script starts the N ranks itself (child
processes, before anything touches a GPU) and exits with rank 0's status.
--config c2 / c4 run the other single-GPU shards (simform20 complete,
B=4096; simform500, B=2048 per GPU = C4's 16384 over 8 GPUs); --config c5
the batched ADMM gain design (N=100, F=1024 formations per GPU, MFMA
roofline, CPU restatement baseline).
--dry-run exercises the launch + gather path on the CPU (gloo, synthetic
outputs, no solve) for the multi-process tests.

Prints ONE JSON line on rank 0 (the driver's contract).
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "swarm assignment+control solves/sec (N=100) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

# per-GPU shards of the BASELINE.json configs
CONFIGS = {
    "c2": dict(n=20, B=4096, L=15.0, complete=True,
               name="simform20_fc (config C2): complete formation graphs"),
    "c3": dict(n=100, B=65536, L=40.0, complete=False,
               name="simform100_nc (config C3): noncomplete random formation graphs"),
    "c4": dict(n=500, B=2048, L=90.0, complete=False,
               name="simform500_nc (config C4 shard: 2048 of 16384 swarms per GPU): "
                    "noncomplete random formation graphs, u16 vehicle indices"),
    "c5": dict(n=100, B=1024, L=40.0, complete=False,
               name="batched ADMM formation-gain design (config C5): N=100, F=1024 "
                    "simform100 noncomplete formations per GPU"),
}
METRIC_C5 = "batched ADMM formation-gain designs/sec (N=100, F=1024); % fp64 MFMA roofline"
FP64_MATRIX_PEAK_TF = 78.6  # MI355X fp64 matrix, AMD spec (the microarch guide has no fp64 row)
# the instruction's ceiling measured on the box: v_mfma_f64_16x16x4f64 chains
# without memory traffic (scripts/mfma_f64_peak.hip, profiles/r4_mfma_f64_peak.txt)
FP64_MFMA_MEASURED_TF = 48.6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """One child process per rank (nothing here has touched a GPU), the
    torchrun environment contract; returns rank 0's exit status (or the first
    failure)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


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
    import torch
    n = w["n"]
    W = (n + 63) // 64
    Bc = hi - lo
    used = torch.unique(w["fidx"][lo:hi])
    E = w["E"][used].sum().item()
    auction = Bc * (4 + n * (24 + 2 + 2) + 16) + used.numel() * (24 * n + 8 * n * W)
    gain = Bc * n * (24 + 24 + 24 + 1) + used.numel() * 8 + 8 * w["planes"] * E
    return auction, gain, 0, E / used.numel()


def graph_group(requested, steps):
    """Steps captured per HIP graph: the largest divisor of `steps` not above
    `requested` (at least 1), so that exactly `steps` steps are timed."""
    top = max(1, min(int(requested), int(steps)))
    return max(g for g in range(1, top + 1) if steps % g == 0)


def committed_profile(prefix, n, B, kernel):
    """The newest committed PMC summary profiles/r*_{prefix}.json measured on
    this same configuration that has `kernel`; (entry, path) or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{prefix}.json")))
    for f in reversed(files):
        d = json.load(open(f))
        c = d.get("config", {})
        if c.get("n") == n and c.get("B_per_gpu") == B and kernel in d.get("kernels", {}):
            return d["kernels"][kernel], os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(w, out, budget_s, nthreads):
    """Time the CPU restatement (oracle/, -O3 -ffp-contract=off, the
    reference's literal 2N-round schedule) on bounded samples of the same
    swarms, on all `nthreads` host threads and on one; also check the
    sample's parity against the GPU outputs."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    from aclswarm_amd import engine, workload
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

    def note(msg):  # progress on stderr (a long CPU leg must not look hung)
        print(f"[bench] cpu_baseline: {msg}", file=sys.stderr, flush=True)

    Btot = w["q"].shape[0]
    # calibrate on one swarm per thread, then size the samples to the time budget
    cal = torch.arange(min(nthreads, Btot))
    args = gather(cal)
    note(f"calibrating on {len(cal)} swarms")
    _, t = O.solve_batch(*args, nthreads=nthreads, early_exit=False, margin=False)
    per = t / len(cal)
    S = int(max(len(cal), min(4096, 0.6 * budget_s / max(per, 1e-6))))
    S = min(S, Btot)
    idx = torch.arange(S)
    args = gather(idx)
    # timed: the reference's work (literal 2N rounds, no margin bookkeeping);
    # the fixed-point-exit run carries the margin for the parity check
    note(f"{S} swarms, literal 2N rounds, {nthreads} threads")
    res, t_lit = O.solve_batch(*args, nthreads=nthreads, early_exit=False, margin=False)
    note(f"{S} swarms, fixed-point exit with margins")
    res_ee, t_ee = O.solve_batch(*args, nthreads=nthreads, early_exit=True)
    # one core: a smaller sample of the same swarms
    S1 = int(max(1, min(S, 0.25 * budget_s / max(per * nthreads, 1e-6))))
    a1 = gather(torch.arange(S1))
    note(f"{S1} swarms on 1 thread")
    _, t1 = O.solve_batch(*a1, nthreads=1, early_exit=False, margin=False)
    # parity of the sample (GPU ran with the exact fixed-point exit)
    gP = out["P_out"][idx].cpu().numpy().view(np.uint16)
    gst = engine.status_to_numpy(out["status"][idx])
    gus = out["u_safe"][idx].cpu().numpy()
    assign_ok = bool((gP == res["P_out"]).all() and (gP == res_ee["P_out"]).all())
    status_ok = bool((gst["flags"] == res_ee["status"]["flags"]).all()
                     and (gst["eff_rounds"] == res["status"]["eff_rounds"]).all()
                     and (gst["eff_rounds"] == res_ee["status"]["eff_rounds"]).all()
                     and (gst["margin"] == res_ee["status"]["margin"]).all())
    rel = np.abs(gus - res["u_safe"]) / np.maximum(np.abs(res["u_safe"]), 1.0)
    return {
        "value": S / t_lit, "unit": "solves/s", "cores": nthreads, "kind": "port",
        "sample": f"{S} of the benchmark's swarms (n={n}) on {nthreads} threads and the "
                  f"first {S1} on 1 thread; CPU restatement oracle/ at -O3 "
                  f"-ffp-contract=off, reference schedule of 2N={2 * n} CBAA rounds",
        "value_1core": S1 / t1,
        "value_fixed_point_exit_with_margin": S / t_ee,
        "parity_sample": {"swarms": S, "assignments_bit_exact": assign_ok,
                          "status_and_margin_exact": status_ok,
                          "u_safe_max_rel_err": float(rel.max())},
    }


def cpu_baseline_admm(pts, adj, G, its, budget_s):
    """The build's CPU ADMM restatement (oracle/admm_oracle.py: the
    codegen's algebra, eigh-based PSD projection) on a bounded sample of the
    same formations, one BLAS thread; checks the sample's gains and iteration
    counts against the GPU."""
    import numpy as np
    from threadpoolctl import threadpool_limits
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import admm_oracle as AO

    def note(msg):
        print(f"[bench] cpu_baseline: {msg}", file=sys.stderr, flush=True)

    F = pts.shape[0]
    # the sample strides over the whole batch (acl_admm_solve_batch runs it
    # in chunks of 512 formations): both ends of every chunk first, then a
    # stride coprime with F
    order = []
    for f in [0, F - 1, F // 2 - 1, F // 2] + [(k * 389) % F for k in range(1, F)]:
        if 0 <= f < F and f not in order:
            order.append(f)
    res, t = [], 0.0
    with threadpool_limits(1):
        for f in order:
            note(f"ADMM formation {f} on 1 thread")
            t0 = time.perf_counter()
            A, it = AO.design_3d(pts[f].cpu().numpy(), adj[f].cpu().numpy())
            t += time.perf_counter() - t0
            res.append((f, A, it))
            if t > budget_s:
                break
    S = len(res)
    err = max(float(np.abs(G[f].cpu().numpy() - A).max() / max(np.abs(A).max(), 1e-300))
              for f, A, _ in res)
    it_ok = all(tuple(int(x) for x in its[f].tolist()) == tuple(it) for f, _, it in res)
    idx = sorted(f for f, _, _ in res)
    return {"value": S / t, "unit": "formations/s", "cores": 1, "kind": "port",
            "sample": f"{S} of the benchmark's formations (n={pts.shape[1]}) spread over the "
                      f"whole batch (indices {idx[0]}..{idx[-1]}, both 512-formation chunks) "
                      "on one thread; CPU restatement oracle/admm_oracle.py (the codegen's ADMM "
                      "algebra with a dense eigh PSD projection)",
            "reference_codegen_s_per_formation": 41.9,
            "parity_sample": {"formations": S, "gains_max_rel_err": err,
                              "iterations_equal": it_ok}}


def bench_c5(args, world, rank, local):
    """Config C5: one step = one acl_admm_solve_batch over F formations per
    GPU (formations shard across ranks; weak scaling)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from aclswarm_amd import _lib as L
    from aclswarm_amd import engine, workload
    cfg = CONFIGS["c5"]
    n, F = cfg["n"], (args.B or cfg["B"])
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    pts, adjb = workload.reference_formations(F, n, cfg["L"], cfg["complete"], rank * F, dev)
    adj = adjb.to(torch.float64)
    torch.cuda.synchronize()
    lib = L.lib()
    # GEMM flops of one batch, counted on the device in an untimed pass
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    lib.acl_internal_admm_flop_counter(ctypes.c_void_p(counter.data_ptr()))
    G, its = engine.admm_design(pts, adj)
    torch.cuda.synchronize()
    lib.acl_internal_admm_flop_counter(ctypes.c_void_p(0))
    flops = float(counter.item())
    for _ in range(max(0, args.warmup - 1)):
        G, its = engine.admm_design(pts, adj)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs[k][0].record(stream)
        G, its = engine.admm_design(pts, adj)
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    batch_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt_max = float(dt_t.item())
    itn = its.cpu()
    ach = flops / (batch_ms * 1e-3) / 1e12
    line = {
        "metric": METRIC_C5, "value": world * F / dt_max, "unit": "formations/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt_max * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": cfg["name"],
                   "formations": "the reference generator (generate_random_formation.py:59-80, "
                                 f"L={cfg['L']:g}, h=2, min_dist=2, fc=False) after "
                                 f"np.random.seed(s), s = {rank * F}..{rank * F + F - 1} per rank",
                   "n": n, "F_per_gpu": F, "F_total": world * F,
                   "parallelism": f"formation-sharded x{world}"},
        "roofline": {"bound": "mfma", "scope": "batch",
                     "what": "the batch's fp64 GEMM flops (counted per tile on the device, "
                             "symmetric products as upper-triangle tiles) / batch time",
                     "achieved": ach, "peak": FP64_MATRIX_PEAK_TF, "unit": "TFLOP/s",
                     "frac": ach / FP64_MATRIX_PEAK_TF, "traffic": None,
                     "measured_instruction_peak": FP64_MFMA_MEASURED_TF,
                     "frac_of_measured_peak": ach / FP64_MFMA_MEASURED_TF,
                     "measured_peak_source": "profiles/r4_mfma_f64_peak.txt (scripts/mfma_f64_peak.hip)",
                     "gemm_flops_per_batch": flops, "batch_ms_events": batch_ms},
        "iters_xy": {int(k): int(v) for k, v in zip(*torch.unique(itn[:, 0], return_counts=True))},
        "iters_z": {int(k): int(v) for k, v in zip(*torch.unique(itn[:, 1], return_counts=True))},
        "finite": bool(torch.isfinite(G).all().item()),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_admm(pts, adj, G, its, args.cpu_budget)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def dry_run(args, world, rank):
    """CPU/gloo rehearsal of the multi-rank path: synthetic outputs of the
    configured shard size, the same gather and max-over-ranks timing; no
    solve, so `value` measures the plumbing only (dry_run: true)."""
    import torch
    import torch.distributed as dist
    from aclswarm_amd import dist as D
    cfg = CONFIGS[args.config]
    B = args.B or cfg["B"]
    n = cfg["n"]
    if world > 1:
        dist.init_process_group("gloo")
    P = torch.arange(n, dtype=torch.int16).expand(B, n).contiguous()
    st = torch.zeros((B, 16), dtype=torch.uint8)
    st[:, 0] = 0x07
    st[:, 4] = 3 + rank
    st[:, 12:16] = torch.tensor([0.5], dtype=torch.float32).view(torch.uint8)
    for _ in range(args.warmup):
        D.gather_results(P, st)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = D.gather_results(P, st)
    if world > 1:
        dist.barrier()
    dt = torch.tensor([(time.perf_counter() - t0) / args.steps], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": world * B / float(dt.item()), "unit": "solves/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": float(dt.item()) * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic", "dry_run": True,
            "config": {"workload": cfg["name"], "n": n, "B_per_gpu": B, "B_total": world * B,
                       "parallelism": f"swarm-sharded x{world}"},
            "gathered": {"swarms": int(res[0].shape[0]), "status_records": int(res[1].shape[0])},
            "stats": D.stats_dict(res[2], res[3])}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--B", type=int, default=0, help="swarms per GPU (default: the config's)")
    ap.add_argument("--formations", type=int, default=0,
                    help="0: every swarm has its own formation; F>0: F shared formations")
    ap.add_argument("--full-rounds", action="store_true",
                    help="run all 2N CBAA rounds instead of stopping at the fixed point")
    ap.add_argument("--cpu-budget", type=float, default=16.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--gain-planes", type=int, default=5, choices=(5, 9),
                    help="5: ADMM-structured gain blocks (the reference's gains); "
                         "9: general 3x3 blocks")
    ap.add_argument("--graph", action="store_true",
                    help="time the step (solve + device-side stats) as a captured HIP graph "
                         "(launch-bound configurations such as C2; one GPU)")
    ap.add_argument("--graph-steps", type=int, default=10,
                    help="with --graph: steps captured per graph (the largest divisor of --steps "
                         "not above it); the K timed steps are K / G replays, with one event "
                         "pair around them all (per-step events add a gap at every replay)")
    ap.add_argument("--no-persistent", action="store_true",
                    help="solve with acl_solve_args_t::ws_persistent = 0 (a memset of the "
                         "collision-list counters per call; A/B of ABI 10's persistent workspace)")
    ap.add_argument("--margin", action="store_true",
                    help="time the headline with the decision margin tracked (default: the "
                         "reference's work only, acl_solve_args_t::skip_margin; the margin-on "
                         "rate is measured beside it either way)")
    ap.add_argument("--no-ca-probe", action="store_true",
                    help="skip the crowded (collision-avoidance) probe reported beside the headline")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo rehearsal of the launch + gather path (no GPU, no solve)")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return spawn_ranks(args.gpus)  # before any GPU call in this process
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.dry_run:
        return dry_run(args, world, rank)
    if args.config == "c5":
        return bench_c5(args, world, rank, local)

    import numpy as np
    import torch
    import torch.distributed as dist
    from aclswarm_amd import _lib as L
    from aclswarm_amd import dist as D
    from aclswarm_amd import engine, workload

    cfg = CONFIGS[args.config]
    n, B = cfg["n"], (args.B or cfg["B"])
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 7919 * rank)
    t0 = time.time()
    w = workload.simform_workload(B, n, gen, dev, F=(args.formations or None), L=cfg["L"],
                                  complete=cfg["complete"], planes=args.gain_planes,
                                  seed0=rank * B)
    torch.cuda.synchronize()
    t_gen = time.time() - t0
    T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"],
                              w["planes"])
    stream = torch.cuda.current_stream(dev)
    out = {
        "P_out": torch.empty((B, n), dtype=torch.int16, device=dev),
        "status": torch.empty((B, 16), dtype=torch.uint8, device=dev),
        "u": torch.empty((B, n, 3), dtype=torch.float64, device=dev),
        "u_safe": torch.empty((B, n, 3), dtype=torch.float64, device=dev),
        "ca_flag": torch.empty((B, n), dtype=torch.uint8, device=dev),
    }

    def solve(margin):
        engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"], early_exit=not args.full_rounds,
                     out=out, stream=stream.cuda_stream, margin=margin,
                     persistent=not args.no_persistent)

    lib = L.lib()

    graph_steps = [0]  # steps per captured graph (0: eager launches)

    def timed(margin, ktimes):
        """W warmup + K timed steps (barrier + synchronize on both sides),
        the max over ranks; per-launch kernel times when ktimes"""
        for _ in range(args.warmup):
            solve(margin)
            D.gather_results(out["P_out"], out["status"])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        if ktimes:
            lib.acl_internal_kernel_timing(1)   # HIP events around each launch, on its stream
        t0 = time.perf_counter()
        res = None
        for k in range(args.steps):
            evs[k][0].record(stream)
            solve(margin)
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
        if ktimes:
            if lib.acl_internal_kernel_times(kms, kcnt) != 0:
                raise RuntimeError("kernel timing failed")
            lib.acl_internal_kernel_timing(0)
        if args.graph and world == 1:
            # the same step captured once into a HIP graph and replayed: the
            # per-kernel times above come from the eager pass, the step time from
            # the replays (no host launch overhead between the step's kernels)
            gs = torch.cuda.Stream()  # (capture needs a non-default stream)
            gs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(gs):  # one eager step on the capture stream first
                engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"],
                             early_exit=not args.full_rounds, out=out, stream=gs.cuda_stream,
                             margin=margin, persistent=not args.no_persistent)
                D.gather_results(out["P_out"], out["status"])
            torch.cuda.synchronize()
            G = graph_group(args.graph_steps, args.steps)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=gs):
                for _ in range(G):
                    engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"],
                                 early_exit=not args.full_rounds, out=out, stream=gs.cuda_stream,
                                 margin=margin, persistent=not args.no_persistent)
                    gres = D.gather_results(out["P_out"], out["status"])
            with torch.cuda.stream(gs):
                graph.replay()
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            with torch.cuda.stream(gs):
                ev0.record(gs)
                for k in range(args.steps // G):
                    graph.replay()
                ev1.record(gs)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            call_ms = ev0.elapsed_time(ev1) / args.steps
            graph_steps[0] = G
            res = gres
        dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        return float(dt_t.item()), call_ms, kms, kcnt, res

    # the headline: the reference's work (no decision-margin bookkeeping,
    # skip_margin) unless --margin; then the other mode on the same swarms,
    # whose margin-on run gives the swarm statistics (fragile counts, min margin)
    # (the margin-on run last: its outputs stay in `out` for the CPU check)
    if args.margin:
        dt_alt, _, _, _, _ = timed(False, False)
        dt_max, call_ms, kms, kcnt, res = timed(True, True)
    else:
        dt_max, call_ms, kms, kcnt, _ = timed(False, True)
        dt_alt, _, _, _, res = timed(True, False)
    margin_line = {
        "headline_tracks_margin": bool(args.margin),
        "value_margin_on": world * B / (dt_max if args.margin else dt_alt),
        "value_margin_off": world * B / (dt_alt if args.margin else dt_max),
        "ms_per_step_margin_on": (dt_max if args.margin else dt_alt) * 1e3,
        "what": "decision-margin bookkeeping (include/aclswarm_amd.h, a parity diagnostic the "
                "reference does not compute) on / off (acl_solve_args_t::skip_margin); the same "
                "assignments, rounds and commands bit for bit (tests/test_gpu_fused.py::"
                "test_skip_margin_same_outcome); `stats` comes from the margin-on run",
    }
    stats = D.stats_dict(res[2], res[3])

    # collision-avoidance probe: the same swarms crowded (positions scaled by
    # 0.3 about each swarm's centre, most vehicles inside the 1.5 m avoidance
    # radius), so the sector algebra of Safety::collisionAvoidance
    # (safety.cpp:412-541) runs for most vehicles; reported beside the
    # headline, which is the reference's spacing (start.sh discs, no CA)
    ca_probe = None
    if not args.no_ca_probe:
        qc = w["q"].clone()
        cen = qc[:, :, :2].mean(dim=1, keepdim=True)
        qc[:, :, :2] = cen + 0.3 * (qc[:, :, :2] - cen)
        outc = {k: torch.empty_like(v) for k, v in out.items()}

        def solve_c():
            engine.solve(T, w["fidx"], qc, w["vel"], w["P_in"], early_exit=not args.full_rounds,
                         out=outc, stream=stream.cuda_stream, margin=args.margin)
        solve_c()
        torch.cuda.synchronize()
        lib.acl_internal_kernel_timing(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(3):
            solve_c()
        e1.record(stream)
        torch.cuda.synchronize()
        kms_c = (ctypes.c_double * 3)()
        kcnt_c = (ctypes.c_int * 3)()
        if lib.acl_internal_kernel_times(kms_c, kcnt_c) != 0:
            raise RuntimeError("kernel timing failed")
        lib.acl_internal_kernel_timing(0)
        ms_c = e0.elapsed_time(e1) / 3
        sc = D.stats_dict(*D.swarm_stats(outc["status"]))
        ca_probe = {"what": "the benchmark's swarms with positions scaled by 0.3 about each "
                            "swarm's centre (collision avoidance active)",
                    "call_ms": ms_c, "value_1gpu": B / (ms_c * 1e-3),
                    "kernel_ms": {k: kms_c[i] / max(kcnt_c[i], 1)
                                  for i, k in enumerate(("auction", "gain", "ca"))},
                    "ca_active_swarms": sc["ca_active"], "ca_vehicles": sc["ca_vehicles"]}
        del outc, qc

    # algorithmic bytes per launch (every kernel is one launch over all B).
    # 5-plane records: the control phase runs inside the auction's workgroups
    # (one fused launch carries every byte; n > 128: the wide kernel's
    # wide_control); the directed gain kernel then runs only for swarms with
    # per-vehicle rows (none here).
    a_all, g_all, s_all, e_avg = algorithmic_bytes(w, 0, B)
    fused = w["planes"] == 5
    mg = "true" if args.margin else "false"  # the timed kernels' margin template argument
    if fused:
        per_launch = {"auction": a_all + g_all, "gain": 0, "ca": s_all}
        auction_sym = (f"acl_amd::auction_kernel<1, 128, true, false, {mg}>" if n <= 32 else
                       f"acl_amd::auction_kernel<1, 256, true, false, {mg}>" if n <= 64 else
                       f"acl_amd::auction_kernel<2, 512, true, false, {mg}>" if n <= 128 else
                       f"acl_amd::solve_wide_kernel<true, false, {mg}>")
        gain_sym = (f"acl_amd::gain_kernel<{w['planes']}, false, 256>" if n <= 128 else
                    f"acl_amd::gain_kernel<{w['planes']}, false, 1024>")
        align_sym = "acl_amd::align_kernel<2>" if n <= 128 else "acl_amd::align_wide_kernel"
    else:
        per_launch = {"auction": a_all, "gain": g_all, "ca": s_all}
        auction_sym = ((f"acl_amd::auction_kernel<1, 128, false, false, {mg}>" if n <= 32 else
                        f"acl_amd::auction_kernel<1, 256, false, false, {mg}>" if n <= 64 else
                        f"acl_amd::auction_kernel<2, 512, false, false, {mg}>") if n <= 128
                       else "acl_amd::solve_wide_kernel")
        # n > 128: the control law is the directed walk on 1 024-thread workgroups
        gain_sym = ("acl_amd::gain_pair_kernel<false, false>" if w["planes"] == 5 and n <= 128
                    else f"acl_amd::gain_kernel<{w['planes']}, false, 1024>" if n > 128
                    else f"acl_amd::gain_kernel<{w['planes']}, false, 256>")
    kern = {}
    for k, (name, sym) in enumerate((("auction", auction_sym), ("gain", gain_sym),
                                     ("ca", "acl_amd::ca_pair_kernel" if n <= 128
                                      else "acl_amd::ca_kernel"))):
        avg = kms[k] / max(kcnt[k], 1)
        ach = per_launch[name] / (avg * 1e-3) / 1e9
        pm, src = (committed_profile("pmc_traffic", n, B, sym) if args.formations == 0
                   else (None, None))
        kern[name] = {"kernel": sym, "launches_per_step": 1, "avg_launch_ms": avg,
                      "bytes_per_launch": per_launch[name], "achieved_GBs": ach,
                      "frac": ach / HBM_PEAK_GBS,
                      "traffic": pm["hbm_bytes"] if pm else None, "traffic_source": src}
    if fused:
        kern["auction"]["what"] = ("fused: CBAA, adoption, then DistCntrl + saturation + the "
                                   "collision test in the same workgroup; for n > 64 the "
                                   f"alignment runs as its own launch just before ({align_sym}), "
                                   "timed with it")
        kern["gain"]["what"] = "directed gain kernel for swarms with per-vehicle rows only"
    # the auction kernel is bound by an issue port, not HBM: its utilisation
    # from the committed SQ counters of the same configuration
    # (scripts/gpu_pmc_auction.sh -> scripts/pmc_auction_summary.py).
    # VALU: SQ_ACTIVE_INST_VALU x 4 / SIMD-cycles (fp64 VALU ops occupy a
    # SIMD for several cycles, which instruction counts under-read);
    # SALU and LDS: instructions per CU-cycle at one issue per cycle.
    iss, isrc = committed_profile("pmc_auction", n, B, auction_sym)
    if iss:
        kern["auction"]["issue"] = dict(iss, source=isrc)
        # the auction's own roofline: its busiest port as profiled (a ratio
        # of the profiled run's counters to its own kernel time; this run's
        # `avg_launch_ms` also spans the alignment launch)
        scale = 1.0
        ports = {}
        if "valu_active" in iss:
            ports["valu-active"] = iss["valu_active"] * scale
        for p in ("salu", "lds"):
            if p + "_issue_frac" in iss:
                ports[p + "-issue"] = iss[p + "_issue_frac"] * scale
        if ports:
            top = max(ports, key=ports.get)
            kern["auction"]["roofline"] = {"bound": top, "frac": ports[top],
                                           "ports": ports, "source": isrc}
    pipe_bytes = a_all + g_all + s_all
    pipe_ach = pipe_bytes / (call_ms * 1e-3) / 1e9
    tr = [kern[k]["traffic"] for k in (("auction",) if fused else ("auction", "gain"))]
    if fused and n > 64:
        # the alignment launch that precedes the fused one (its inputs and the
        # workspace round trip of its results) is in the same timed window
        am, _ = (committed_profile("pmc_traffic", n, B, align_sym)
                 if args.formations == 0 else (None, None))
        tr.append(am["hbm_bytes"] if am else None)
        kern["auction"]["traffic_align_kernel"] = am["hbm_bytes"] if am else None
    pipe_traffic = sum(tr) if all(x is not None for x in tr) else None
    pipe_traffic_src = kern["auction"]["traffic_source"] if pipe_traffic is not None else None
    gk = kern["auction" if fused else "gain"]
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
            "workload": cfg["name"] + (", a unique formation (points, graph, gain blocks) per swarm"
                                       if not args.formations else
                                       f", {args.formations} shared formations"),
            "formations": "the reference generator (generate_random_formation.py:59-80, "
                          f"L={cfg['L']:g}, h=2, min_dist=2, fc={cfg['complete']}) after "
                          f"np.random.seed(s), s = {rank * B}..{rank * B + (args.formations or B) - 1}"
                          " per rank, reproduced bit-exact on the device",
            "n": n, "B_per_gpu": B, "B_total": world * B,
            "edges_per_formation_avg": e_avg,
            "cbaa": "all 2N rounds" if args.full_rounds else "exact fixed-point exit",
            "decision_margin": ("tracked" if args.margin else
                                "not tracked in the timed steps (skip_margin); see `margin`"),
            "parallelism": f"swarm-sharded x{world}",
            "launch": (f"captured HIP graph of {graph_steps[0]} step(s) (solve + device-side "
                       "stats per step), replayed; one event pair around the timed replays"
                       if args.graph and world == 1 else "eager launches on one stream"),
            "gains": ("synthetic ADMM-structured blocks [a b 0; c d 0; 0 0 e] "
                      "(solver.cpp:49-77), 5-entry records = 40 B/edge" if w["planes"] == 5 else
                      "synthetic random 3x3 blocks, 9 planes = 72 B/edge"),
            "gain_layout": "row-major 40-byte records (no formation-setup re-layout)",
            "kernels": ("the alignment launch (n > 64), one fused auction + control launch (+ "
                        "the collision-avoidance launch over the listed vehicles)" if fused else
                        "auction launch, gain launch, collision-avoidance launch"),
        },
        "roofline": {
            "bound": "hbm", "scope": "pipeline",
            "what": "whole acl_solve_batch call (every kernel of the solve): algorithmic "
                    "bytes (SURVEY.md 8d, `kernels.*.bytes_per_launch`) / call time "
                    "(HIP events on the solve's stream)",
            "achieved": pipe_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": pipe_ach / HBM_PEAK_GBS,
            "traffic": pipe_traffic, "traffic_source": pipe_traffic_src,
            "call_ms": call_ms, "bytes_per_call": pipe_bytes,
            "stream_kernel": {"kernel": gk["kernel"], "achieved": gk["achieved_GBs"],
                            "frac": gk["frac"], "avg_launch_ms": gk["avg_launch_ms"],
                            "bytes_per_launch": gk["bytes_per_launch"],
                            "traffic": gk["traffic"], "traffic_source": gk["traffic_source"]},
            "note": "frac is the whole call's HBM fraction (the north-star quantity); the "
                    "gain stream carries nearly all algorithmic bytes (" +
                    ("inside the fused auction launch" if fused else "`gain_kernel`") +
                    "); the CBAA rounds are issue-port bound (kernels.auction.roofline)",
            "kernels": kern,
        },
        "margin": margin_line,
        "ca_probe": ca_probe,
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
    return 0


if __name__ == "__main__":
    sys.exit(main())
