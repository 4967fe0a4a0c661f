"""Config C5: batched ADMM formation-gain design, N=100, B=1024 formations
(BASELINE.json configs[4]), timed on one GPU.

Prints one JSON line: formations/s, ms per batch, the GEMM flops the batch
executed (counted on the device per tile), achieved fp64 TFLOP/s vs the
MI355X fp64 matrix peak, and the iteration histogram.
Usage: python scripts/admm_bench.py [--F 1024] [--n 100] [--reps 3]
"""
import argparse
import ctypes as ct
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from aclswarm_amd import _lib as L  # noqa: E402
from aclswarm_amd import engine, workload  # noqa: E402

FP64_MATRIX_PEAK_TF = 78.6  # MI355X fp64 matrix (AMD spec; not in the microarch guide)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--F", type=int, default=1024)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    n = a.n
    Lside = 15.0 if n <= 20 else 40.0 * (n / 100.0) ** 0.5
    pts = workload.nonoverlapping_points(a.F, n, Lside, Lside, 0.0, 2.0, 2.0, gen, dev)
    adj = workload.random_adjacency(a.F, n, False, gen, dev).to(torch.float64)
    torch.cuda.synchronize()
    lib = L.lib()
    engine.admm_design(pts[:8], adj[:8])  # warm up (allocations, code objects)
    torch.cuda.synchronize()
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    times = []
    for r in range(a.reps):
        counter.zero_()
        lib.acl_internal_admm_flop_counter(ct.c_void_p(counter.data_ptr()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        G, its = engine.admm_design(pts, adj)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        lib.acl_internal_admm_flop_counter(ct.c_void_p(0))
    t = min(times)
    flops = float(counter.item())
    itn = its.cpu()
    res = {
        "metric": "batched ADMM formation-gain designs/sec (N=%d)" % n,
        "value": a.F / t, "unit": "formations/s", "F": a.F, "n": n,
        "ms_per_batch": 1e3 * t, "all_ms": [1e3 * x for x in times],
        "dtype": "f64",
        "gemm_flops": flops,
        "mfma": {"achieved_TFs": flops / t / 1e12, "peak_TFs": FP64_MATRIX_PEAK_TF,
                 "frac": flops / t / 1e12 / FP64_MATRIX_PEAK_TF},
        "iters_xy": {int(k): int(v) for k, v in zip(*torch.unique(itn[:, 0], return_counts=True))},
        "iters_z": {int(k): int(v) for k, v in zip(*torch.unique(itn[:, 1], return_counts=True))},
        "finite": bool(torch.isfinite(G).all().item()),
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
