#!/usr/bin/env python3
"""Per-tally latency of the facade's bid-exchange mode (ABI 11): fleets of
exchange-mode Auctioneers (tests/facade_driver.cpp facade_exchange) on one
bus, every completed bid iteration tallied on the GPU by
acl_cbaa_step_batch (V = 1, host-synchronous). The reference's vehicles tick
their Auctioneer every 1 ms (coordination_ros.cpp:146-153); one tally here
must fit well inside that. Prints one JSON line per fleet size.

Usage (GPU box): python scripts/exchange_latency.py
"""
import ctypes as ct
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import helpers as H  # noqa: E402

LIB = os.path.join(ROOT, "aclswarm_amd", "lib", "libfacade_driver.so")


def run(name, idx, seed):
    Pf, Af = H.simform(name)
    p, adj = Pf[idx, 0], Af[idx]
    n = p.shape[0]
    rng = np.random.RandomState(seed)
    q = H.random_positions(rng, n, 20.0 if n <= 20 else 45.0)
    P_in = H.random_perm(rng, n).astype(np.uint8)
    lib = ct.CDLL(LIB)
    f = lib.facade_exchange
    f.restype = ct.c_int
    f.argtypes = [ct.c_int] + [ct.c_void_p] * 4 + [ct.c_uint32, ct.c_int] + [ct.c_void_p] * 6
    outs = [np.zeros((n, n), np.uint8), np.zeros(n, np.uint8), np.zeros(n, np.int32),
            np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros((n, n), np.int32)]
    ins = [np.asfortranarray(p, np.float64), np.asfortranarray(np.asarray(adj, np.uint8)),
           np.asfortranarray(q, np.float64), np.ascontiguousarray(P_in)]
    ptr = lambda a: a.ctypes.data_as(ct.c_void_p)  # noqa: E731
    t0 = time.perf_counter()
    rc = f(n, *[ptr(a) for a in ins], seed, 0, *[ptr(a) for a in outs])
    dt = time.perf_counter() - t0
    assert rc == 0
    tallies = n * (2 * n + 1)  # each vehicle: its START bid and 2n iterations
    starts = n                 # each start() also runs a B = 1 acl_solve_batch (alignment)
    return dict(fleet=name, n=n, seconds=dt, tallies=tallies, starts=starts,
                us_per_tally_incl_starts=1e6 * dt / tallies)


def main():
    import torch
    torch.cuda.init()
    run("simform20_nc", 0, 1)  # warm-up (module load, first launches)
    for name, idx, seed in (("simform20_nc", 1, 2), ("simform20_fc", 2, 3), ("simform100_nc", 0, 4)):
        print(json.dumps(run(name, idx, seed)), flush=True)


if __name__ == "__main__":
    main()
