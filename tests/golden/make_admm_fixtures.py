#!/usr/bin/env python3
"""Generate tests/golden/admm_golden.npz from the reference's own ADMM.

Runs ONLY in the build container: it calls oracle/_ref/libadmm_ref.so, which
`make -C oracle ref` compiles from aclswarm/lib/codegen_admm where it lies in
the read-only reference tree. The file holds data only -- inputs and the
reference's outputs -- for tests/test_admm.py and the GPU parity tests.

Cases (inputs are committed fixtures or seeded synthetic formations):
  swarm6_*     formations.yaml swarm6_3d points/adjmat (tests/golden/swarm6_3d.json)
  nc20_s*      generator formations, n=20 noncomplete (simform20_nc.npz)
  fc20_s*      generator formations, n=20 complete (simform20_fc.npz)
  flat20_s*    nc20 with z = 1 + 1e-3 N(0,1): planar branch, std(qz) < 1e-2
  rand{n}      uniform points in a 10 m cube, random symmetric graph, n=3,5,9
  nc100_s0     generator formation, n=100 noncomplete (simform100_nc.npz), C5
Per case: p (n x 3), adj (n x n u8), Axy (2n x 2n) and Az (n x n) -- the two
nonzero parts of ADMM::calculateFormationGains' 3n x 3n result
(admm.cpp:32-51, |a| < 1e-10 zeroed).

Usage: python tests/golden/make_admm_fixtures.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import helpers as H  # noqa: E402
import pyadmm_ref as R  # noqa: E402


def split(A, n):
    Axy = np.zeros((2 * n, 2 * n))
    for i in range(n):
        for j in range(n):
            Axy[2 * i:2 * i + 2, 2 * j:2 * j + 2] = A[3 * i:3 * i + 2, 3 * j:3 * j + 2]
    return Axy, A[2::3, 2::3].copy()


def random_case(rng, n):
    p = rng.uniform(-5, 5, size=(n, 3))
    adj = np.ones((n, n), np.uint8) - np.eye(n, dtype=np.uint8)
    for _ in range(max(0, n - 3)):
        i, j = rng.choice(n, 2, replace=False)
        adj[i, j] = adj[j, i] = 0
    return p, adj


def main():
    cases = []
    pts, adjs, _, _ = H.swarm6()
    for k, (p, a) in enumerate(zip(pts, adjs)):
        cases.append((f"swarm6_{k}", p, a))
    P, A = H.simform("simform20_nc")
    rng = np.random.RandomState(7)
    for s in range(4):
        cases.append((f"nc20_s{s}", P[s, 0], A[s]))
    for s in range(2):
        pf = P[s, 1].copy()
        pf[:, 2] = 1.0 + 1e-3 * rng.randn(pf.shape[0])
        cases.append((f"flat20_s{s}", pf, A[s]))
    P, A = H.simform("simform20_fc")
    for s in range(2):
        cases.append((f"fc20_s{s}", P[s, 0], A[s]))
    for n in (3, 5, 9):
        p, a = random_case(rng, n)
        cases.append((f"rand{n}", p, a))
    P, A = H.simform("simform100_nc")
    cases.append(("nc100_s0", P[0, 0], A[0]))

    out = {"names": np.array([c[0] for c in cases])}
    for name, p, a in cases:
        n = p.shape[0]
        G = R.solve(p, a)
        Axy, Az = split(G, n)
        out[name + "/p"] = np.asarray(p, np.float64)
        out[name + "/adj"] = np.asarray(a, np.uint8)
        out[name + "/Axy"] = Axy
        out[name + "/Az"] = Az
        print(name, n, float(np.trace(G)))
    np.savez_compressed(os.path.join(HERE, "admm_golden.npz"), **out)


if __name__ == "__main__":
    main()
