#!/usr/bin/env python3
"""Generate tests/golden/hungarian_golden_large.json from the reference's
centralized comparator, aclswarm/src/aclswarm/assignment.py:94-137
(find_optimal_assignment), imported from the read-only reference tree.

Runs ONLY in the build container (/root/reference mounted); the tests read
the JSON this writes (data only: inputs and the reference's outputs).
hungarian_golden.json (make_fixtures.py) holds 12 small swarms (n = 6..15);
this adds the bench-sized cases:
  nc100_s{k}  the simform100_nc.npz formations (the reference's own
              generator, make_fixtures.py), q uniform in a 45 m square at
              z = 1 (start.sh:19-61 area scaled), random last
  fc20_s{k}   simform20_fc.npz formations, q in a 20 m square
  grid{n}     q and p on integer grids (many equal costs: SciPy's tie rule)
              with last = identity

Usage: python tests/golden/make_hungarian_fixtures.py
"""
import json
import os
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, os.path.join(REF, "aclswarm", "src"))
    from aclswarm import assignment  # noqa: E402
    rng = np.random.RandomState(2024)
    cases = []

    def add(name, q, p, last):
        n = q.shape[0]
        P, paligned = assignment.find_optimal_assignment(q.T.copy(), p.T.copy(),
                                                         [int(x) for x in last])
        cases.append({"name": name, "n": n, "q": q.tolist(), "p": p.tolist(),
                      "last": [int(x) for x in last], "P": [int(x) for x in P],
                      "paligned": np.asarray(paligned).T.tolist()})

    f100 = np.load(os.path.join(HERE, "simform100_nc.npz"))["points"][:, 0]
    for k in range(4):
        p = f100[k % f100.shape[0]]
        q = np.column_stack([rng.uniform(0, 45, 100), rng.uniform(0, 45, 100), np.ones(100)])
        add(f"nc100_s{k}", q, p, rng.permutation(100))
    f20 = np.load(os.path.join(HERE, "simform20_fc.npz"))["points"][:, 0]
    for k in range(2):
        q = np.column_stack([rng.uniform(0, 20, 20), rng.uniform(0, 20, 20), np.ones(20)])
        add(f"fc20_s{k}", q, f20[k], rng.permutation(20))
    for n, w in ((16, 4), (30, 6)):
        g = np.array([[k % w, k // w, 0.0] for k in range(n)], dtype=np.float64)
        q = g[rng.permutation(n)] + np.array([0.0, 0.0, 1.0])
        add(f"grid{n}", q, g.copy(), np.arange(n))
    out = {"source": "aclswarm/src/aclswarm/assignment.py:94-137 (imported, scipy "
                     + __import__("scipy").__version__ + ")", "cases": cases}
    with open(os.path.join(HERE, "hungarian_golden_large.json"), "w") as fh:
        json.dump(out, fh)
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
