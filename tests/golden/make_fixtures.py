#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Runs ONLY in the build container, where the read-only reference tree is
mounted at /root/reference. Nothing at test time reads the reference: the
tests load the files this script writes.

Fixtures (all data -- inputs and expected outputs):
  swarm6_3d.json     formations.yaml:141-249 (points, adjmat, gains) and the
                     start.sh:129-136 grid start positions (config C1).
  simform_*.npz      formation groups from the reference's own generator
                     aclswarm_sim/nodes/generate_random_formation.py:61-96,
                     imported with rospy stubbed, seeded with np.random.seed
                     (trial.sh:60 recipe; L=40 for N=100 since L=15 cannot
                     hold 100 points at 2 m spacing).
  arun_golden.json   R, t from the reference's Python Arun/Procrustes
                     (aclswarm/src/aclswarm/assignment.py:15-53) on random 2-D
                     neighbourhoods: pins the oracle's Eigen-umeyama
                     restatement on generic (full-rank) inputs.
  hungarian_golden.json  find_optimal_assignment (assignment.py:94-137) on
                     small swarms: the centralized comparator (§8f row 2).
  admm_test_admm.json    the two n=4 MATLAB goldens of
                     aclswarm/test/test_admm.cpp:26-37,64-75 with their inputs.

Usage: python tests/golden/make_fixtures.py [simform set names ...]
  (no names: every fixture; names: only those simform sets)
"""
import json
import os
import sys
import types

import numpy as np
import yaml

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference_modules():
    # generate_random_formation.py imports rospy at module scope but only
    # uses it under __main__; a stub module is enough.
    sys.modules.setdefault("rospy", types.ModuleType("rospy"))
    sys.path.insert(0, os.path.join(REF, "aclswarm_sim", "nodes"))
    sys.path.insert(0, os.path.join(REF, "aclswarm", "src"))
    import generate_random_formation as grf  # noqa: E402
    from aclswarm import assignment  # noqa: E402
    return grf, assignment


def swarm6_fixture():
    with open(os.path.join(REF, "aclswarm", "param", "formations.yaml")) as f:
        doc = yaml.safe_load(f)
    grp = doc["swarm6_3d"]
    n = int(grp["agents"])
    forms = []
    for fm in grp["formations"]:
        forms.append({
            "name": fm["name"],
            "points": fm["points"],
            "adjmat": fm["adjmat"],
            "gains": fm["gains"],
        })
    # start.sh:129-136 grid (no -r option): x=(k%5)*1.5-4, y=(k/5)*1.5 (bc
    # integer division), z = takeoff_alt = 1.0 (coordination.launch:4)
    q0 = [[(k % 5) * 1.5 - 4.0, (k // 5) * 1.5, 1.0] for k in range(n)]
    return {"n": n, "formations": forms, "q0": q0,
            "source": "aclswarm/param/formations.yaml:141-249; "
                      "aclswarm_sim/scripts/start.sh:129-136"}


def simform_fixture(grf, n, fc, L, seeds, h=2.0, min_dist=2.0):
    pts, adjs, used = [], [], []
    for s in seeds:
        np.random.seed(s)
        g = grf.generate_formation_group(n, fc, L, L, h, min_dist, 2, False)
        if not g["formations"][0] or not g["formations"][1]:
            raise RuntimeError(f"generator timed out for n={n} L={L} seed={s}")
        adjs.append(np.array(g["adjmat"], dtype=np.uint8))
        pts.append(np.stack([np.array(f["points"], dtype=np.float64)
                             for f in g["formations"]]))
        used.append(s)
    return dict(points=np.stack(pts), adjmat=np.stack(adjs),
                seeds=np.array(used), n=n, fc=int(fc), L=L, h=h,
                min_dist=min_dist)


def arun_fixture(assignment, count=80, seed=1234):
    rng = np.random.RandomState(seed)
    cases = []
    for c in range(count):
        k = int(rng.randint(3, 40))
        p = rng.uniform(-10, 10, size=(2, k))
        th = rng.uniform(-np.pi, np.pi)
        Rt = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
        q = Rt @ p + rng.uniform(-5, 5, size=(2, 1)) + rng.normal(0, 0.3, size=(2, k))
        R, t = assignment.arun(q, p)
        cases.append({"p": p.T.tolist(), "q": q.T.tolist(),
                      "R": R.tolist(), "t": t.tolist()})
    return {"source": "aclswarm/src/aclswarm/assignment.py:15-53 (arun)",
            "cases": cases}


def hungarian_fixture(assignment, grf, count=12, seed=99):
    rng = np.random.RandomState(seed)
    cases = []
    for c in range(count):
        n = int(rng.choice([6, 10, 15]))
        p = rng.uniform(-6, 6, size=(3, n))
        p[2] = rng.uniform(0, 2, size=n)
        q = rng.uniform(-8, 8, size=(3, n))
        q[2] = 1.0
        last = list(rng.permutation(n))
        P, paligned = assignment.find_optimal_assignment(q, p, [int(x) for x in last])
        cases.append({"n": n, "q": q.T.tolist(), "p": p.T.tolist(),
                      "last": [int(x) for x in last], "P": [int(x) for x in P],
                      "paligned": np.asarray(paligned).T.tolist()})
    return {"source": "aclswarm/src/aclswarm/assignment.py:94-137", "cases": cases}


def admm_test_fixture():
    # aclswarm/test/test_admm.cpp:10-80: inputs and MATLAB golden matrices
    p = [[0.0, 0.0, 2.5], [2.0, 0.0, 3.5], [2.0, 2.0, 4.5], [0.0, 2.0, 1.5]]
    full = [
        [-0.50, 0, 0, 0.25, 0.25, 0, 0, 0, 0, 0.25, -0.25, 0],
        [0, -0.50, 0, -0.25, 0.25, 0, 0, 0, 0, 0.25, 0.25, 0],
        [0, 0, -0.70, 0, 0, 0.20, 0, 0, 0.10, 0, 0, 0.40],
        [0.25, -0.25, 0, -0.50, 0, 0, 0.25, 0.25, 0, 0, 0, 0],
        [0.25, 0.25, 0, 0, -0.50, 0, -0.25, 0.25, 0, 0, 0, 0],
        [0, 0, 0.20, 0, 0, -0.70, 0, 0, 0.40, 0, 0, 0.10],
        [0, 0, 0, 0.25, -0.25, 0, -0.50, 0, 0, 0.25, 0.25, 0],
        [0, 0, 0, 0.25, 0.25, 0, 0, -0.50, 0, -0.25, 0.25, 0],
        [0, 0, 0.10, 0, 0, 0.40, 0, 0, -0.30, 0, 0, -0.20],
        [0.25, 0.25, 0, 0, 0, 0, 0.25, -0.25, 0, -0.50, 0, 0],
        [-0.25, 0.25, 0, 0, -0, 0, 0.25, 0.25, 0, -0, -0.50, 0],
        [0, 0, 0.40, 0, 0, 0.10, 0, 0, -0.20, 0, 0, -0.30],
    ]
    noncomplete = [
        [-0.500, 0, 0, 0.250, 0.250, 0, 0, 0, 0, 0.250, -0.250, 0],
        [0, -0.500, 0, -0.250, 0.250, 0, 0, 0, 0, 0.250, 0.250, 0],
        [0, 0, -0.750, 0, 0, 0.375, 0, 0, 0, 0, 0, 0.375],
        [0.250, -0.250, 0, -0.500, 0, 0, 0.250, 0.250, 0, 0, 0, 0],
        [0.250, 0.250, 0, 0, -0.500, 0, -0.250, 0.250, 0, 0, 0, 0],
        [0, 0, 0.375, 0, 0, -0.750, 0, 0, 0.375, 0, 0, 0],
        [0, 0, 0, 0.250, -0.250, 0, -0.500, 0, 0, 0.250, 0.250, 0],
        [0, 0, 0, 0.250, 0.250, 0, 0, -0.500, 0, -0.250, 0.250, 0],
        [0, 0, 0, 0, 0, 0.375, 0, 0, -0.250, 0, 0, -0.125],
        [0.250, 0.250, 0, 0, 0, 0, 0.250, -0.250, 0, -0.500, 0, 0],
        [-0.250, 0.250, 0, 0, 0, 0, 0.250, 0.250, 0, 0, -0.500, 0],
        [0, 0, 0.375, 0, 0, 0, 0, 0, -0.125, 0, 0, -0.250],
    ]
    adj_full = [[0 if i == j else 1 for j in range(4)] for i in range(4)]
    adj_nc = [row[:] for row in adj_full]
    adj_nc[0][2] = adj_nc[2][0] = 0
    adj_nc[1][3] = adj_nc[3][1] = 0
    return {"source": "aclswarm/test/test_admm.cpp:10-80", "tol": 1e-8,
            "cases": [
                {"name": "fourAgentSquareFullyConnected", "p": p,
                 "adj": adj_full, "A": full},
                {"name": "fourAgentSquareNonComplete", "p": p,
                 "adj": adj_nc, "A": noncomplete}]}


def admm_nine_fixture():
    # aclswarm/test/test_admm.cpp:84-187 (nineAgentSquareNonCompleteZeroBlocks,
    # ...BlockStructure): inputs only -- the test asserts properties, not a
    # matrix: zero 3x3 blocks at the non-edges (sum < 1e-8) and every block of
    # the form [a b 0; -b a 0; 0 0 c] (one-sided "< 1e-8" checks, :165-171).
    n = 9
    adj = [[0 if i == j else 1 for j in range(n)] for i in range(n)]
    for i, j in [(0, 6), (2, 4), (5, 7), (5, 8), (6, 7),
                 (4, 2), (6, 0), (7, 5), (7, 6), (8, 5)]:
        adj[i][j] = 0
    p = [[-1.7484733199059646, 1.7306756147165174, 0.2977622220453062],
         [6.8174866001631180, -6.2778267151168700, 1.7416024649609380],
         [-3.8137004331127518, -2.3232057308608365, 0.4655014204423282],
         [2.7536551200474015, -5.5700708736518450, 1.7252000594155040],
         [-3.5935365621834463, 4.8028457222331170, 1.2981050175550286],
         [-2.5820075847777666, 7.4136205487374910, 1.5131454738258028],
         [0.8900655441583734, 3.2902893860285527, 1.5581930129432586],
         [0.4370445360276376, -5.7714142992744755, 0.2531727259898202],
         [-6.1065377928157310, -5.7852241311701940, 1.7663507973073431]]
    return {"source": "aclswarm/test/test_admm.cpp:84-187", "tol": 1e-8,
            "name": "nineAgentSquareNonComplete", "p": p, "adj": adj}


SETS = [
    ("simform20_fc", 20, True, 15.0, range(0, 8)),
    ("simform20_nc", 20, False, 15.0, range(0, 8)),
    ("simform100_nc", 100, False, 40.0, range(0, 4)),
    ("simform500_nc", 500, False, 90.0, range(0, 2)),
]


def main():
    only = sys.argv[1:]
    if only == ["admm"]:   # data transcribed from test_admm.cpp; no imports
        with open(os.path.join(OUT, "admm_test_admm.json"), "w") as f:
            json.dump(admm_test_fixture(), f)
        with open(os.path.join(OUT, "admm_nine_agent.json"), "w") as f:
            json.dump(admm_nine_fixture(), f)
        return
    grf, assignment = _import_reference_modules()
    if only:
        for name, n, fc, L, seeds in SETS:
            if name in only:
                d = simform_fixture(grf, n, fc, L, list(seeds))
                np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)
                print("wrote", name)
        return
    with open(os.path.join(OUT, "swarm6_3d.json"), "w") as f:
        json.dump(swarm6_fixture(), f)
    for name, n, fc, L, seeds in SETS:
        d = simform_fixture(grf, n, fc, L, list(seeds))
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **d)
    with open(os.path.join(OUT, "arun_golden.json"), "w") as f:
        json.dump(arun_fixture(assignment), f)
    with open(os.path.join(OUT, "hungarian_golden.json"), "w") as f:
        json.dump(hungarian_fixture(assignment, grf), f)
    with open(os.path.join(OUT, "admm_test_admm.json"), "w") as f:
        json.dump(admm_test_fixture(), f)
    with open(os.path.join(OUT, "admm_nine_agent.json"), "w") as f:
        json.dump(admm_nine_fixture(), f)
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
