"""Shared test inputs: committed fixtures + seeded synthetic swarms."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def swarm6():
    """Config C1: formations.yaml swarm6_3d + start.sh grid (tests/golden)."""
    d = load_json("swarm6_3d.json")
    pts = [np.array(f["points"], np.float64) for f in d["formations"]]
    adj = [np.array(f["adjmat"], np.uint8) for f in d["formations"]]
    gains = [np.array(f["gains"], np.float64) for f in d["formations"]]
    return pts, adj, gains, np.array(d["q0"], np.float64)


def simform(name):
    """Formation groups from the reference generator (tests/golden/*.npz).
    Returns points [S][2][n][3], adjmat [S][n][n]."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    return z["points"], z["adjmat"]


def random_positions(rng, n, side, r=0.75, z=1.0):
    """n non-overlapping discs of radius r, uniform in a side x side square
    centred at the origin (start.sh:19-61 recipe), at altitude z."""
    pts = np.zeros((0, 2))
    while pts.shape[0] < n:
        c = rng.uniform(-side / 2, side / 2, size=2)
        if pts.shape[0] == 0 or np.min(np.hypot(*(pts - c).T)) >= 2 * r:
            pts = np.vstack([pts, c])
    return np.c_[pts, np.full(n, z)]


def dense_positions(rng, n, side):
    """Uniform positions without spacing: exercises collision avoidance."""
    return np.c_[rng.uniform(-side / 2, side / 2, size=(n, 2)), rng.uniform(0.5, 1.5, size=n)]


def synth_gains(rng, adj, scale=0.3):
    """A GainMat with the reference's block structure [a b 0; -b a 0; 0 0 c]
    on edges and the negated row sum on the diagonal (synthetic values)."""
    n = adj.shape[0]
    G = np.zeros((3 * n, 3 * n))
    for i in range(n):
        for j in range(n):
            if i != j and adj[i, j]:
                a, b, c = rng.uniform(-scale, scale, 3)
                G[3 * i:3 * i + 3, 3 * j:3 * j + 3] = [[a, b, 0], [-b, a, 0], [0, 0, c]]
        G[3 * i:3 * i + 3, 3 * i:3 * i + 3] = -sum(
            G[3 * i:3 * i + 3, 3 * j:3 * j + 3] for j in range(n) if j != i)
    return G


def random_perm(rng, n):
    return rng.permutation(n).astype(np.uint16)


def random_block_gains(rng, adj, scale=0.3):
    """A GainMat with unstructured random 3x3 blocks on the edges (the
    general 9-plane layout; no ADMM structure)."""
    n = adj.shape[0]
    G = np.zeros((3 * n, 3 * n))
    for i in range(n):
        for j in range(n):
            if adj[i, j]:
                G[3 * i:3 * i + 3, 3 * j:3 * j + 3] = rng.uniform(-scale, scale, (3, 3))
    return G
