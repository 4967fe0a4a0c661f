"""Diagnostic: config C2 full batch (test_c2_full_batch's inputs) on the GPU
vs the oracle; prints the mismatching swarms' status, rounds and tables."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "oracle"))
sys.path.insert(0, R)
import helpers as H  # noqa: E402
import pyoracle as O  # noqa: E402
from test_gpu_parity import _gpu_solve  # noqa: E402

P, A = H.simform("simform20_fc")
rng = np.random.RandomState(4096)
pts = [P[s, k] for s in range(P.shape[0]) for k in range(2)]
adjs = [A[s] for s in range(P.shape[0]) for k in range(2)]
gains = [H.synth_gains(rng, a) for a in adjs]
B, n = 4096, 20
fidx = (np.arange(B) % len(pts)).astype(np.int32)
q = np.stack([H.random_positions(rng, n, 20.0) for _ in range(B)])
vel = rng.normal(0, 0.2, (B, n, 3))
P_in = np.stack([H.random_perm(rng, n) if b % 2 else np.arange(n, dtype=np.uint16) for b in range(B)])
if len(sys.argv) > 1 and sys.argv[1] == "rev":  # same swarms in reverse batch order
    fidx, q, vel, P_in = fidx[::-1].copy(), q[::-1].copy(), vel[::-1].copy(), P_in[::-1].copy()
if len(sys.argv) > 1 and sys.argv[1] == "few":  # only the swarms that failed in order
    sel = np.array([2455, 2500] * 64)
    fidx, q, vel, P_in = fidx[sel].copy(), q[sel].copy(), vel[sel].copy(), P_in[sel].copy()
    B = len(sel)
g = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
bad = np.nonzero((g["P_out"] != np.stack([O.solve(q[b], vel[b], pts[fidx[b]], adjs[fidx[b]], gains[fidx[b]], P_in[b])["P_out"] for b in range(B)])).any(1))[0]
print('B', B)
print("mismatching swarms", bad)
for b in bad[:4]:
    r = O.solve(q[b], vel[b], pts[fidx[b]], adjs[fidx[b]], gains[fidx[b]], P_in[b])
    print("swarm", b, "gpu status", g["status"][b], "ref status", r["status"])
    dw = np.argwhere(g["who"][b] != r["who"])
    print("  who diffs (v, j):", dw[:20].tolist(), "count", len(dw))
    print("  gpu P_out", g["P_out"][b].tolist())
    print("  ref P_out", r["P_out"].tolist())
    two = g.get("who")
    for v, j in dw[:5]:
        print("   v%d j%d gpu who %d ref who %d" % (v, j, g["who"][b][v, j], r["who"][v, j]))
