"""CPU restatement of one vehicle's CBAA bid iteration (acl_cbaa_step_batch).

TEST INFRASTRUCTURE ONLY: imported by tests/, never by the product package.

Restates, for one vehicle of the reference's per-vehicle Auctioneer:
  reset                 aclswarm/src/auctioneer.cpp:448-465 (price 0, who -1)
  updateTaskAssignment  auctioneer.cpp:469-513 (std::map bids_curr_ with the
                        vehicle's own bid inserted, :475; ascending vehid,
                        the first of equal prices kept: strict >)
  selectTaskAssignment  auctioneer.cpp:517-542 (max = 0, price > max and
                        price > bid.price[j], ascending j)
  getPrice              auctioneer.cpp:546-549 on aligned = (R p + t, p.z)
                        (:400-414), in orc_prices_rows' f64 order (numpy: one
                        rounding per operation, no contraction)
and, to pin it, the lockstep message protocol of processBid (:182-306) for
all vehicles of a swarm, whose tables after 2n iterations are the oracle's
orc_cbaa tables (tests/test_cbaa_step.py).
"""
import numpy as np


def price_row(p, q_v, rt):
    """getPrice(q_v, aligned_j) for every task j (float32[n])."""
    p = np.asarray(p, np.float64)
    R0, R1, R2, R3, t0, t1 = (float(x) for x in rt)
    px, py, pz = p[:, 0], p[:, 1], p[:, 2]
    ax = ((R0 * px + R1 * py) + 0.0 * pz) + t0
    ay = ((R2 * px + R3 * py) + 0.0 * pz) + t1
    az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0
    dx, dy, dz = q_v[0] - ax, q_v[1] - ay, q_v[2] - az
    nrm = np.sqrt((dx * dx + dy * dy) + dz * dz)
    return (1.0 / (nrm + 1e-8)).astype(np.float32)


def step(vehid, start, price, who, cands, row):
    """One tally of vehicle `vehid`. price float32[n], who int32[n] (its
    table); cands: [(vehid, price, who)] in ascending vehid including its own
    entry (ignored when start); row: its price_row. Returns (price, who,
    task, outbid)."""
    n = len(row)
    price = np.array(price, np.float32)
    who = np.array(who, np.int32)
    outbid = False
    if start:
        price[:] = 0.0
        who[:] = -1
    else:
        for j in range(n):
            mp, mw = cands[0][1][j], cands[0][2][j]
            for _, cp, cw in cands[1:]:
                if cp[j] > mp:
                    mp, mw = cp[j], cw[j]
            if who[j] == vehid and mw != vehid:
                outbid = True
            who[j] = mw
            price[j] = mp
    task = -1
    if start or outbid:
        mx = np.float32(0.0)
        for j in range(n):
            if row[j] > mx and row[j] > price[j]:
                mx = row[j]
                task = j
        if task >= 0:
            price[task] = mx
            who[task] = vehid
    return price, who, task, outbid


def lockstep(C, adj, P, rounds=None):
    """Every vehicle's table after the protocol's 2n iterations (all vehicles
    start from one snapshot, bids of iteration k tallied with the neighbours'
    bids of iteration k): C[v] its price row, adj row-major [i][j], P vehicle
    -> formation point. Returns who int32[n][n], price float32[n][n]."""
    C = np.asarray(C, np.float32)
    n = C.shape[0]
    P = np.asarray(P, np.int64)
    Pt = np.empty(n, np.int64)
    Pt[P] = np.arange(n)
    nbrs = [sorted(int(Pt[j]) for j in range(n) if adj[P[v]][j]) for v in range(n)]
    tabs = []
    for v in range(n):
        pr, wh, _, _ = step(v, True, np.zeros(n, np.float32), np.full(n, -1, np.int32), [], C[v])
        tabs.append((pr, wh))
    for _ in range(rounds if rounds is not None else 2 * n):
        new = []
        for v in range(n):
            cands = sorted({u: tabs[u] for u in nbrs[v] + [v]}.items())
            cl = [(u, t[0], t[1]) for u, t in cands]
            pr, wh, _, _ = step(v, False, tabs[v][0], tabs[v][1], cl, C[v])
            new.append((pr, wh))
        tabs = new
    return np.array([t[1] for t in tabs]), np.array([t[0] for t in tabs])
