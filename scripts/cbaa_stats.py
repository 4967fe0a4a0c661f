"""Work statistics of the lockstep CBAA (oracle/aclswarm_oracle.c orc_cbaa_m
restated in numpy, no margins) on C3-like swarms: per round the dirty
columns the auction kernel resolves, how many of them are a fixed point
before the update ("full") and how many become one after it ("uniform"),
the price levels a column needs, and the outbid re-selects. A design tool
for csrc/auction.hip (CPU only; prices from the oracle)."""
import sys
import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from aclswarm_amd import workload  # noqa: E402
from oracle import pyoracle  # noqa: E402

NONE = -1


def select(C, v, who_row, pr_row):
    c = C[v]
    ok = (c > 0.0) & (c > pr_row)
    if not ok.any():
        return -1
    cand = np.where(ok, c, -1.0)
    return int(np.argmax(cand))  # first maximum = strict > scan


def run(C, nb):
    n = C.shape[0]
    who = np.full((n, n), NONE, np.int64)
    pr = np.zeros((n, n), np.float32)
    dirty = np.zeros(n, bool)
    for v in range(n):
        t = select(C, v, who[v], pr[v])
        if t >= 0:
            who[v, t] = v; pr[v, t] = C[v, t]; dirty[t] = True
    st = []
    for r in range(1, 2 * n + 1):
        who2 = who.copy(); pr2 = pr.copy()
        ndirty = int(dirty.sum()); nfull = 0; nuni = 0; lv = []
        ndirty_next = np.zeros(n, bool)
        for j in np.nonzero(dirty)[0]:
            col_p = pr[:, j]; col_w = who[:, j]
            full = (col_w == col_w[0]).all()
            if full:
                nfull += 1
                continue
            # levels: distinct price keys from the top, vehicles resolved per level
            keys = np.unique(col_p)[::-1]
            unres = np.ones(n, bool); k = 0
            for key in keys:
                holders = col_p == key
                hit = unres & (nb[:, holders].any(axis=1))
                unres &= ~hit; k += 1
                if not unres.any():
                    break
            lv.append(k)
            # exact update
            for v in range(n):
                m = nb[v]
                idx = np.nonzero(m)[0]
                a = idx[np.argmax(col_p[idx])]  # first max in ascending order
                who2[v, j] = col_w[a]; pr2[v, j] = col_p[a]
            if (who2[:, j] != who[:, j]).any():
                ndirty_next[j] = True
                if (who2[:, j] == who2[0, j]).all():
                    nuni += 1
        nsel = 0
        for v in range(n):
            if ((who[v] == v) & (who2[v] != v)).any():  # outbid (auctioneer.cpp:502)
                t = select(C, v, who2[v], pr2[v]); nsel += 1
                if t >= 0:
                    who2[v, t] = v; pr2[v, t] = C[v, t]; ndirty_next[t] = True
        changed = (who2 != who).any()
        who, pr = who2, pr2
        st.append((r, ndirty, nfull, nuni, nsel, lv))
        dirty = ndirty_next
        if not changed:
            break
    return st


def main(B=8, n=100, seed=0, crowd_pct=100):
    """crowd_pct < 100: positions scaled by crowd_pct/100 about each swarm's
    centre (bench.py's ca_probe uses 30)."""
    gen = torch.Generator().manual_seed(seed)
    w = workload.simform_workload(B, n, gen, "cpu", formations="philox")
    if crowd_pct != 100:
        q = w["q"]
        cen = q[:, :, :2].mean(dim=1, keepdim=True)
        q[:, :, :2] = cen + (crowd_pct / 100.0) * (q[:, :, :2] - cen)
    tot = dict(rounds=0, dirty=0, full=0, uni=0, sel=0, lv=[])
    for b in range(B):
        q = w["q"][b].numpy(); p = w["p"][b].numpy(); adj = w["adj"][b].numpy().astype(np.uint8)
        P = np.arange(n, dtype=np.uint16)
        C, _ = pyoracle.prices(q, p, adj, P)
        nb = adj.astype(bool) | np.eye(n, dtype=bool)  # P = identity
        st = run(C, nb)
        tot["rounds"] += len(st)
        for (r, nd, nf, nu, ns, lv) in st:
            tot["dirty"] += nd; tot["full"] += nf; tot["uni"] += nu; tot["sel"] += ns
            tot["lv"] += lv
        if b == 0:
            for s in st:
                print("round %d dirty %d full %d becomes-uniform %d selects %d levels %s"
                      % (s[0], s[1], s[2], s[3], s[4], np.bincount(s[5]).tolist() if s[5] else []))
    print("per swarm: rounds %.2f dirty %.1f full %.1f uniform-after %.1f selects %.1f"
          % tuple(x / B for x in (tot["rounds"], tot["dirty"], tot["full"], tot["uni"], tot["sel"])))
    print("levels histogram", np.bincount(tot["lv"]).tolist())


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
