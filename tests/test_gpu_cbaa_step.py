"""GPU parity of acl_cbaa_step_batch (ABI 11: one vehicle's CBAA bid iteration,
the message-level protocol of auctioneer.cpp:182-306,469-549) against the
CPU restatement oracle/cbaa_step_oracle.py (itself pinned to the oracle's
lockstep CBAA by tests/test_cbaa_step.py).

Bar: tables (price bits, who), selected task and flags bit-exact (integer
and float32 compare-and-copy work; the prices are the f64 getPrice in the
reference's operation order, rounded to float)."""
import numpy as np
import pytest

import cbaa_step_oracle as S
import helpers as H

pytestmark = pytest.mark.gpu


def _dev():
    import torch
    return torch.device("cuda:0")


def _t(a, dt):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dt)).to(_dev())


def _run(ps, fidx, vehid, q, Rt, start, price, who, cands):
    """cands[k]: [(vehid, price, who)] of vehicle k."""
    import torch
    from aclswarm_amd import engine
    n = ps[0].shape[0]
    T = engine.FormationTable.from_host(ps, [np.ones((n, n), np.uint8)] * len(ps), None,
                                        device=_dev())
    off = np.zeros(len(vehid) + 1, np.int32)
    off[1:] = np.cumsum([len(c) for c in cands])
    K = int(off[-1])
    cv = np.array([u for c in cands for u, _, _ in c], np.int32)
    cp = np.array([x for c in cands for _, x, _ in c], np.float32).reshape(K, n)
    cw = np.array([w for c in cands for _, _, w in c], np.int32).reshape(K, n)
    pr_d, wh_d = _t(price, np.float32), _t(who, np.int32)
    task, flags = engine.cbaa_step(
        T, _t(fidx, np.int32), _t(vehid, np.int32), _t(q, np.float64), _t(Rt, np.float64),
        _t(start, np.uint8), pr_d, wh_d, _t(off, np.int32),
        _t(cv, np.int32) if K else None, _t(cp, np.float32) if K else None,
        _t(cw, np.int32) if K else None)
    torch.cuda.synchronize()
    return pr_d.cpu().numpy(), wh_d.cpu().numpy(), task.cpu().numpy(), flags.cpu().numpy()


def _random_batch(rng, n, V, F):
    ps = [np.column_stack([rng.uniform(0, 20, n), rng.uniform(0, 20, n), rng.uniform(0, 2, n)])
          for _ in range(F)]
    fidx = rng.randint(0, F, V).astype(np.int32)
    vehid = rng.randint(0, n, V).astype(np.int32)
    q = np.column_stack([rng.uniform(0, 22, V), rng.uniform(0, 22, V), np.ones(V)])
    th = rng.uniform(-np.pi, np.pi, V)
    Rt = np.column_stack([np.cos(th), -np.sin(th), np.sin(th), np.cos(th),
                          rng.normal(0, 1, V), rng.normal(0, 1, V)])
    start = (rng.uniform(size=V) < 0.25).astype(np.uint8)
    levels = np.array([0.0, 0.05, 0.1, 0.2, 0.5], np.float32)  # equal prices: ties
    price = np.empty((V, n), np.float32)
    who = np.empty((V, n), np.int32)
    cands = []
    for k in range(V):
        price[k] = np.where(rng.uniform(size=n) < 0.5, rng.choice(levels, n),
                            rng.uniform(0, 0.3, n)).astype(np.float32)
        who[k] = rng.randint(-1, n, n)
        who[k][rng.uniform(size=n) < 0.2] = vehid[k]  # tasks it holds
        if start[k]:
            cands.append([])
            continue
        K = rng.randint(1, 7)
        ids = set(rng.choice(n, size=min(K, n), replace=False).tolist())
        if rng.uniform() < 0.8:
            ids.add(int(vehid[k]))
        c = []
        for u in sorted(ids):
            if u == vehid[k]:
                c.append((u, price[k].copy(), who[k].copy()))
            else:
                cp = np.where(rng.uniform(size=n) < 0.5, rng.choice(levels, n),
                              rng.uniform(0, 0.3, n)).astype(np.float32)
                cp[rng.uniform(size=n) < 0.02] = np.nan
                c.append((u, cp, rng.randint(-1, n, n).astype(np.int32)))
        cands.append(c)
    return ps, fidx, vehid, q, Rt, start, price, who, cands


@pytest.mark.parametrize("n", [7, 64, 100, 130, 300, 500])
def test_step_random_batch(n):
    rng = np.random.RandomState(n)
    ps, fidx, vehid, q, Rt, start, price, who, cands = _random_batch(rng, n, 96, 3)
    pr, wh, task, flags = _run(ps, fidx, vehid, q, Rt, start, price, who, cands)
    n_sel = n_ob = 0
    for k in range(len(vehid)):
        row = S.price_row(ps[fidx[k]], q[k], Rt[k])
        ep, ew, et, eo = S.step(int(vehid[k]), bool(start[k]), price[k], who[k], cands[k], row)
        np.testing.assert_array_equal(pr[k].view(np.uint32), ep.view(np.uint32), err_msg=str(k))
        np.testing.assert_array_equal(wh[k], ew, err_msg=str(k))
        assert task[k] == et, k
        assert flags[k] == (0x01 if eo else 0) | (0x02 if et >= 0 else 0), k
        n_sel += et >= 0
        n_ob += eo
    assert n_sel > 10 and n_ob > 5  # the cases exercise both paths


def test_step_bad_input_leaves_tables():
    rng = np.random.RandomState(3)
    n = 10
    ps, fidx, vehid, q, Rt, start, price, who, cands = _random_batch(rng, n, 6, 2)
    start[:] = 0
    z = (np.zeros(n, np.float32), np.zeros(n, np.int32))
    cands = [[(3, *z), (1, *z)],          # not ascending
             [(2, *z), (2, *z)],          # duplicate
             [(0, *z), (n, *z)],          # vehid out of range
             [(0, *z)],                   # fidx out of range (below)
             [],                          # no candidates on an iteration
             [(0, *z), (4, *z)]]          # vehicle id out of range (below)
    fidx[3] = 7
    vehid[5] = n
    pr, wh, task, flags = _run(ps, fidx, vehid, q, Rt, start, price, who, cands)
    assert (flags == 0x10).all() and (task == -1).all()
    np.testing.assert_array_equal(pr.view(np.uint32), price.view(np.uint32))
    np.testing.assert_array_equal(wh, who)


@pytest.mark.parametrize("name,b", [("simform20_nc", 0), ("simform100_nc", 1)])
def test_protocol_on_gpu_equals_one_call_consensus(name, b):
    """Every vehicle of a swarm runs the message protocol on the GPU (START
    bids, then 2n iterations tallied from its neighbours' bids of the same
    iteration, V = n vehicles per launch) from its acl_solve_batch alignment:
    the tables equal acl_solve_batch's one-call consensus bit for bit."""
    import torch
    from aclswarm_amd import engine
    Pf, Af = H.simform(name)
    p, adj = Pf[b, 0], Af[b].astype(np.uint8)
    n = p.shape[0]
    rng = np.random.RandomState(b + 5)
    q = H.random_positions(rng, n, 20.0 if n <= 20 else 45.0)
    P = H.random_perm(rng, n)
    dev = _dev()
    T = engine.FormationTable.from_host([p], [adj], None, device=dev)
    out = engine.solve(T, torch.zeros(1, dtype=torch.int32, device=dev),
                       _t(q[None], np.float64), torch.zeros((1, n, 3), dtype=torch.float64,
                                                            device=dev),
                       _t(P[None].view(np.int16), np.int16), do_control=False, want_who=True,
                       want_align=True, early_exit=True)
    torch.cuda.synchronize()
    who_1 = out["who"].cpu().numpy().view(np.uint16)[0].astype(np.int32)
    Rt = out["align_Rt"].cpu().numpy()[0]
    Pt = np.empty(n, np.int64)
    Pt[P] = np.arange(n)
    nbrs = [sorted(int(Pt[j]) for j in range(n) if adj[P[v]][j]) for v in range(n)]
    ids = np.arange(n, dtype=np.int32)
    price = np.zeros((n, n), np.float32)
    who = np.full((n, n), -1, np.int32)
    pr, wh, _, fl = _run([p], np.zeros(n, np.int32), ids, q, Rt, np.ones(n, np.uint8),
                         price, who, [[] for _ in range(n)])
    assert (fl & 0x02).all()
    for _ in range(2 * n):
        cands = [[(u, pr[u], wh[u]) for u in sorted(set(nbrs[v]) | {v})] for v in range(n)]
        pr, wh, _, fl = _run([p], np.zeros(n, np.int32), ids, q, Rt, np.zeros(n, np.uint8),
                             pr, wh, cands)
        assert not (fl & 0x10).any()
    who_1 = np.where(who_1 == 0xFFFF, -1, who_1)
    np.testing.assert_array_equal(wh, who_1)


def test_step_candidate_range_checked():
    """A candidate range outside [0, K] (cand_off[k + 1] > K, or a reversed
    range) is BAD_INPUT: nothing past the candidate arrays is read and the
    tables are left as they were."""
    import torch
    from aclswarm_amd import engine
    n, V, K = 5, 3, 2
    ps = [np.column_stack([np.arange(n, dtype=float), np.zeros(n), np.ones(n)])]
    T = engine.FormationTable.from_host(ps, [np.ones((n, n), np.uint8)], None, device=_dev())
    price = np.full((V, n), 0.25, np.float32)
    who = np.full((V, n), -1, np.int32)
    pr_d, wh_d = _t(price, np.float32), _t(who, np.int32)
    off = np.array([0, 3, 2, 2], np.int32)  # vehicle 0: rows 0..2 (> K); 1: reversed; 2: empty
    task, flags = engine.cbaa_step(
        T, _t(np.zeros(V), np.int32), _t([0, 1, 2], np.int32), _t(np.zeros((V, 3)), np.float64),
        _t(np.tile([1.0, 0, 0, 1.0, 0, 0], (V, 1)), np.float64), _t(np.zeros(V), np.uint8),
        pr_d, wh_d, _t(off, np.int32), _t([0, 1], np.int32), _t(np.zeros((K, n)), np.float32),
        _t(np.zeros((K, n)), np.int32))
    torch.cuda.synchronize()
    assert (flags.cpu().numpy() == 0x10).all() and (task.cpu().numpy() == -1).all()
    np.testing.assert_array_equal(pr_d.cpu().numpy(), price)
    np.testing.assert_array_equal(wh_d.cpu().numpy(), who)
