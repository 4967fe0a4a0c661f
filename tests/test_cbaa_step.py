"""CPU: the per-vehicle bid iteration restatement (oracle/cbaa_step_oracle.py,
the reference's updateTaskAssignment / selectTaskAssignment / getPrice,
auctioneer.cpp:469-549) pinned against the oracle's lockstep CBAA: run as the
message protocol (every vehicle's START bid, then 2n iterations of
neighbour-bid tallies), its tables equal orc_cbaa's with all 2n rounds, and
its price rows equal orc_prices'."""
import numpy as np
import pytest

import cbaa_step_oracle as S
import helpers as H
import pyoracle as O


def _case(name, seed):
    rng = np.random.RandomState(seed)
    if name == "swarm6":
        pts, adj, _, q0 = H.swarm6()
        p, adj = pts[1], adj[1]
        q = q0 + rng.normal(0, 0.3, q0.shape)
    else:
        Pf, Af = H.simform(name)
        p, adj = Pf[seed % Pf.shape[0], 0], Af[seed % Af.shape[0]]
        q = H.random_positions(rng, p.shape[0], 20.0)
    return p, adj.astype(np.uint8), q, H.random_perm(rng, p.shape[0])


@pytest.mark.parametrize("name,seed", [("swarm6", 1), ("swarm6", 2), ("simform20_nc", 3),
                                       ("simform20_fc", 4)])
def test_protocol_equals_lockstep_oracle(name, seed):
    p, adj, q, P = _case(name, seed)
    C, Rt = O.prices(q, p, adj, P)
    n = p.shape[0]
    for v in range(n):  # the step's getPrice from (R, t) = the oracle's price row
        row = S.price_row(p, q[v], Rt[v])
        np.testing.assert_array_equal(row.view(np.uint32), C[v].view(np.uint32))
    who, pr = S.lockstep(C, adj, P)
    who_o, pr_o, _ = O.cbaa(C, adj, P, early_exit=False)
    np.testing.assert_array_equal(who, who_o)
    np.testing.assert_array_equal(pr.view(np.uint32), pr_o.view(np.uint32))


def test_step_rules():
    """Hand cases: the first of equal prices wins in vehid order, a NaN first
    candidate is never beaten, outbid only on a task the vehicle held, select
    takes the lowest task of the largest eligible price."""
    n = 4
    row = np.array([0.5, 0.9, 0.9, 0.2], np.float32)
    # START: reset, then the lowest of the two 0.9 tasks
    pr, wh, task, ob = S.step(2, True, np.ones(n, np.float32), np.zeros(n, np.int32), [], row)
    assert task == 1 and not ob and wh.tolist() == [-1, 2, -1, -1]
    assert pr.tolist() == [0.0, np.float32(0.9), 0.0, 0.0]
    # tie on task 1 between vehicles 0 and 2 (equal price): vehicle 0 is first
    own = (np.array([0, 0.9, 0, 0], np.float32), np.array([-1, 2, -1, -1], np.int32))
    c0 = (0, np.array([0, 0.9, 0, 0], np.float32), np.array([-1, 0, -1, -1], np.int32))
    c2 = (2, own[0], own[1])
    pr, wh, task, ob = S.step(2, False, own[0], own[1], [c0, c2], row)
    assert ob and wh[1] == 0 and task == 2 and wh[2] == 2
    # NaN first candidate: nothing beats it
    cn = (0, np.array([np.nan, 0, 0, 0], np.float32), np.array([1, -1, -1, -1], np.int32))
    pr, wh, task, ob = S.step(2, False, own[0], own[1], [cn, c2], row)
    assert np.isnan(pr[0]) and wh[0] == 1 and not ob and task == -1


def test_engine_step_rejects_bad_tensors():
    """engine.cbaa_step checks dtype, shape, contiguity and device before any
    pointer reaches the library (no GPU needed: it raises first)."""
    import types

    import torch
    from aclswarm_amd import engine
    V, n = 3, 5
    T = types.SimpleNamespace(n=n)
    good = dict(fidx=torch.zeros(V, dtype=torch.int32), vehid=torch.zeros(V, dtype=torch.int32),
                q=torch.zeros(V, 3, dtype=torch.float64), Rt=torch.zeros(V, 6, dtype=torch.float64),
                start=torch.ones(V, dtype=torch.uint8), price=torch.zeros(V, n),
                who=torch.zeros(V, n, dtype=torch.int32), cand_off=torch.zeros(V + 1, dtype=torch.int32))
    bad = [("price", torch.zeros(V, n, dtype=torch.float64)),        # dtype
           ("who", torch.zeros(n, V, dtype=torch.int32).t()),        # not contiguous
           ("q", torch.zeros(V, 2, dtype=torch.float64)),            # shape
           ("cand_off", torch.zeros(V, dtype=torch.int32))]          # V + 1 entries
    for name, t in bad:
        kw = dict(good, **{name: t})
        with pytest.raises(ValueError, match=name):
            engine.cbaa_step(T, **kw)
