"""GPU parity of the centralized comparator (acl_hungarian_batch, SURVEY
§8f row 2) against the CPU restatement (oracle/hungarian_oracle.c) and the
reference's own outputs (tests/golden/hungarian_golden*.json).

Bar: P_opt bit-exact (integer work); cost sums and the alignment bit-exact
too (the kernel runs the oracle's operation order without contraction).
"""
import json
import os

import numpy as np
import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _gpu(ps, fidx, q, P_last=None, P_cmp=None):
    import torch
    from aclswarm_amd import engine
    dev = torch.device("cuda:0")
    n = q.shape[1]
    adjs = [np.ones((n, n), np.uint8)] * len(ps)
    T = engine.FormationTable.from_host(ps, adjs, None, device=dev)
    t16 = lambda a: None if a is None else torch.from_numpy(  # noqa: E731
        np.ascontiguousarray(np.asarray(a, np.uint16)).view(np.int16)).to(dev)
    out = engine.hungarian(T, torch.from_numpy(np.asarray(fidx, np.int32)).to(dev),
                           torch.from_numpy(np.ascontiguousarray(q, np.float64)).to(dev),
                           t16(P_last), t16(P_cmp), want_Rt=True)
    torch.cuda.synchronize()
    r = {k: v.cpu().numpy() for k, v in out.items()}
    r["P_opt"] = r["P_opt"].view(np.uint16)
    return r


def _check_vs_oracle(ps, fidx, q, P_last=None, P_cmp=None):
    g = _gpu(ps, fidx, q, P_last, P_cmp)
    for b in range(q.shape[0]):
        P, cost, Rt, st = O.hungarian(q[b], ps[fidx[b]],
                                      None if P_last is None else P_last[b],
                                      None if P_cmp is None else P_cmp[b])
        assert g["status"][b] == st, b
        assert np.array_equal(g["P_opt"][b], P), b
        np.testing.assert_array_equal(g["cost"][b].view(np.uint64), cost.view(np.uint64))
        if not st & 0x01:
            np.testing.assert_array_equal(g["align_Rt"][b].view(np.uint64), Rt.view(np.uint64))
    return g


def _swarms(rng, n, B, F, side):
    ps = [np.column_stack([rng.uniform(0, side, n), rng.uniform(0, side, n),
                           rng.uniform(0, 2, n)]) for _ in range(F)]
    q = np.stack([np.column_stack([rng.uniform(0, side * 1.1, n), rng.uniform(0, side * 1.1, n),
                                   np.ones(n)]) for _ in range(B)])
    fidx = rng.integers(0, F, B).astype(np.int32)
    P_last = np.stack([rng.permutation(n) for _ in range(B)]).astype(np.uint16)
    return ps, fidx, q, P_last


@pytest.mark.parametrize("fn", ["hungarian_golden.json", "hungarian_golden_large.json"])
def test_reference_goldens(fn):
    with open(os.path.join(HERE, "golden", fn)) as fh:
        cases = json.load(fh)["cases"]
    by_n = {}
    for c in cases:
        by_n.setdefault(c["n"], []).append(c)
    for n, cs in by_n.items():
        ps = [np.array(c["p"]) for c in cs]
        q = np.stack([np.array(c["q"]) for c in cs])
        last = np.stack([np.array(c["last"]) for c in cs]).astype(np.uint16)
        g = _check_vs_oracle(ps, np.arange(len(cs), dtype=np.int32), q, last)
        for b, c in enumerate(cs):
            assert list(g["P_opt"][b]) == c["P"]


@pytest.mark.parametrize("n", [1, 2, 6, 20, 64, 100, 128])
def test_random_swarms_small_kernel(n):
    rng = np.random.default_rng(n)
    ps, fidx, q, P_last = _swarms(rng, n, 96, 5, max(4.0, 4.5 * np.sqrt(n)))
    P_cmp = np.stack([rng.permutation(n) for _ in range(96)]).astype(np.uint16)
    _check_vs_oracle(ps, fidx, q, P_last, P_cmp)


@pytest.mark.parametrize("n", [129, 200, 300, 512])
def test_random_swarms_wide(n):
    rng = np.random.default_rng(n)
    ps, fidx, q, P_last = _swarms(rng, n, 6, 2, 4.5 * np.sqrt(n))
    _check_vs_oracle(ps, fidx, q, P_last)


@pytest.mark.parametrize("n,w", [(16, 4), (64, 8), (100, 10), (200, 20)])
def test_integer_grids_ties(n, w):
    # q and p on the same integer grid: many equal distances, SciPy's tie
    # rule decides (pinned for the oracle in tests/test_hungarian.py)
    rng = np.random.default_rng(w)
    g = np.array([[k % w, k // w, 0.0] for k in range(n)], np.float64)
    B = 8
    q = np.stack([g[rng.permutation(n)] + [0, 0, 1.0] for _ in range(B)])
    P_last = np.stack([np.arange(n) if b % 2 == 0 else rng.permutation(n)
                       for b in range(B)]).astype(np.uint16)
    _check_vs_oracle([g, g + [0.5, 0, 0]], (np.arange(B) % 2).astype(np.int32), q, P_last)


def test_flags():
    rng = np.random.default_rng(5)
    n, B = 30, 6
    ps, fidx, q, P_last = _swarms(rng, n, B, 2, 20.0)
    P_last[1, 3] = P_last[1, 4]        # not a permutation -> BAD_INPUT
    q[2, 7, 1] = np.nan                # NaN cost -> NONFINITE
    q[3, 0, 0] = np.inf                # inf coordinate -> NaN costs
    P_cmp = np.stack([rng.permutation(n) for _ in range(B)]).astype(np.uint16)
    P_cmp[4, 0] = P_cmp[4, 1]          # P_cmp invalid -> CMP_INVALID
    fidx[5] = 7                        # formation out of range -> BAD_INPUT
    g = _check_vs_oracle(ps, np.minimum(fidx, 1), q, P_last, P_cmp)
    assert list(g["status"][:5]) == [0, 0x01, 0x02, 0x02, 0x04]
    g2 = _gpu(ps, fidx, q, P_last, P_cmp)
    assert g2["status"][5] == 0x01 and (g2["P_opt"][5] == 0xFFFF).all()


def test_cbaa_optimality_gap():
    # the comparator's purpose: price CBAA's consensus assignment under the
    # centralized alignment (assignment.py's docstring, :1-8)
    import torch
    import helpers as Hh
    from aclswarm_amd import engine
    Pf, A = Hh.simform("simform100_nc")
    dev = torch.device("cuda:0")
    rng = np.random.RandomState(11)
    points = [Pf[s, 0] for s in range(Pf.shape[0])]
    adjs = [A[s] for s in range(Pf.shape[0])]
    gains = [Hh.synth_gains(rng, a) for a in adjs]
    B = 32
    fidx = (np.arange(B) % len(points)).astype(np.int32)
    q = np.stack([Hh.random_positions(rng, 100, 44.7) for _ in range(B)])
    P_in = np.tile(np.arange(100, dtype=np.uint16), (B, 1))
    T = engine.FormationTable.from_host(points, adjs, gains, device=dev)
    out = engine.solve(T, torch.from_numpy(fidx).to(dev), torch.from_numpy(q).to(dev),
                       torch.zeros((B, 100, 3), dtype=torch.float64, device=dev),
                       torch.from_numpy(P_in.view(np.int16)).to(dev))
    P_cbaa = out["P_out"].cpu().numpy().view(np.uint16)
    g = _check_vs_oracle(list(points), fidx, q, P_in, P_cbaa)
    assert (g["status"] == 0).all()
    assert (g["cost"][:, 1] >= g["cost"][:, 0] * (1 - 1e-12)).all()


def test_reference_shaped_module():
    # aclswarm_amd.assignment mirrors assignment.py's names and returns
    from aclswarm_amd import assignment as A
    with open(os.path.join(HERE, "golden", "hungarian_golden.json")) as fh:
        cases = json.load(fh)["cases"][:4]
    for c in cases:
        q, p = np.array(c["q"]).T, np.array(c["p"]).T   # d x n, as the reference takes
        P, pal = A.find_optimal_assignment(q, p, c["last"])
        assert P == c["P"]
        np.testing.assert_allclose(pal, np.array(c["paligned"]).T, rtol=0, atol=1e-12)
        np.testing.assert_allclose(A.align(q, p).shape, p.shape)
    q, p = np.array(cases[0]["q"]).T, np.array(cases[0]["p"]).T
    with pytest.raises(ValueError):
        A.find_optimal_assignment(q, p, [0] * q.shape[1])
