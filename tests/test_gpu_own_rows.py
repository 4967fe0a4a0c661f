"""GPU: auctions from the vehicles' own assignments (acl_solve_args_t::P_rows,
ABI 8). While the vehicles of a swarm hold different assignments -- an
episode after a disagreeing auction -- each reference vehicle aligns the
formation with its own P_ / Pt_ (auctioneer.cpp:357,369), takes its CBAA
neighbours from them (bidIterComplete, :422-427) and keeps its own when its
final table is invalid. Checked through the C ABI against the oracle's
orc_solve_rows (tables, assignments, flags, margins bit-exact; commands 1e-5
relative) on the n <= 64 inline-alignment kernel, the 65 ... 128 kernel and
the wide (n > 128) kernel, mixed with swarms that use P_in."""
import numpy as np
import pytest

import pyoracle as O
from test_gpu_fused import _case
from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu


def _own_rows(rng, P_in, frac):
    """Each vehicle's table: the shared inverse of P_in, or (for a fraction of
    the vehicles) another permutation that still puts the vehicle at its own
    point -- two other entries swapped, several times."""
    n = len(P_in)
    Pt = np.zeros(n, np.uint16)
    Pt[P_in] = np.arange(n, dtype=np.uint16)
    rows = np.tile(Pt, (n, 1))
    for v in range(n):
        if rng.rand() < frac:
            others = [j for j in range(n) if j != P_in[v]]
            for _ in range(max(1, n // 8)):
                a, c = rng.choice(others, 2, replace=False)
                rows[v, a], rows[v, c] = rows[v, c], rows[v, a]
            assert rows[v, P_in[v]] == v
    return rows


def _run(pts, adjs, gains, fidx, q, vel, P_in, rows, on, margin=True):
    import torch
    from aclswarm_amd import engine
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(pts, adjs, gains, device=dev)
    out = engine.solve(
        T, torch.from_numpy(np.asarray(fidx, np.int32)).to(dev),
        torch.from_numpy(np.ascontiguousarray(q)).to(dev),
        torch.from_numpy(np.ascontiguousarray(vel)).to(dev),
        torch.from_numpy(np.asarray(P_in, np.uint16).view(np.int16)).to(dev),
        want_who=True, want_gate_margin=True, margin=margin,
        P_rows=torch.from_numpy(np.ascontiguousarray(rows, np.uint16).view(np.int16)).to(dev),
        P_rows_on=torch.from_numpy(np.asarray(on, np.uint8)).to(dev))
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in out.items()}
    res["P_out"] = res["P_out"].view(np.uint16)
    res["who"] = res["who"].view(np.uint16)
    res["status"] = np.ascontiguousarray(res["status"]).view(O.STATUS_DTYPE).reshape(-1)
    return res


def _oracle_rows(pts, adjs, gains, fidx, q, vel, P_in, rows, on):
    return [O.solve(q[b], vel[b], pts[fidx[b]], adjs[fidx[b]], gains[fidx[b]], P_in[b],
                    P_rows=rows[b] if on[b] else None) for b in range(q.shape[0])]


@pytest.mark.parametrize("n", [7, 20, 64, 100, 128, 160])
def test_own_rows_match_oracle(cuda, n):
    rng = np.random.RandomState(8100 + n)
    F, B = 3, 24 if n <= 128 else 8
    pts, adjs, gains = _case(rng, n, F, disconnected=True)
    fidx = np.arange(B) % F
    q = np.stack([np.c_[rng.uniform(-n, n, (n, 2)), np.ones(n)] for _ in range(B)])
    vel = rng.normal(0, 0.3, (B, n, 3))
    P_in = np.stack([rng.permutation(n).astype(np.uint16) for _ in range(B)])
    rows = np.stack([_own_rows(rng, P_in[b], 0.5 if b % 4 else 0.0) for b in range(B)])
    on = (np.arange(B) % 3 != 2).astype(np.uint8)  # every third swarm uses P_in alone
    gpu = _run(pts, adjs, gains, fidx, q, vel, P_in, rows, on)
    ref = _oracle_rows(pts, adjs, gains, fidx, q, vel, P_in, rows, on)
    _compare(gpu, ref)
    # the rows matter: some swarm's tables differ from its P_in-only auction
    shared = _oracle_rows(pts, adjs, gains, fidx, q, vel, P_in, rows, np.zeros(B, np.uint8))
    assert any(not np.array_equal(ref[b]["who"], shared[b]["who"]) for b in range(B)
               if on[b] and b % 4)
    # identical rows (b % 4 == 0) are the shared auction bit for bit
    for b in range(0, B, 4):
        np.testing.assert_array_equal(ref[b]["who"], shared[b]["who"])


@pytest.mark.parametrize("n", [20, 100, 160])
def test_own_rows_bad_rows_are_bad_input(cuda, n):
    """A row that is not a permutation, or that does not hold its vehicle at
    the vehicle's P_in point, makes the swarm BAD_INPUT (as a bad P_in)."""
    rng = np.random.RandomState(8200 + n)
    F, B = 2, 6
    pts, adjs, gains = _case(rng, n, F, disconnected=False)
    fidx = np.arange(B) % F
    q = np.stack([np.c_[rng.uniform(-n, n, (n, 2)), np.ones(n)] for _ in range(B)])
    vel = np.zeros((B, n, 3))
    P_in = np.stack([rng.permutation(n).astype(np.uint16) for _ in range(B)])
    rows = np.stack([_own_rows(rng, P_in[b], 0.3) for b in range(B)])
    rows[1, 3, 0] = rows[1, 3, 1]                     # a duplicate entry
    v = 5
    j = (int(P_in[2, v]) + 1) % n
    rows[2, v, P_in[2, v]], rows[2, v, j] = rows[2, v, j], rows[2, v, P_in[2, v]]  # v moved
    rows[3, 0, 0] = n                                 # out of range
    on = np.ones(B, np.uint8)
    gpu = _run(pts, adjs, gains, fidx, q, vel, P_in, rows, on)
    ref = _oracle_rows(pts, adjs, gains, fidx, q, vel, P_in, rows, on)
    for b in (1, 2, 3):
        assert gpu["status"]["flags"][b] & 0x10, b  # ACL_SWARM_BAD_INPUT
        assert ref[b]["status"]["flags"] & 0x10, b
    _compare(gpu, ref)
