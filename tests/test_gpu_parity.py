"""GPU parity: the HIP engine (through the C ABI) vs the CPU restatement.

Bar (BASELINE.json north_star): assignment permutations, CBAA tables and
round counts bit-exact; control commands within 1e-5 relative (fp64).
"""
import numpy as np
import pytest

import helpers as H
import pyoracle as O

pytestmark = pytest.mark.gpu

U_RTOL = 1e-5  # north_star: control commands within 1e-5 relative (fp64)


def _gpu_solve(points, adjs, gains, fidx, q, vel, P_in, early_exit=True, do_control=True,
               margin=True):
    import torch
    from aclswarm_amd import engine
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(points, adjs, gains, device=dev)
    out = engine.solve(
        T,
        torch.from_numpy(np.asarray(fidx, np.int32)).to(dev),
        torch.from_numpy(np.ascontiguousarray(q)).to(dev),
        torch.from_numpy(np.ascontiguousarray(vel)).to(dev),
        torch.from_numpy(np.asarray(P_in, np.uint16).view(np.int16)).to(dev),
        early_exit=early_exit, do_control=do_control, want_who=True,
        want_gate_margin=do_control, margin=margin)
    torch.cuda.synchronize()
    res = {k: v.cpu().numpy() for k, v in out.items()}
    res["P_out"] = res["P_out"].view(np.uint16)
    res["who"] = res["who"].view(np.uint16)
    res["status"] = np.ascontiguousarray(res["status"]).view(O.STATUS_DTYPE).reshape(-1)
    return res


def _oracle(points, adjs, gains, fidx, q, vel, P_in, early_exit=True):
    outs = []
    for b in range(q.shape[0]):
        f = fidx[b]
        outs.append(O.solve(q[b], vel[b], points[f], adjs[f], gains[f], P_in[b],
                            early_exit=early_exit))
    return outs


def _compare(gpu, ref, check_control=True):
    B = len(ref)
    worst = 0.0
    for b in range(B):
        r = ref[b]
        np.testing.assert_array_equal(gpu["who"][b], r["who"], err_msg=f"who swarm {b}")
        np.testing.assert_array_equal(gpu["P_out"][b], r["P_out"], err_msg=f"P_out swarm {b}")
        st = gpu["status"][b]
        for k in ("flags", "eff_rounds", "rounds", "n_invalid"):
            assert int(st[k]) == int(r["status"][k]), (b, k, st, r["status"])
        # decision margin: an exact function of the compared values (bit-exact)
        assert np.float32(st["margin"]) == np.float32(r["status"]["margin"]), (
            b, st["margin"], r["status"]["margin"])
        if check_control:
            # gate margin from the fast e (tolerance), the gates themselves exact
            gm, rg = float(gpu["gate_margin"][b]), r["gate_margin"]
            assert (gm == rg) if not np.isfinite(rg) else abs(gm - rg) <= 1e-10, (b, gm, rg)
            assert int(st["n_ca"]) == int(r["status"]["n_ca"]), (b, st, r["status"])
            np.testing.assert_array_equal(gpu["ca_flag"][b], r["ca"], err_msg=f"ca swarm {b}")
            for key, rk in (("u", "u"), ("u_safe", "u_safe")):
                scale = np.maximum(np.abs(r[rk]), 1.0)
                err = np.abs(gpu[key][b] - r[rk]) / scale
                worst = max(worst, float(err.max()))
                assert err.max() <= U_RTOL, (b, key, err.max())
    return worst


def test_swarm6_formations_yaml(cuda):
    """Config C1: formations.yaml swarm6_3d (3 formations, given gains), start.sh
    grid, identity and random P_in."""
    pts, adj, gains, q0 = H.swarm6()
    rng = np.random.RandomState(6)
    B = 48
    fidx = np.arange(B) % 3
    q = np.stack([q0 + (rng.normal(0, 0.2, q0.shape) if b >= 3 else 0) for b in range(B)])
    vel = rng.normal(0, 0.1, (B, 6, 3))
    P_in = np.stack([np.arange(6, dtype=np.uint16) if b < 6 else H.random_perm(rng, 6)
                     for b in range(B)])
    gpu = _gpu_solve(pts, adj, gains, fidx, q, vel, P_in)
    ref = _oracle(pts, adj, gains, fidx, q, vel, P_in)
    _compare(gpu, ref)


@pytest.mark.parametrize("name", ["simform20_fc", "simform20_nc"])
def test_simform20(cuda, name):
    """Config C2 shape (n=20, reference generator formations)."""
    P, A = H.simform(name)
    rng = np.random.RandomState(20)
    pts = [P[s, k] for s in range(P.shape[0]) for k in range(2)]
    adjs = [A[s] for s in range(P.shape[0]) for k in range(2)]
    gains = [H.synth_gains(rng, a) for a in adjs]
    B = 96
    fidx = rng.randint(0, len(pts), B)
    q = np.stack([H.random_positions(rng, 20, 20.0) for _ in range(B)])
    vel = rng.normal(0, 0.2, (B, 20, 3))
    P_in = np.stack([H.random_perm(rng, 20) if b % 2 else np.arange(20, dtype=np.uint16)
                     for b in range(B)])
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    ref = _oracle(pts, adjs, gains, fidx, q, vel, P_in)
    _compare(gpu, ref)


def test_c2_full_batch(cuda):
    """Config C2 at its full size: B = 4096 swarms on the 16 simform20_fc
    formations, every swarm against the CPU restatement's batch entry point
    (assignments, status and margin bit-exact, commands 1e-5)."""
    P, A = H.simform("simform20_fc")
    rng = np.random.RandomState(4096)
    pts = [P[s, k] for s in range(P.shape[0]) for k in range(2)]
    adjs = [A[s] for s in range(P.shape[0]) for k in range(2)]
    gains = [H.synth_gains(rng, a) for a in adjs]
    B, n = 4096, 20
    fidx = (np.arange(B) % len(pts)).astype(np.int32)
    q = np.stack([H.random_positions(rng, n, 20.0) for _ in range(B)])
    vel = rng.normal(0, 0.2, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) if b % 2 else np.arange(n, dtype=np.uint16)
                     for b in range(B)])
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    ref, _ = O.solve_batch(fidx, q, vel, np.stack(pts), np.stack(adjs), np.stack(gains), P_in,
                           nthreads=8)
    np.testing.assert_array_equal(gpu["P_out"], ref["P_out"])
    for k in ("flags", "eff_rounds", "rounds", "n_invalid", "n_ca"):
        np.testing.assert_array_equal(gpu["status"][k], ref["status"][k], err_msg=k)
    np.testing.assert_array_equal(gpu["status"]["margin"], ref["status"]["margin"])
    # the same swarms in reverse batch order (other co-resident workgroups,
    # other wave timing): a lost START bid from an unsynchronised table reset
    # showed up in some orders only
    rv = _gpu_solve(pts, adjs, gains, fidx[::-1].copy(), q[::-1].copy(), vel[::-1].copy(),
                    P_in[::-1].copy())
    np.testing.assert_array_equal(rv["P_out"][::-1], ref["P_out"])
    np.testing.assert_array_equal(rv["status"]["flags"][::-1], ref["status"]["flags"])
    np.testing.assert_array_equal(gpu["ca_flag"], ref["ca"])
    for k in ("u", "u_safe"):
        err = np.abs(gpu[k] - ref[k]) / np.maximum(np.abs(ref[k]), 1.0)
        assert err.max() <= U_RTOL, (k, err.max())


def test_simform100(cuda):
    """Config C3 shape (n=100 noncomplete, L=40 generator formations)."""
    P, A = H.simform("simform100_nc")
    rng = np.random.RandomState(100)
    pts = [P[s, k] for s in range(P.shape[0]) for k in range(2)]
    adjs = [A[s] for s in range(P.shape[0]) for k in range(2)]
    gains = [H.synth_gains(rng, a) for a in adjs]
    B = 24
    fidx = np.arange(B) % len(pts)
    q = np.stack([H.random_positions(rng, 100, 44.7) for _ in range(B)])
    vel = rng.normal(0, 0.2, (B, 100, 3))
    P_in = np.stack([H.random_perm(rng, 100) if b % 3 == 1 else np.arange(100, dtype=np.uint16)
                     for b in range(B)])
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    ref = _oracle(pts, adjs, gains, fidx, q, vel, P_in)
    _compare(gpu, ref)


def test_full_rounds_equal_early_exit(cuda):
    """early_exit=0 (all 2N rounds, the reference's literal schedule) gives the
    same tables as stopping at the fixed point."""
    P, A = H.simform("simform20_nc")
    rng = np.random.RandomState(7)
    pts = [P[0, 0], P[1, 1]]
    adjs = [A[0], A[1]]
    gains = [H.synth_gains(rng, a) for a in adjs]
    B = 16
    fidx = np.arange(B) % 2
    q = np.stack([H.random_positions(rng, 20, 20.0) for _ in range(B)])
    vel = np.zeros((B, 20, 3))
    P_in = np.stack([H.random_perm(rng, 20) for _ in range(B)])
    g1 = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in, early_exit=True)
    g0 = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in, early_exit=False)
    np.testing.assert_array_equal(g1["who"], g0["who"])
    np.testing.assert_array_equal(g1["P_out"], g0["P_out"])
    np.testing.assert_array_equal(g1["status"]["eff_rounds"], g0["status"]["eff_rounds"])
    ref = _oracle(pts, adjs, gains, fidx, q, vel, P_in, early_exit=False)
    _compare(g0, ref)


@pytest.mark.parametrize("n", [12, 140])
def test_price_signed_zeros_and_nonfinite_points(cuda, n):
    """The price phase drops the 0 * p terms of the aligned point when every
    formation coordinate is finite (signed zeros only, squared away): points
    and positions with exact +-0.0 coordinates must give the oracle's tables
    bit for bit; a formation with an infinite or NaN coordinate keeps the full
    expression (0 * inf = NaN). n = 140 runs the wide kernel."""
    rng = np.random.RandomState(n)
    adj = (rng.rand(n, n) < 0.7).astype(np.uint8)
    adj = np.triu(adj, 1)
    adj = adj + adj.T
    L = 4.5 * np.sqrt(n)  # (random_positions keeps a minimum spacing)
    pz = H.random_positions(rng, n, L)
    pz[: n // 2, 0] = 0.0
    pz[n // 4: n // 2, 1] = -0.0
    pz[::3, 2] = -0.0
    pz[1::3, 2] = 0.0
    p_inf = pz.copy()
    p_inf[2, 2] = np.inf
    p_nan = pz.copy()
    p_nan[3, 0] = np.nan
    pts = [pz, p_inf, p_nan]
    adjs = [adj] * 3
    gains = [H.synth_gains(rng, adj)] * 3
    B = 9
    fidx = np.arange(B) % 3
    q = np.stack([pz.copy() if b < 3 else H.random_positions(rng, n, L) for b in range(B)])
    q[3:6, : n // 3, 0] = -0.0
    q[3:6, n // 3: n // 2, 2] = 0.0
    vel = np.zeros((B, n, 3))
    P_in = np.stack([np.arange(n, dtype=np.uint16) if b % 2 else H.random_perm(rng, n)
                     for b in range(B)])
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in, do_control=False)
    ref = _oracle(pts, adjs, gains, fidx, q, vel, P_in)
    for r in ref:  # the oracle always runs the control stage; the GPU call did not
        r["status"]["flags"] = int(r["status"]["flags"]) & ~0x20  # ACL_SWARM_CA_ACTIVE
    _compare(gpu, ref, check_control=False)


def test_collision_avoidance_dense(cuda):
    """Crowded swarms: many vehicles inside d_avoid_thresh, wrap-around
    sectors, surrounded vehicles (safety.cpp:412-541)."""
    P, A = H.simform("simform20_fc")
    rng = np.random.RandomState(11)
    pts = [P[0, 0], P[2, 1], P[3, 0]]
    adjs = [A[0], A[2], A[3]]
    gains = [H.synth_gains(rng, a, scale=1.0) for a in adjs]
    B = 64
    fidx = np.arange(B) % 3
    q = np.stack([H.dense_positions(rng, 20, 4.0 + (b % 8)) for b in range(B)])
    vel = rng.normal(0, 0.5, (B, 20, 3))
    P_in = np.stack([H.random_perm(rng, 20) for _ in range(B)])
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    ref = _oracle(pts, adjs, gains, fidx, q, vel, P_in)
    assert sum(int(r["status"]["n_ca"]) for r in ref) > 100
    _compare(gpu, ref)


def test_edge_cases(cuda):
    """Invalid P_in (not a permutation), duplicate positions (price ties),
    n=1 and n=2 swarms, NaN positions."""
    rng = np.random.RandomState(3)
    # ties: all vehicles at the same spot -> equal prices across vehicles
    n = 8
    p = H.random_positions(rng, n, 10.0)
    adj = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
    adj[0, 5] = adj[5, 0] = 0
    G = H.synth_gains(rng, adj)
    B = 6
    q = np.stack([np.zeros((n, 3)), np.tile(p[:1], (n, 1)), p.copy(), p.copy(), p.copy(),
                  H.random_positions(rng, n, 10.0)])
    q[4, 3, 0] = np.nan
    P_in = np.stack([np.arange(n, dtype=np.uint16)] * B)
    P_in[2, 1] = P_in[2, 2]          # duplicate -> BAD_INPUT
    P_in[3, 0] = n + 3               # out of range -> BAD_INPUT
    vel = np.zeros((B, n, 3))
    gpu = _gpu_solve([p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in)
    ref = _oracle([p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in)
    assert gpu["status"]["flags"][2] & 0x10 and gpu["status"]["flags"][3] & 0x10
    assert gpu["status"]["flags"][4] & 0x08
    # NaN swarm: compare only the auction (control outputs are NaN on both sides)
    _compare({k: (v[:4] if k != "status" else v[:4]) for k, v in gpu.items()}, ref[:4])
    _compare({k: v[5:] for k, v in gpu.items()}, ref[5:])
    np.testing.assert_array_equal(gpu["who"][4], ref[4]["who"])
    np.testing.assert_array_equal(gpu["P_out"][4], ref[4]["P_out"])
    for n in (1, 2, 3):
        p = H.random_positions(rng, n, 6.0)
        adj = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
        G = H.synth_gains(rng, adj)
        q = np.stack([H.random_positions(rng, n, 6.0) for _ in range(4)])
        vel = np.zeros((4, n, 3))
        P_in = np.stack([H.random_perm(rng, n) for _ in range(4)])
        gpu = _gpu_solve([p], [adj], [G], np.zeros(4, np.int32), q, vel, P_in)
        ref = _oracle([p], [adj], [G], np.zeros(4, np.int32), q, vel, P_in)
        _compare(gpu, ref)


def test_max_n_128(cuda):
    """Largest supported swarm (two 64-bit mask words, u8 indices)."""
    rng = np.random.RandomState(128)
    n = 128
    p = H.random_positions(rng, n, 60.0)
    adj = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
    for _ in range(60):
        i, j = rng.randint(0, n, 2)
        adj[i, j] = adj[j, i] = 0
    G = H.synth_gains(rng, adj)
    B = 6
    q = np.stack([H.random_positions(rng, n, 60.0) for _ in range(B)])
    vel = rng.normal(0, 0.1, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    gpu = _gpu_solve([p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in)
    ref = _oracle([p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in)
    _compare(gpu, ref)


def _wide_case(rng, n, B, side, missing):
    p = H.random_positions(rng, n, side)
    p[:, 2] = rng.uniform(0.0, 2.0, n)
    adj = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
    for _ in range(missing):
        i, j = rng.randint(0, n, 2)
        adj[i, j] = adj[j, i] = 0
    G = H.synth_gains(rng, adj)
    q = np.stack([H.random_positions(rng, n, side) for _ in range(B)])
    vel = rng.normal(0, 0.1, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) if b % 2 else np.arange(n, dtype=np.uint16)
                     for b in range(B)])
    return [p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in


@pytest.mark.parametrize("n", [129, 200, 320])
def test_wide_n(cuda, n):
    """128 < n <= 512: the tables-in-HBM auction kernel (solve_wide.hip) and
    the control kernels with more than two 64-lane chunks, u16 indices."""
    rng = np.random.RandomState(n)
    side = 20.0 * (n / 20.0) ** 0.5
    args = _wide_case(rng, n, 3, side, n // 2)
    gpu = _gpu_solve(*args)
    ref = _oracle(*args)
    _compare(gpu, ref)


@pytest.mark.parametrize("early_exit", [True, False])
def test_wide_unconverged_and_sparse_graphs(cuda, early_exit):
    """n > 128 auctions that end at the 2n-round limit with re-selects in the
    last round (chain and lollipop formation graphs: consensus needs more
    than 2n lockstep rounds along a long path), and a 70%-dense graph whose
    column updates leave many vehicles on other entries: the wide kernel's
    sparse columns, their dense fallback and the fold-in of the last round's
    bids against the oracle, tables bit for bit."""
    rng = np.random.RandomState(136)
    pts, adjs = [], []
    for n_tail in (None, 60, 0):
        n = 136
        adj = np.zeros((n, n), np.uint8)
        perm = rng.permutation(n)
        if n_tail is None:      # a chain
            chain = perm
        elif n_tail == 0:       # 70% dense, no chain
            adj = np.triu((rng.rand(n, n) < 0.7).astype(np.uint8), 1)
            adj = adj + adj.T
            chain = perm[:0]
        else:                   # a lollipop: clique + tail
            core = perm[:n - n_tail]
            adj[np.ix_(core, core)] = 1
            np.fill_diagonal(adj, 0)
            chain = perm[n - n_tail - 1:]
        for x, y in zip(chain[:-1], chain[1:]):
            adj[x, y] = adj[y, x] = 1
        pts.append(np.c_[rng.uniform(-34, 34, (n, 2)), rng.uniform(0, 2, n)])
        adjs.append(adj)
    gains = [H.synth_gains(rng, a) for a in adjs]
    B = 6
    fidx = np.arange(B) % 3
    q = np.stack([np.c_[rng.uniform(-34, 34, (136, 2)), np.ones(136)] for _ in range(B)])
    vel = np.zeros((B, 136, 3))
    P_in = np.stack([H.random_perm(rng, 136) for _ in range(B)])
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in, early_exit=early_exit)
    ref = _oracle(pts, adjs, gains, fidx, q, vel, P_in, early_exit=early_exit)
    _compare(gpu, ref)
    # the chain / lollipop swarms really ran to the limit
    assert (gpu["status"]["eff_rounds"][fidx < 2] == 2 * 136).any()


def test_wide_collision_avoidance(cuda):
    """Crowded n = 160 swarms: the collision-avoidance list over three chunks."""
    rng = np.random.RandomState(160)
    n = 160
    p = H.random_positions(rng, n, 56.0)
    adj = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
    G = H.synth_gains(rng, adj, scale=1.0)
    B = 3
    q = np.stack([H.dense_positions(rng, n, 14.0 + 2 * b) for b in range(B)])
    vel = rng.normal(0, 0.5, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    args = ([p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in)
    gpu = _gpu_solve(*args)
    ref = _oracle(*args)
    assert sum(int(r["status"]["n_ca"]) for r in ref) > 20
    _compare(gpu, ref)


@pytest.mark.parametrize("n", [24, 64, 128, 200])
def test_collision_avoidance_packed(cuda, n):
    """Packed swarms: most vehicles have more than 16 others within
    d_avoid_thresh (more than 64 sector edges: ca_kernel's rank-sort path),
    beside sparser swarms of the same batch (the bitonic paths)."""
    from aclswarm_amd import _lib
    rng = np.random.RandomState(900 + n)
    p = H.random_positions(rng, n, 3.0 * n)
    adj = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
    G = H.synth_gains(rng, adj, scale=1.0)
    B = 4
    side = [2.0, 3.0, 0.25 * n ** 0.5 + 2.0, 0.6 * n ** 0.5 + 3.0]
    q = np.stack([H.dense_positions(rng, n, side[b]) for b in range(B)])
    vel = rng.normal(0, 0.5, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    thr = _lib.default_safety().d_avoid_thresh
    d = np.hypot(q[:, :, None, 0] - q[:, None, :, 0], q[:, :, None, 1] - q[:, None, :, 1])
    close = (d <= thr).sum(axis=2) - 1
    assert (close > 16).sum() > n // 2 and ((close > 0) & (close <= 16)).sum() > 0
    args = ([p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in)
    gpu = _gpu_solve(*args)
    ref = _oracle(*args)
    assert sum(int(r["status"]["n_ca"]) for r in ref) > n // 2
    _compare(gpu, ref)


def _c4_inputs(B, seed):
    """Config C4: simform500 formations (N=500, L=90, the reference generator's
    own output, tests/golden/simform500_nc.npz), u16 indices."""
    P, A = H.simform("simform500_nc")
    rng = np.random.RandomState(seed)
    pts = [P[s, k] for s in range(P.shape[0]) for k in range(2)]
    adjs = [A[s] for s in range(P.shape[0]) for k in range(2)]
    gains = [H.synth_gains(rng, a) for a in adjs]
    n = 500
    fidx = np.arange(B) % len(pts)
    q = np.stack([H.random_positions(rng, n, 20.0 * (n / 20.0) ** 0.5) for _ in range(B)])
    vel = rng.normal(0, 0.1, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) if b % 2 else np.arange(n, dtype=np.uint16)
                     for b in range(B)])
    return pts, adjs, gains, fidx, q, vel, P_in


def test_n500_config_c4(cuda):
    """Config C4 (simform500 formations): every output of three swarms against
    the CPU restatement (~8 s of oracle time per swarm)."""
    args = _c4_inputs(3, 500)
    gpu = _gpu_solve(*args)
    ref = _oracle(*args)
    _compare(gpu, ref)


def test_c4_batch_sampled(cuda):
    """C4 at a batch of 256 swarms (the tables-in-HBM kernel with many
    workgroups in flight): every P_out a permutation, status valid, a second
    run bit-identical, and two sampled swarms against the oracle."""
    B = 256
    pts, adjs, gains, fidx, q, vel, P_in = _c4_inputs(B, 501)
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    again = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    for k in ("P_out", "who", "u", "u_safe"):
        np.testing.assert_array_equal(gpu[k], again[k])
    assert (gpu["status"]["flags"] & 0x01).all()  # valid
    srt = np.sort(gpu["P_out"].astype(np.int64), axis=1)
    assert (srt == np.arange(500)).all()
    for b in (17, 200):
        ref = _oracle(pts, adjs, gains, fidx[[b]], q[[b]], vel[[b]], P_in[[b]])
        _compare({k: v[[b]] for k, v in gpu.items()}, ref)


def test_control_batch_given_assignment(cuda):
    """acl_control_batch (DistCntrl + Safety with given P, no auction) against
    the oracle's DistCntrl::compute / saturation / collisionAvoidance, and a
    non-permutation P -> BAD_INPUT."""
    import torch
    from aclswarm_amd import engine
    P20, A20 = H.simform("simform20_fc")
    rng = np.random.RandomState(21)
    pts = [P20[0, 0], P20[1, 1]]
    adjs = [A20[0], A20[1]]
    gains = [H.synth_gains(rng, a, scale=1.0) for a in adjs]
    B, n = 12, 20
    fidx = np.arange(B) % 2
    q = np.stack([H.dense_positions(rng, n, 6.0 + b) for b in range(B)])
    vel = rng.normal(0, 0.3, (B, n, 3))
    P = np.stack([H.random_perm(rng, n) for _ in range(B)])
    P[3, 4] = P[3, 5]                                   # not a permutation
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(pts, adjs, gains, device=dev)
    out = engine.control(T, torch.from_numpy(fidx.astype(np.int32)).to(dev),
                         torch.from_numpy(q).to(dev), torch.from_numpy(vel).to(dev),
                         torch.from_numpy(P.astype(np.uint16).view(np.int16)).to(dev))
    torch.cuda.synchronize()
    u = out["u"].cpu().numpy(); us = out["u_safe"].cpu().numpy()
    ca = out["ca_flag"].cpu().numpy()
    st = engine.status_to_numpy(out["status"])
    assert st["flags"][3] & 0x10 and not np.any(us[3])
    nca = 0
    for b in range(B):
        if b == 3:
            continue
        f = fidx[b]
        Pt = np.argsort(P[b]).astype(np.uint16)
        for v in range(n):
            ur = O.control(v, q[b], vel[b, v], Pt, adjs[f], gains[f], pts[f])
            sr, mod = O.collision_avoidance(v, q[b], O.saturate(ur))
            np.testing.assert_allclose(u[b, v], ur, rtol=U_RTOL, atol=U_RTOL)
            np.testing.assert_allclose(us[b, v], sr, rtol=U_RTOL, atol=U_RTOL)
            assert bool(ca[b, v]) == mod
            nca += mod
        assert int(st["n_ca"][b]) == int(ca[b].sum())
    assert nca > 10


def test_align_rt_output(cuda):
    """solve's optional align_Rt is each vehicle's Auctioneer::alignFormation
    (R, t), bit-exact against the oracle (the logAssignment `aligned`)."""
    import torch
    from aclswarm_amd import engine
    P20, A20 = H.simform("simform20_nc")
    rng = np.random.RandomState(5)
    pts = [P20[0, 0]]
    adjs = [A20[0]]
    gains = [H.synth_gains(rng, A20[0])]
    for n_, (pts_, adjs_, gains_) in ((20, (pts, adjs, gains)),):
        B = 6
        q = np.stack([H.random_positions(rng, n_, 20.0) for _ in range(B)])
        Pin = np.stack([H.random_perm(rng, n_) for _ in range(B)])
        dev = torch.device("cuda:0")
        T = engine.FormationTable.from_host(pts_, adjs_, gains_, device=dev)
        out = engine.solve(T, torch.zeros(B, dtype=torch.int32, device=dev),
                           torch.from_numpy(q).to(dev), torch.zeros((B, n_, 3), dtype=torch.float64, device=dev),
                           torch.from_numpy(Pin.view(np.int16)).to(dev), want_align=True)
        torch.cuda.synchronize()
        Rt = out["align_Rt"].cpu().numpy()
        for b in range(B):
            _, Rt_ref = O.prices(q[b], pts_[0], adjs_[0], Pin[b])
            np.testing.assert_array_equal(Rt[b], Rt_ref)


def test_gain_layouts_5_and_9_planes(cuda):
    """ADMM-structured gains: the 5-entry record table gives the commands of
    the 9-plane table of the same GainMat (to summation order); unstructured
    blocks (9 planes only) match the oracle."""
    import torch
    from aclswarm_amd import engine
    P20, A20 = H.simform("simform20_nc")
    rng = np.random.RandomState(59)
    pts = [P20[s, 0] for s in range(4)]
    adjs = [A20[s] for s in range(4)]
    B, n = 64, 20
    fidx = np.arange(B) % 4
    q = np.stack([H.dense_positions(rng, n, 9.0 + b % 5) for b in range(B)])
    vel = rng.normal(0, 0.3, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    dev = torch.device("cuda:0")

    def run(gains, planes):
        T = engine.FormationTable.from_host(pts, adjs, gains, device=dev, planes=planes)
        assert T.gain_planes == (planes or T.gain_planes)
        out = engine.solve(T, torch.from_numpy(fidx.astype(np.int32)).to(dev),
                           torch.from_numpy(q).to(dev), torch.from_numpy(vel).to(dev),
                           torch.from_numpy(P_in.astype(np.uint16).view(np.int16)).to(dev))
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in out.items()}, T.gain_planes

    structured = [H.synth_gains(rng, a, scale=1.0) for a in adjs]
    r5, np5 = run(structured, None)
    r9, np9 = run(structured, 9)
    assert (np5, np9) == (5, 9)
    # the 5-entry table runs gain_pair_kernel (one evaluation per undirected
    # edge), the 9-plane table the directed walk: same terms, different
    # summation order
    for k in ("ca_flag", "P_out"):
        np.testing.assert_array_equal(r5[k], r9[k], err_msg=k)
    for k in ("u", "u_safe"):
        np.testing.assert_allclose(r5[k], r9[k], rtol=1e-12, atol=1e-12, err_msg=k)
    general = [H.random_block_gains(rng, a, scale=1.0) for a in adjs]
    gpu = _gpu_solve(pts, adjs, general, fidx, q, vel, P_in)
    ref = _oracle(pts, adjs, general, fidx, q, vel, P_in)
    _compare(gpu, ref)


def _tile_order(adj):
    """Row-major edge index of every record in acl_tile_gains order (the
    layout include/aclswarm_amd.h documents), restated on the host."""
    n = adj.shape[0]
    eidx = -np.ones((n, n), np.int64)
    ii, jj = np.nonzero(adj)
    eidx[ii, jj] = np.arange(ii.size)
    nb = (n + 7) // 8
    order = []
    for I in range(nb):
        for J in range(I, nb):
            for run in (1, 2):  # lane order: edge (i, j), then edge (j, i)
                for r in range(8):
                    for c in range(8):
                        i, j = 8 * I + r, 8 * J + c
                        if I == J and (r > c or (run == 2 and r == c)):
                            continue
                        if run == 2:
                            i, j = j, i
                        if i < n and j < n and adj[i, j]:
                            order.append(eidx[i, j])
    return np.array(order, np.int64)


@pytest.mark.parametrize("n,complete", [(1, True), (7, True), (20, False), (37, False),
                                        (100, False), (128, False)])
def test_tiled_gain_records(cuda, n, complete):
    """acl_tile_gains writes the records in the documented tile order, and the
    pair kernel of acl_control_batch reading the tiled copy gives the same
    commands, bit for bit, as reading the row-major records (same terms, same
    summation order). (acl_solve_batch's fused control phase reads the
    row-major records whatever the table holds.)"""
    import torch
    from aclswarm_amd import engine
    rng = np.random.RandomState(1000 + n)
    F, B = 3, 24
    pts, adjs = [], []
    for f in range(F):
        p = np.c_[rng.uniform(-n, n, (n, 2)), rng.uniform(0, 2, n)]
        a = np.ones((n, n), np.uint8) - np.eye(n, dtype=np.uint8)
        if not complete:
            for _ in range(max(1, n // 3)):
                i, j = rng.randint(0, n, 2)
                if i != j:
                    a[i, j] = a[j, i] = 0
        if f == 1 and n > 1:
            a[0, 0] = 1  # a diagonal edge is an edge of the control law too
        pts.append(p)
        adjs.append(a)
    gains = [H.synth_gains(rng, a, scale=1.0) for a in adjs]
    for G in gains:  # the diagonal row sums carry -0.0 at the structural zeros
        for i in range(n):
            G[3 * i + np.array([0, 1, 2, 2]), 3 * i + np.array([2, 2, 0, 1])] = 0.0
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(pts, adjs, gains, device=dev, planes=5)
    assert T.gain_planes == 5
    T.tile_gains()
    torch.cuda.synchronize()
    assert T.gains_tiled is not None
    rows = T.gains.cpu().numpy()
    tiled = T.gains_tiled.cpu().numpy()
    off = 0
    for f in range(F):
        order = _tile_order(adjs[f])
        E = order.size
        want = rows[5 * off:5 * (off + E)].reshape(E, 5)[order]
        np.testing.assert_array_equal(tiled[5 * off:5 * (off + E)].reshape(E, 5), want)
        off += E
    fidx = torch.from_numpy((np.arange(B) % F).astype(np.int32)).to(dev)
    q = torch.from_numpy(np.stack([H.dense_positions(rng, n, 2.0 * n) for _ in range(B)])).to(dev)
    vel = torch.from_numpy(rng.normal(0, 0.3, (B, n, 3))).to(dev)
    P_in = torch.from_numpy(np.stack([H.random_perm(rng, n) for _ in range(B)])
                            .astype(np.uint16).view(np.int16)).to(dev)
    P = engine.solve(T, fidx, q, vel, P_in)["P_out"]
    r_t = {k: v.cpu().numpy() for k, v in engine.control(T, fidx, q, vel, P).items()}
    T.gains_tiled = None
    r_r = {k: v.cpu().numpy() for k, v in engine.control(T, fidx, q, vel, P).items()}
    for k in ("ca_flag", "u", "u_safe"):
        np.testing.assert_array_equal(r_t[k], r_r[k], err_msg=k)
