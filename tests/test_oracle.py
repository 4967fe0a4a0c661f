"""CPU suite: the oracle against the reference's golden vectors and against
independent formulations (runs without a GPU)."""
import numpy as np
import pytest

import helpers as H
import pyoracle as O


# --------------------------------------------------------------- alignment --

def test_umeyama_matches_reference_arun():
    """Pinned: Eigen-umeyama restatement vs the reference's own Python
    Procrustes (assignment.py:15-53) on committed golden vectors."""
    d = H.load_json("arun_golden.json")
    assert len(d["cases"]) >= 50
    for c in d["cases"]:
        R, t = O.umeyama2(np.array(c["p"]), np.array(c["q"]))
        np.testing.assert_allclose(R, np.array(c["R"]), atol=1e-12)
        np.testing.assert_allclose(t, np.array(c["t"]), atol=1e-10)


def test_jacobi_svd_properties():
    rng = np.random.RandomState(0)
    mats = [rng.normal(size=(2, 2)) * 10 ** rng.uniform(-6, 6) for _ in range(400)]
    mats += [np.zeros((2, 2)), np.eye(2), np.diag([3.0, -2.0]), np.array([[1, 2], [2, 4.0]]),
             np.array([[0, 1], [0, 0.0]]), np.array([[1e-300, 0], [0, 1e-300]]),
             np.array([[5, 0], [0, 7.0]]), np.array([[0, -3], [3, 0.0]])]
    for A in mats:
        rc, U, s, V = O.jacobi_svd2(A)
        assert rc == 0
        assert s[0] >= s[1] >= 0
        np.testing.assert_allclose(U @ U.T, np.eye(2), atol=1e-14)
        np.testing.assert_allclose(V @ V.T, np.eye(2), atol=1e-14)
        np.testing.assert_allclose(U @ np.diag(s) @ V.T, A, atol=1e-13 * max(1, np.abs(A).max()))
        np.testing.assert_allclose(s, np.linalg.svd(A, compute_uv=False),
                                   atol=1e-13 * max(1, np.abs(A).max()))
    rc, *_ = O.jacobi_svd2(np.array([[np.nan, 0], [0, 1.0]]))
    assert rc == -1


def test_umeyama_variants_agree_full_rank():
    """Eigen 3.3 (rank rule) and 3.4 (det(U)det(V) rule) differ only on
    rank-deficient neighbourhoods."""
    rng = np.random.RandomState(1)
    for _ in range(200):
        k = rng.randint(3, 30)
        src = rng.uniform(-5, 5, (k, 2))
        dst = src @ np.array([[0.6, -0.8], [0.8, 0.6]]).T + rng.normal(0, 0.5, (k, 2))
        R0, t0 = O.umeyama2(src, dst, 0)
        R1, t1 = O.umeyama2(src, dst, 1)
        np.testing.assert_array_equal(R0, R1)
        np.testing.assert_array_equal(t0, t1)
        assert abs(np.linalg.det(R0) - 1) < 1e-12


def test_alignment_collinear_is_rotation():
    """Rank-deficient (collinear) neighbourhood, swarm4 'Line'-like: still a
    proper rotation (3.3 rank-1 branch)."""
    src = np.array([[0, 0], [1, 0], [2, 0], [3, 0.0]])
    dst = np.array([[5, 5], [5, 6], [5, 7], [5, 8.0]])
    R, t = O.umeyama2(src, dst, 0)
    assert abs(np.linalg.det(R) - 1) < 1e-12
    np.testing.assert_allclose(R @ src.T + t[:, None], dst.T, atol=1e-12)


# --------------------------------------------------------------------- CBAA --

def _gap(hi, lo):
    """Relative gap of one decisive comparison of f32 values hi >= lo >= 0
    (include/aclswarm_amd.h): (hi - lo) / hi in double (the numerator is
    exact there), 1 when lo < 2^-28 hi."""
    hi, lo = float(hi), float(lo)
    if lo * 2.0 ** 28 < hi:
        return 1.0
    return (hi - lo) / hi


def _py_cbaa(C, adj, P, rounds, gaps=None):
    """Second, independent formulation of the lockstep CBAA (App. A) with
    explicit (price, who) pairs, pure Python, for small n. With a list
    `gaps`, appends the gap of every decisive comparison (the literal
    definition of the decision margin: the minimum over them)."""
    n = C.shape[0]
    nb = [[u for u in range(n) if u == v or adj[P[v], P[u]]] for v in range(n)]
    price = np.zeros((n, n), np.float32)
    who = -np.ones((n, n), np.int64)

    def select(v, pr, wh):
        best, task, ok = np.float32(0), 0, False
        for j in range(n):
            c = C[v, j]
            if c > best and c > pr[j]:
                best, task, ok = c, j, True
        if gaps is not None:
            js = task if ok else -1
            for k in range(n):
                c = C[v, k]
                if wh[k] == v:
                    continue
                if k == js:
                    gaps.append(_gap(c, pr[k]))
                elif c > pr[k] and c > 0:
                    gaps.append(_gap(best, c))
                elif c > 0 and (js < 0 or c > best or (c == best and k < js)):
                    gaps.append(_gap(pr[k], c))
        if ok:
            pr[task], wh[task] = best, v

    for v in range(n):
        select(v, price[v], who[v])
    for _ in range(rounds):
        np_, nw_ = price.copy(), who.copy()
        for v in range(n):
            outbid = False
            for j in range(n):
                win = nb[v][0]
                for u in nb[v]:
                    if price[u, j] > price[win, j]:
                        win = u
                if gaps is not None:
                    others = [price[u, j] for u in nb[v] if who[u, j] != who[win, j]]
                    if others:
                        gaps.append(_gap(price[win, j], max(others)))
                if who[v, j] == v and who[win, j] != v:
                    outbid = True
                nw_[v, j], np_[v, j] = who[win, j], price[win, j]
            if outbid:
                select(v, np_[v], nw_[v])
        price, who = np_, nw_
    return who, price


def test_cbaa_independent_formulation():
    P, A = H.simform("simform20_nc")
    rng = np.random.RandomState(5)
    for s in range(3):
        n = 20
        p = P[s, 0]
        adj = A[s]
        q = H.random_positions(rng, n, 20.0)
        Pin = H.random_perm(rng, n)
        C, _ = O.prices(q, p, adj, Pin)
        who, pr, eff = O.cbaa(C, adj, Pin, early_exit=False)
        who2, pr2 = _py_cbaa(C, adj, Pin, 2 * n)
        np.testing.assert_array_equal(who, who2)
        np.testing.assert_array_equal(pr, pr2)


def test_margin_independent_formulation():
    """The decision margin (include/aclswarm_amd.h) of the oracle equals the
    literal minimum over every decisive comparison of the pure-Python CBAA
    (a different evaluation order: every (v, j) every round, plain min over
    rounded gaps), and the swarm margin is min(CBAA, alignment) as f32."""
    for name, L in (("simform20_nc", 20.0), ("simform20_fc", 20.0)):
        P, A = H.simform(name)
        rng = np.random.RandomState(11)
        for s in range(3):
            n = P.shape[2]
            q = H.random_positions(rng, n, L)
            Pin = H.random_perm(rng, n)
            C, _, ga = O.prices_gap(q, P[s, 0], A[s], Pin)
            who, pr, eff, gc = O.cbaa_margin(C, A[s], Pin, early_exit=False)
            gaps = []
            _py_cbaa(C, A[s], Pin, 2 * n, gaps)
            assert gc == min(gaps + [1.0])
            r = O.solve(q, np.zeros((n, 3)), P[s, 0], A[s], np.zeros((3 * n, 3 * n)), Pin)
            assert r["status"]["margin"] == np.float32(min(gc, ga))
            assert bool(r["status"]["flags"] & 0x40) == (min(gc, ga) < 1e-6)
            # the early exit drops only repeated evaluations
            _, _, _, ge = O.cbaa_margin(C, A[s], Pin, early_exit=True)
            assert ge == gc


def test_margin_ties_are_fragile():
    """Two vehicles with bit-identical prices for a task they both want: the
    update (or select) is decided by vehid order alone -> margin 0, FRAGILE."""
    n = 6
    adj = np.ones((n, n), np.uint8) - np.eye(n, dtype=np.uint8)
    C = np.random.RandomState(4).uniform(0.1, 1.0, (n, n)).astype(np.float32)
    C[0, 3] = C[1, 3] = np.float32(5.0)   # vehicles 0 and 1 both prefer task 3 equally
    _, _, _, g = O.cbaa_margin(C, adj, np.arange(n, dtype=np.uint16), early_exit=False)
    assert g == 0.0
    gaps = []
    _py_cbaa(C, adj, np.arange(n), 2 * n, gaps)
    assert min(gaps) == 0.0
    C[1, 3] = np.float32(4.0)             # distinct prices: no tie
    _, _, _, g2 = O.cbaa_margin(C, adj, np.arange(n, dtype=np.uint16), early_exit=False)
    gaps = []
    _py_cbaa(C, adj, np.arange(n), 2 * n, gaps)
    assert g2 == min(gaps) > 0.0


def test_alignment_gap():
    """Alignment decision gap: the determinant-sign and rank tests of
    Eigen::umeyama (3.3.x), against numpy on the same cross-covariance."""
    rng = np.random.RandomState(3)
    for _ in range(100):
        k = rng.randint(3, 25)
        src = rng.uniform(-5, 5, (k, 2))
        dst = rng.uniform(-5, 5, (k, 2))
        _, _, g = O.umeyama2_gap(src, dst)
        S = (dst - dst.mean(0)).T @ (src - src.mean(0)) / k
        s = np.linalg.svd(S, compute_uv=False)
        gd = abs(np.linalg.det(S)) / (abs(S[0, 0] * S[1, 1]) + abs(S[0, 1] * S[1, 0]))
        gr = abs(s[1] - 1e-12 * s[0]) / max(s[1], 1e-12 * s[0])
        assert abs(g - min(gd, gr, 1.0)) < 1e-9
    # collinear points: rank 1 -> the rank test is decided by 1e-12 s0 vs ~0
    src = np.array([[0, 0], [1, 0], [2, 0], [3, 0.0]])
    dst = np.array([[5, 5], [5, 6], [5, 7], [5, 8.0]])
    _, _, g = O.umeyama2_gap(src, dst)
    assert g == 0.0 or g > 0.5  # det exactly 0 -> 0


def test_cbaa_early_exit_exact_and_invariants():
    """Fixed-point exit is exact; price == C[who][j] (the table invariant the
    GPU kernel relies on); consensus is a valid permutation on the
    generator's (always connected) graphs."""
    for name in ("simform20_fc", "simform20_nc"):
        P, A = H.simform(name)
        rng = np.random.RandomState(2)
        for s in range(P.shape[0]):
            n = P.shape[2]
            q = H.random_positions(rng, n, 20.0)
            Pin = H.random_perm(rng, n)
            C, _ = O.prices(q, P[s, 1], A[s], Pin)
            w1, p1, e1 = O.cbaa(C, A[s], Pin, True)
            w0, p0, e0 = O.cbaa(C, A[s], Pin, False)
            np.testing.assert_array_equal(w1, w0)
            np.testing.assert_array_equal(p1, p0)
            assert e1 == e0 and 0 < e0 <= 2 * n
            ref_price = np.where(w0 >= 0, C[np.maximum(w0, 0), np.arange(n)[None, :]], 0)
            np.testing.assert_array_equal(p0, ref_price.astype(np.float32))
            assert (w0 == w0[0]).all()
            assert sorted(w0[0]) == list(range(n))


def test_swarm6_c1_solve():
    """Config C1 on the CPU: formations.yaml swarm6_3d from the start.sh grid."""
    pts, adj, gains, q0 = H.swarm6()
    for f in range(3):
        r = O.solve(q0, np.zeros((6, 3)), pts[f], adj[f], gains[f], np.arange(6))
        assert r["status"]["flags"] & 0x3 == 0x3  # valid and agree
        assert sorted(r["P_out"]) == list(range(6))
        assert r["status"]["rounds"] == 12
        r0 = O.solve(q0, np.zeros((6, 3)), pts[f], adj[f], gains[f], np.arange(6),
                     early_exit=False)
        np.testing.assert_array_equal(r["P_out"], r0["P_out"])


# ---------------------------------------------------------------- control --

def test_pdist_gram_formula():
    rng = np.random.RandomState(4)
    p = rng.uniform(-10, 10, (30, 3))
    dxy, dz = O.pdist(p)
    ref_xy = np.hypot(p[:, None, 0] - p[None, :, 0], p[:, None, 1] - p[None, :, 1])
    ref_z = np.abs(p[:, None, 2] - p[None, :, 2])
    ok = ~np.isnan(dxy)
    np.testing.assert_allclose(dxy[ok], ref_xy[ok], atol=1e-6)
    okz = ~np.isnan(dz)
    np.testing.assert_allclose(dz[okz], ref_z[okz], atol=1e-6)


def test_control_vs_numpy():
    """DistCntrl::compute against a direct numpy formulation."""
    pts, adj, gains, q0 = H.swarm6()
    rng = np.random.RandomState(9)
    g = O.default_gains()
    for f in range(3):
        p, A, G = pts[f], adj[f], gains[f]
        n = 6
        dxy, dz = O.pdist(p)
        for trial in range(5):
            q = q0 + rng.normal(0, 0.5, q0.shape)
            Pt = H.random_perm(rng, n)
            for v in range(n):
                vel = rng.normal(0, 0.2, 3)
                u = O.control(v, q, vel, Pt, A, G, p)
                i = int(np.where(Pt == v)[0][0])
                ref = np.zeros(3)
                for j in range(n):
                    if not A[i, j]:
                        continue
                    qij = q[Pt[j]] - q[v]
                    exy = np.hypot(qij[0], qij[1]) - dxy[i, j]
                    ez = abs(qij[2]) - dz[i, j]
                    F = np.zeros(3)
                    if abs(exy) > g.e_xy_thr:
                        F[:2] = g.K1_xy * np.arctan(g.K2_xy * exy)
                    if abs(ez) > g.e_z_thr:
                        F[2] = g.K1_z * np.arctan(g.K2_z * ez)
                    ref += g.kp * (G[3 * i:3 * i + 3, 3 * j:3 * j + 3] @ qij + F * qij) - g.kd * vel
                np.testing.assert_allclose(u, ref, rtol=1e-12, atol=1e-12)


# ----------------------------------------------------------------- safety --

def test_saturation():
    np.testing.assert_allclose(O.saturate([3.0, 4.0, 1.0]), [0.3, 0.4, 0.3])
    np.testing.assert_allclose(O.saturate([0.1, 0.1, -0.1]), [0.1, 0.1, -0.1])
    np.testing.assert_allclose(O.saturate([0.0, 0.0, -2.0]), [0.0, 0.0, -0.3])


def test_collision_avoidance_cases():
    q = np.array([[0, 0, 1.0], [1.0, 0, 1.0], [10, 10, 1.0]])
    # heading straight at the obstacle (theta=0, alpha=asin(1)=pi/2): snap to an edge
    c, mod = O.collision_avoidance(0, q, [0.4, 0.0, 0.1])
    assert mod
    assert abs(np.hypot(c[0], c[1]) - 0.4) < 1e-12 and abs(abs(np.arctan2(c[1], c[0])) - np.pi / 2) < 1e-12
    # heading away: unmodified
    c, mod = O.collision_avoidance(0, q, [-0.4, 0.0, 0.1])
    assert not mod and np.allclose(c, [-0.4, 0, 0.1])
    # far obstacle only: no edges
    c, mod = O.collision_avoidance(2, q, [0.4, 0.4, 0.0])
    assert not mod
    # surrounded: four obstacles at 1 m -> no safe edge -> stop
    q2 = np.array([[0, 0, 1.0], [1, 0, 1], [-1, 0, 1], [0, 1, 1], [0, -1, 1.0]])
    c, mod = O.collision_avoidance(0, q2, [0.3, 0.1, 0.2])
    assert mod and np.all(c == 0)
    # obstacle behind across +-pi (wrap-around sector), heading into it
    q3 = np.array([[0, 0, 1.0], [-1.4, 0.01, 1.0]])
    c, mod = O.collision_avoidance(0, q3, [-0.3, -0.01, 0.0])
    assert mod
    # heading exactly pi lies on the split edge of the zones [-pi,.] and [.,pi]:
    # the reference's strict test calls it safe (safety.cpp:489)
    c, mod = O.collision_avoidance(0, q3, [-0.3, 0.0, 0.0])
    assert not mod


def test_oracle_batch_threads_match_serial():
    P, A = H.simform("simform20_nc")
    rng = np.random.RandomState(8)
    F = 4
    pts = np.stack([P[s, 0] for s in range(F)])
    adjs = np.stack([A[s] for s in range(F)])
    gains = np.stack([H.synth_gains(rng, a) for a in adjs])
    B = 12
    fidx = np.arange(B, dtype=np.int32) % F
    q = np.stack([H.random_positions(rng, 20, 20.0) for _ in range(B)])
    vel = rng.normal(0, 0.1, (B, 20, 3))
    Pin = np.stack([H.random_perm(rng, 20) for _ in range(B)])
    out, t = O.solve_batch(fidx, q, vel, pts, adjs, gains, Pin, nthreads=4)
    for b in range(B):
        r = O.solve(q[b], vel[b], pts[fidx[b]], adjs[fidx[b]], gains[fidx[b]], Pin[b])
        np.testing.assert_array_equal(out["P_out"][b], r["P_out"])
        np.testing.assert_array_equal(out["u_safe"][b], r["u_safe"])
        assert out["status"][b]["eff_rounds"] == r["status"]["eff_rounds"]


def test_umeyama_rule_switch_reaches_the_solve():
    """orc_set_umeyama_variant (the Eigen 3.3 / 3.4 umeyama rule, SURVEY
    App. B) applies to every vehicle alignment of the solve: the aligned
    (R, t) equal orc_umeyama2 under that rule, and on the reference
    generator's N = 100 formations both rules give the same assignments,
    flags and rounds (the rules differ only where det(sigma) and
    det(U) det(V) disagree in sign by rounding: the C3 count over the bench
    workload is scripts/eigen_variant_risk.py's)."""
    P, A = H.simform("simform100_nc")
    rng = np.random.RandomState(11)
    F = 3
    pts = np.stack([P[s, 0] for s in range(F)])
    adjs = np.stack([A[s] for s in range(F)])
    gains = np.stack([H.synth_gains(rng, a) for a in adjs])
    B = 6
    fidx = np.arange(B, dtype=np.int32) % F
    q = np.stack([H.random_positions(rng, 100, 45.0) for _ in range(B)])
    vel = rng.normal(0, 0.1, (B, 100, 3))
    Pin = np.stack([H.random_perm(rng, 100) for _ in range(B)])
    L = O.lib()
    outs = []
    try:
        for var in (0, 1):
            L.orc_set_umeyama_variant(var)
            assert L.orc_get_umeyama_variant() == var
            outs.append(O.solve_batch(fidx, q, vel, pts, adjs, gains, Pin, nthreads=4)[0])
            # one vehicle's alignment against the plain entry point
            b, v = 1, 17
            f = fidx[b]
            i = Pin[b][v]
            Pt = np.argsort(Pin[b])
            nb = [j for j in range(100) if adjs[f][i, j] or j == i]
            src = pts[f][nb, :2]
            dst = q[b][Pt[nb], :2]
            R, t = O.umeyama2(src, dst, var)
            Ra, ta = O.align(100, v, q[b], pts[f], adjs[f], Pin[b])
            np.testing.assert_array_equal(R, Ra)
            np.testing.assert_array_equal(t, ta)
    finally:
        L.orc_set_umeyama_variant(0)
    for k in ("P_out", "u_safe"):
        np.testing.assert_array_equal(outs[0][k], outs[1][k])
    np.testing.assert_array_equal(outs[0]["status"]["flags"], outs[1]["status"]["flags"])
    np.testing.assert_array_equal(outs[0]["status"]["eff_rounds"], outs[1]["status"]["eff_rounds"])
