"""The C++ facade (include/aclswarm_amd.hpp) driven the way the reference's
CoordinationROS drives its objects: one Auctioneer and one DistCntrl per
vehicle, one admm::Solver (tests/facade_driver.cpp, built into
aclswarm_amd/lib/libfacade_driver.so and loaded here by ctypes).

Checked against the CPU restatement: each vehicle adopts its own final CBAA
table exactly as auctioneer.cpp:250-295 does (bit-exact), DistCntrl::compute
within 1e-5 relative, and the ADMM gains of test_admm.cpp's cases within the
reference test's own tolerance.
"""
import ctypes as ct
import os

import numpy as np
import pytest

import helpers as H
import pyoracle as O

pytestmark = pytest.mark.gpu

U_RTOL = 1e-5  # north_star: control commands within 1e-5 relative (fp64)
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "aclswarm_amd", "lib", "libfacade_driver.so")


def _run(tmp_path, p, adj, gains, q, vel, P_in, pts=None, adjf=None):
    n = p.shape[0]
    m = 0 if pts is None else pts.shape[0]
    fin, fout = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    with open(fin, "wb") as f:
        f.write(np.int32(n).tobytes())
        f.write(np.asfortranarray(p, np.float64).tobytes(order="F"))
        f.write(np.asarray(adj, np.uint8).tobytes(order="F"))
        f.write(np.asarray(gains, np.float64).tobytes(order="F"))
        f.write(np.asarray(q, np.float64).tobytes(order="F"))
        f.write(np.ascontiguousarray(vel, np.float64).tobytes())
        f.write(np.asarray(P_in, np.uint8).tobytes())
        f.write(np.int32(m).tobytes())
        if m:
            f.write(np.ascontiguousarray(pts, np.float64).tobytes())  # 3 x m column-major
            f.write(np.asarray(adjf, np.float64).tobytes(order="F"))
    if not os.path.exists(LIB):
        raise RuntimeError(f"{LIB} missing: run python -m aclswarm_amd.build")
    lib = ct.CDLL(LIB)
    lib.facade_run.argtypes = [ct.c_char_p, ct.c_char_p]
    assert lib.facade_run(fin.encode(), fout.encode()) == 0
    raw = open(fout, "rb").read()
    o = 0
    P, inv, calls = [], [], []
    for _ in range(n):
        P.append(np.frombuffer(raw, np.uint8, n, o)); o += n
        inv.append(raw[o]); calls.append(raw[o + 1]); o += 2
    bid_calls, bid_iter, bid_who, bid_price = [], [], [], []
    for _ in range(n):
        bid_calls.append(raw[o]); o += 1
        bid_iter.append(int(np.frombuffer(raw, np.uint32, 1, o)[0])); o += 4
        bid_who.append(np.frombuffer(raw, np.int32, n, o)); o += 4 * n
        bid_price.append(np.frombuffer(raw, np.float32, n, o)); o += 4 * n
    start_errors_ok = raw[o]; o += 1
    u = np.frombuffer(raw, np.float64, 3 * n, o).reshape(n, 3); o += 24 * n
    its = np.frombuffer(raw, np.int32, 2, o); o += 8
    A = np.frombuffer(raw, np.float64, 9 * m * m, o).reshape(3 * m, 3 * m, order="F")
    return dict(P=np.array(P), invalid=np.array(inv), calls=np.array(calls), u=u,
                iters=its, A=A, bid_calls=np.array(bid_calls), bid_iter=np.array(bid_iter),
                bid_who=np.array(bid_who), bid_price=np.array(bid_price),
                start_errors_ok=start_errors_ok)


def _expect(p, adj, gains, q, vel, P_in):
    """Per vehicle: its final table (oracle), adopted as auctioneer.cpp:250-295
    does after setFormation (adopt when valid, flag when not)."""
    n = p.shape[0]
    r = O.solve(q, np.zeros_like(q), p, adj, gains, np.asarray(P_in, np.uint16))
    P, inv = [], []
    for v in range(n):
        who = r["who"][v].astype(np.int64)
        if np.array_equal(np.sort(who), np.arange(n)):
            Pv = np.empty(n, np.int64); Pv[who] = np.arange(n)
            P.append(Pv); inv.append(0)
        else:
            P.append(np.arange(n)); inv.append(1)   # setFormation reset P to identity
    u = np.stack([O.control(v, q, vel[v], np.argsort(P[v]).astype(np.uint16), adj, gains, p)
                  for v in range(n)])
    return np.array(P), np.array(inv), u


def _check(got, p, adj, gains, q, vel, P_in):
    P, inv, u = _expect(p, adj, gains, q, vel, P_in)
    np.testing.assert_array_equal(got["invalid"], inv)
    np.testing.assert_array_equal(got["calls"], 1 - inv)
    # the send-bid handler: once per vehicle per auction, iter = 2n, the bid
    # equal to the oracle's final bid table row (who and price, bit for bit)
    n = p.shape[0]
    C, _ = O.prices(q, p, adj, np.asarray(P_in, np.uint16))
    who, pr, _ = O.cbaa(C, adj, np.asarray(P_in, np.uint16))
    np.testing.assert_array_equal(got["bid_calls"], np.ones(n))
    np.testing.assert_array_equal(got["bid_iter"], np.full(n, 2 * n))
    np.testing.assert_array_equal(got["bid_who"], who)
    np.testing.assert_array_equal(got["bid_price"].view(np.uint32), pr.view(np.uint32))
    assert got["start_errors_ok"] == 1
    for v in range(p.shape[0]):
        if not inv[v]:
            np.testing.assert_array_equal(got["P"][v], P[v], err_msg=f"vehicle {v}")
    err = np.abs(got["u"] - u) / np.maximum(np.abs(u), 1.0)
    assert err.max() <= U_RTOL, err.max()


def test_facade_swarm6_and_test_admm(tmp_path):
    """formations.yaml swarm6_3d with its given gains from a perturbed
    start.sh grid, plus admm::Solver on test_admm.cpp's first case."""
    pts, adj, gains, q0 = H.swarm6()
    rng = np.random.RandomState(61)
    q = q0 + rng.normal(0, 0.3, q0.shape)
    vel = rng.normal(0, 0.1, q.shape)
    P_in = H.random_perm(rng, 6)
    d = H.load_json("admm_test_admm.json")
    c = d["cases"][0]
    pa = np.array(c["p"], np.float64)
    got = _run(tmp_path, pts[1], adj[1], gains[1], q, vel, P_in,
               pts=pa, adjf=np.array(c["adj"], np.float64))
    _check(got, pts[1], adj[1], gains[1], q, vel, P_in)
    assert np.linalg.norm(got["A"] - np.array(c["A"])) < d["tol"]
    assert (got["iters"] > 0).all()


@pytest.mark.parametrize("name", ["simform20_fc", "simform20_nc"])
def test_facade_simform20(tmp_path, name):
    """n = 20 generator formations with synthetic gains, random P_in."""
    Pf, Af = H.simform(name)
    rng = np.random.RandomState(7)
    p, adj = Pf[1, 0], Af[1]
    gains = H.synth_gains(rng, adj)
    q = H.random_positions(rng, 20, 20.0)
    vel = rng.normal(0, 0.2, q.shape)
    P_in = H.random_perm(rng, 20)
    got = _run(tmp_path, p, adj, gains, q, vel, P_in)
    _check(got, p, adj, gains, q, vel, P_in)


def test_facade_admm_solver_nine_agent(tmp_path):
    """The facade's admm::Solver (basis ACL_ADMM_BASIS_COMPLEX by default)
    passes aclswarm/test/test_admm.cpp:84-187 on that test's own nine-agent
    formation: zero non-edge blocks and [a b 0; -b a 0; 0 0 c] blocks at the
    test's 1e-8."""
    from test_admm import nine_agent_violations
    pts, adj, gains, q0 = H.swarm6()
    rng = np.random.RandomState(62)
    q = q0 + rng.normal(0, 0.3, q0.shape)
    vel = rng.normal(0, 0.1, q.shape)
    P_in = H.random_perm(rng, 6)
    d = H.load_json("admm_nine_agent.json")
    adj9 = np.array(d["adj"], np.float64)
    got = _run(tmp_path, pts[1], adj[1], gains[1], q, vel, P_in,
               pts=np.array(d["p"], np.float64), adjf=adj9)
    zs, worst = nine_agent_violations(got["A"], adj9)
    assert abs(zs) < d["tol"] and worst < d["tol"], (zs, worst)
    assert (got["iters"] > 0).all()


def test_facade_admm_wrapper_class_codegen():
    """The reference's ADMM wrapper (aclswarm/src/admm.cpp:34-55,
    include/aclswarm/admm.h:27-40) through the facade's ADMM class: codegen
    semantics, so the reference's own codegen outputs (tests/golden,
    admm_golden.npz) within 1e-5 relative and the MATLAB 12 x 12 matrices of
    test_admm.cpp:10-80 within 1e-8."""
    import admm_cases as AC
    lib = ct.CDLL(LIB)
    lib.facade_admm_codegen.argtypes = [ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_void_p]

    def run(p, adj):
        n = p.shape[0]
        P = np.asfortranarray(p, np.float64)
        A8 = np.asfortranarray(np.asarray(adj) != 0, np.uint8)
        out = np.zeros((3 * n, 3 * n), np.float64, order="F")
        assert lib.facade_admm_codegen(n, P.ctypes.data, A8.ctypes.data, out.ctypes.data) == 0
        return out
    d = H.load_json("admm_test_admm.json")
    for c in d["cases"]:
        A = run(np.array(c["p"]), np.array(c["adj"]))
        assert np.linalg.norm(A - np.array(c["A"])) < d["tol"]
    for c in [c for c in AC.load() if c["p"].shape[0] <= 20][:4]:
        A = run(c["p"], c["adj"])
        assert AC.rel_err(A, AC.assemble(c["Axy"], c["Az"])) < 1e-5, c["name"]


def _exchange(p, adj, q, P_in, seed, late):
    n = p.shape[0]
    lib = ct.CDLL(LIB)
    f = lib.facade_exchange
    f.restype = ct.c_int
    P = np.zeros((n, n), np.uint8)
    inv = np.zeros(n, np.uint8)
    sends, handler, last_iter = (np.zeros(n, np.int32) for _ in range(3))
    who = np.zeros((n, n), np.int32)
    pc = np.asfortranarray(p, np.float64)
    qc = np.asfortranarray(q, np.float64)
    ac = np.asfortranarray(np.asarray(adj, np.uint8))
    Pi = np.ascontiguousarray(P_in, np.uint8)
    ptr = lambda a: a.ctypes.data_as(ct.c_void_p)  # noqa: E731
    f.argtypes = [ct.c_int] + [ct.c_void_p] * 4 + [ct.c_uint32, ct.c_int] + [ct.c_void_p] * 6
    assert f(n, ptr(pc), ptr(ac), ptr(qc), ptr(Pi), seed, late, ptr(P), ptr(inv), ptr(sends),
             ptr(handler), ptr(last_iter), ptr(who)) == 0
    return dict(P=P, invalid=inv, sends=sends, handler=handler, last_iter=last_iter, who=who)


@pytest.mark.parametrize("case,seed,late", [("swarm6", 1, 0), ("swarm6", 2, 3),
                                            ("simform20_nc", 3, 0), ("simform20_nc", 4, 7),
                                            ("simform20_fc", 5, 19)])
def test_facade_bid_exchange(case, seed, late):
    """Exchange mode (Auctioneer::setBidExchange, ABI 11): every vehicle runs
    the reference's message protocol -- START bid, enqueueBid / tick /
    processBid with iteration buckets, its tallies on the GPU
    (acl_cbaa_step_batch) -- over a bus that delivers bids in a seeded random
    order, some vehicles starting late (their neighbours' START bids wait in
    their queues). Each vehicle adopts the same assignment as the one-call
    consensus (the oracle's tables, adopted as auctioneer.cpp:250-295 does),
    sends 2n bids (iterations 0 .. 2n - 1), and its last bid equals the
    lockstep protocol's table after 2n - 1 iterations (the CPU restatement)."""
    import cbaa_step_oracle as S
    rng = np.random.RandomState(seed)
    if case == "swarm6":
        pts, adjs, gains, q0 = H.swarm6()
        p, adj, g = pts[1], adjs[1], gains[1]
        q = q0 + rng.normal(0, 0.3, q0.shape)
    else:
        Pf, Af = H.simform(case)
        p, adj = Pf[seed % Pf.shape[0], 0], Af[seed % Af.shape[0]]
        g = H.synth_gains(rng, adj)
        q = H.random_positions(rng, p.shape[0], 20.0)
    n = p.shape[0]
    P_in = H.random_perm(rng, n)
    got = _exchange(p, adj, q, P_in, seed, late)
    P, inv, _ = _expect(p, adj, g, q, np.zeros_like(q), P_in)
    np.testing.assert_array_equal(got["invalid"], inv)
    np.testing.assert_array_equal(got["handler"], 1 - inv)
    for v in range(n):
        if not inv[v]:
            np.testing.assert_array_equal(got["P"][v], P[v], err_msg=f"vehicle {v}")
    np.testing.assert_array_equal(got["sends"], np.full(n, 2 * n))
    np.testing.assert_array_equal(got["last_iter"], np.full(n, 2 * n - 1))
    C, _ = O.prices(q, p, adj, np.asarray(P_in, np.uint16))
    who, _ = S.lockstep(C, adj, P_in, rounds=2 * n - 1)
    np.testing.assert_array_equal(got["who"], who)


@pytest.mark.parametrize("case,seed,mask", [("swarm6", 11, "alternate"), ("swarm6", 12, "one"),
                                            ("simform20_nc", 13, "alternate"),
                                            ("simform20_fc", 14, "half")])
def test_facade_mixed_fleet(case, seed, mask):
    """A mixed fleet (some vehicles on the reference's own
    Auctioneer): exchange-mode facades (GPU tallies) and CPU stand-ins of the
    reference's protocol (tests/facade_driver.cpp RefVehicle, its prices from
    the CPU oracle) on one bus. Every vehicle, of either kind, adopts the
    one-call consensus's assignment and sends 2n bids; the last bids equal
    the lockstep protocol's tables after 2n - 1 iterations."""
    import cbaa_step_oracle as S
    rng = np.random.RandomState(seed)
    if case == "swarm6":
        pts, adjs, gains, q0 = H.swarm6()
        p, adj, g = pts[1], adjs[1], gains[1]
        q = q0 + rng.normal(0, 0.3, q0.shape)
    else:
        Pf, Af = H.simform(case)
        p, adj = Pf[seed % Pf.shape[0], 0], Af[seed % Af.shape[0]]
        g = H.synth_gains(rng, adj)
        q = H.random_positions(rng, p.shape[0], 20.0)
    n = p.shape[0]
    P_in = H.random_perm(rng, n)
    fm = {"alternate": np.arange(n) % 2 == 0, "one": np.arange(n) == 3,
          "half": np.arange(n) < n // 2}[mask].astype(np.uint8)
    C, _ = O.prices(q, p, adj, np.asarray(P_in, np.uint16))
    lib = ct.CDLL(LIB)
    f = lib.facade_mixed
    f.restype = ct.c_int
    f.argtypes = [ct.c_int] + [ct.c_void_p] * 6 + [ct.c_uint32] + [ct.c_void_p] * 5
    Pout = np.zeros((n, n), np.uint8)
    inv = np.zeros(n, np.uint8)
    sends, last_iter = np.zeros(n, np.int32), np.zeros(n, np.int32)
    who = np.zeros((n, n), np.int32)
    arrs = [np.asfortranarray(p, np.float64), np.asfortranarray(np.asarray(adj, np.uint8)),
            np.asfortranarray(q, np.float64), np.ascontiguousarray(P_in, np.uint8),
            np.ascontiguousarray(C, np.float32), fm]
    ptr = lambda a: a.ctypes.data_as(ct.c_void_p)  # noqa: E731
    assert f(n, *[ptr(a) for a in arrs], seed, ptr(Pout), ptr(inv), ptr(sends), ptr(last_iter),
             ptr(who)) == 0
    P, inv_e, _ = _expect(p, adj, g, q, np.zeros_like(q), P_in)
    np.testing.assert_array_equal(inv, inv_e)
    for v in range(n):
        if not inv_e[v]:
            np.testing.assert_array_equal(Pout[v], P[v], err_msg=f"vehicle {v} ({mask})")
    np.testing.assert_array_equal(sends, np.full(n, 2 * n))
    np.testing.assert_array_equal(last_iter, np.full(n, 2 * n - 1))
    who_l, _ = S.lockstep(C, adj, P_in, rounds=2 * n - 1)
    np.testing.assert_array_equal(who, who_l)
