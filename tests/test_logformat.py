"""Auctioneer::logAssignment records: the writer in the C
ABI produces the reference's byte layout (aclswarm/src/auctioneer.cpp:577-597)
and the reader inverts it. The layout is checked against an independent
Python decoder written from the reference's MATLAB reader
(aclswarm/matlab/Helpers/read_alignment.m:1-19: u8 n, then column-major
[n,3] f64 q, [n,n] u8 adjmat, [1,n] u8 lastP, [n,3] f64 p, [n,3] f64 aligned,
[1,n] u8 P)."""
import numpy as np

import helpers as H


def _decode_like_read_alignment(buf):
    o = 0
    n = buf[0]
    o += 1

    def take(count, dt):
        nonlocal o
        a = np.frombuffer(buf, dtype=dt, count=count, offset=o)
        o += a.nbytes
        return a

    q = take(3 * n, "<f8").reshape(3, n).T            # fread(..., [n, 3]) column-major
    adj = take(n * n, "u1").reshape(n, n).T
    s1 = take(n, "u1")
    p = take(3 * n, "<f8").reshape(3, n).T
    al = take(3 * n, "<f8").reshape(3, n).T
    s2 = take(n, "u1")
    assert o == len(buf)
    return n, q, adj, s1, p, al, s2


def test_record_layout_and_round_trip(tmp_path):
    from aclswarm_amd import engine
    pts, adj, _, q0 = H.swarm6()
    rng = np.random.RandomState(4)
    n = 6
    lastP = rng.permutation(n).astype(np.uint16)
    P = rng.permutation(n).astype(np.uint16)
    th = 0.3
    Rt = np.array([np.cos(th), -np.sin(th), np.sin(th), np.cos(th), 0.5, -1.25])
    f = tmp_path / "veh0_assignment1.bin"
    engine.write_assignment_log(f, q0, adj[1], lastP, pts[1], Rt, P)
    buf = f.read_bytes()
    assert len(buf) == 1 + 3 * 8 * n * 3 + n * n + 2 * n
    m, q, A, s1, p, al, s2 = _decode_like_read_alignment(buf)
    assert m == n
    np.testing.assert_array_equal(q, q0)
    np.testing.assert_array_equal(A, adj[1])
    np.testing.assert_array_equal(s1, lastP)
    np.testing.assert_array_equal(p, pts[1])
    np.testing.assert_array_equal(s2, P)
    # aligned = R p + t with the z row identity (alignFormation's expression)
    R = Rt[:4].reshape(2, 2)
    exp = np.c_[pts[1][:, :2] @ R.T + Rt[4:], pts[1][:, 2]]
    np.testing.assert_allclose(al, exp, rtol=0, atol=1e-15)
    r = engine.read_assignment_log(f)
    np.testing.assert_array_equal(r["q"], q0)
    np.testing.assert_array_equal(r["adj"], adj[1])
    np.testing.assert_array_equal(r["lastP"], lastP)
    np.testing.assert_array_equal(r["P"], P)
    np.testing.assert_array_equal(r["aligned"], al)


def test_record_rejects_n_above_u8(tmp_path):
    import ctypes as ct
    from aclswarm_amd import _lib as L
    lib = L.lib()
    z = np.zeros(3 * 300)
    assert lib.acl_write_assignment_log(str(tmp_path / "x.bin").encode(), 300, z.ctypes.data,
                                        z.ctypes.data, z.ctypes.data, z.ctypes.data,
                                        z.ctypes.data, z.ctypes.data) != 0
    n = ct.c_int32(0)
    assert lib.acl_read_assignment_log(str(tmp_path / "missing.bin").encode(), ct.byref(n),
                                       None, None, None, None, None, None) != 0
