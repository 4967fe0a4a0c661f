"""ctypes binding of the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package `aclswarm_amd`.
"""
import ctypes as ct
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


class CntrlGains(ct.Structure):
    _fields_ = [(n, ct.c_double) for n in
                ("K1_xy", "K2_xy", "K1_z", "K2_z", "e_xy_thr", "e_z_thr", "kp", "kd")]


class SafetyParams(ct.Structure):
    _fields_ = [(n, ct.c_double) for n in
                ("max_vel_xy", "max_vel_z", "d_avoid_thresh", "r_keep_out")]


class SwarmStatus(ct.Structure):
    _fields_ = [("flags", ct.c_uint32), ("eff_rounds", ct.c_uint16),
                ("rounds", ct.c_uint16), ("n_invalid", ct.c_uint16),
                ("n_ca", ct.c_uint16), ("margin", ct.c_float)]


STATUS_DTYPE = np.dtype([("flags", "<u4"), ("eff_rounds", "<u2"),
                         ("rounds", "<u2"), ("n_invalid", "<u2"),
                         ("n_ca", "<u2"), ("margin", "<f4")])


def default_gains():
    # aclswarm/launch/coordination.launch:32-39
    return CntrlGains(0.1, 0.1, 0.5, 0.3, 0.3, 0.1, 1.5, 0.5)


def default_safety():
    # aclswarm/src/safety.cpp:49-52
    return SafetyParams(0.5, 0.3, 1.5, 1.2)


def _p(a, t):
    return a.ctypes.data_as(ct.POINTER(t))


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-C", _HERE, "liboracle.so"])
        L = ct.CDLL(path)
        D, F, U8, U16, I32 = (ct.POINTER(ct.c_double), ct.POINTER(ct.c_float),
                              ct.POINTER(ct.c_uint8), ct.POINTER(ct.c_uint16),
                              ct.POINTER(ct.c_int32))
        L.orc_jacobi_svd2.argtypes = [D, D, D, D]
        L.orc_jacobi_svd2.restype = ct.c_int
        L.orc_umeyama2.argtypes = [ct.c_int, D, D, D, D, ct.c_int]
        L.orc_umeyama2.restype = ct.c_int
        L.orc_align.argtypes = [ct.c_int, ct.c_int, D, D, U8, U16, D, D]
        L.orc_prices.argtypes = [ct.c_int, D, D, U8, U16, F, D]
        L.orc_prices_gap.argtypes = [ct.c_int, D, D, U8, U16, F, D, D]
        L.orc_umeyama2_gap.argtypes = [ct.c_int, D, D, D, D, ct.c_int, D]
        L.orc_umeyama2_gap.restype = ct.c_int
        L.orc_cbaa_m.argtypes = [ct.c_int, F, U8, U16, ct.c_int, I32, F, F]
        L.orc_cbaa_m.restype = ct.c_int
        L.orc_margin_gap.argtypes = [F]
        L.orc_margin_gap.restype = ct.c_double
        L.orc_cbaa.argtypes = [ct.c_int, F, U8, U16, ct.c_int, I32, F]
        L.orc_cbaa.restype = ct.c_int
        L.orc_pdist.argtypes = [ct.c_int, D, D, D]
        L.orc_control.argtypes = [ct.c_int, ct.c_int, D, D, U16, U8, D, D, D,
                                  ct.POINTER(CntrlGains), D]
        L.orc_saturate.argtypes = [ct.POINTER(SafetyParams), D]
        L.orc_collision_avoidance.argtypes = [ct.c_int, ct.c_int, D,
                                              ct.POINTER(SafetyParams), D]
        L.orc_collision_avoidance.restype = ct.c_int
        L.orc_solve.argtypes = [ct.c_int, D, D, D, U8, D, U16,
                                ct.POINTER(CntrlGains), ct.POINTER(SafetyParams),
                                ct.c_int, U16, ct.POINTER(SwarmStatus), D, D, U8, U16]
        L.orc_solve_g.argtypes = L.orc_solve.argtypes + [D]
        L.orc_solve_rows.argtypes = [ct.c_int, D, D, D, U8, D, U16, U16,
                                     ct.POINTER(CntrlGains), ct.POINTER(SafetyParams),
                                     ct.c_int, U16, ct.POINTER(SwarmStatus), D, D, U8, U16, D]
        L.orc_solve_batch.argtypes = [ct.c_int, ct.c_int, ct.c_int, I32, D, D, D,
                                      U8, D, U16, ct.POINTER(CntrlGains),
                                      ct.POINTER(SafetyParams), ct.c_int, U16,
                                      ct.c_void_p, D, D, U8, ct.c_int]
        L.orc_solve_batch.restype = ct.c_double
        L.orc_lsap.argtypes = [ct.c_int, D, I32]
        L.orc_lsap.restype = ct.c_int
        L.orc_arun2.argtypes = [ct.c_int, D, D, D]
        L.orc_hungarian.argtypes = [ct.c_int, D, D, U16, U16, U16, D, D]
        L.orc_hungarian.restype = ct.c_int
        _lib = L
    return _lib


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def jacobi_svd2(A):
    A = _c(np.asarray(A, dtype=np.float64).reshape(2, 2).T.copy(), np.float64)  # column-major
    U = np.zeros(4); V = np.zeros(4); s = np.zeros(2)
    rc = lib().orc_jacobi_svd2(_p(A, ct.c_double), _p(U, ct.c_double),
                               _p(s, ct.c_double), _p(V, ct.c_double))
    return rc, U.reshape(2, 2).T, s, V.reshape(2, 2).T


def umeyama2(src, dst, variant=0):
    """src, dst: [k][2]. Returns (R 2x2, t 2)."""
    src = _c(src, np.float64); dst = _c(dst, np.float64)
    R = np.zeros(4); t = np.zeros(2)
    lib().orc_umeyama2(src.shape[0], _p(src, ct.c_double), _p(dst, ct.c_double),
                       _p(R, ct.c_double), _p(t, ct.c_double), variant)
    return R.reshape(2, 2), t


def align(n, v, q, p, adj, P):
    """orc_align: vehicle v's alignment (auctioneer.cpp:347-415) under the
    current umeyama rule. Returns (R 2x2, t 2)."""
    q = _c(q, np.float64); p = _c(p, np.float64); adj = _c(adj, np.uint8)
    P = _c(P, np.uint16)
    R = np.zeros(4); t = np.zeros(2)
    lib().orc_align(n, v, _p(q, ct.c_double), _p(p, ct.c_double), _p(adj, ct.c_uint8),
                    _p(P, ct.c_uint16), _p(R, ct.c_double), _p(t, ct.c_double))
    return R.reshape(2, 2), t


def prices(q, p, adj, P):
    n = q.shape[0]
    q = _c(q, np.float64); p = _c(p, np.float64); adj = _c(adj, np.uint8)
    P = _c(P, np.uint16)
    C = np.zeros((n, n), np.float32); Rt = np.zeros((n, 6))
    lib().orc_prices(n, _p(q, ct.c_double), _p(p, ct.c_double), _p(adj, ct.c_uint8),
                     _p(P, ct.c_uint16), _p(C, ct.c_float), _p(Rt, ct.c_double))
    return C, Rt


def prices_gap(q, p, adj, P):
    """orc_prices plus the smallest alignment decision gap (det sign / rank
    tests) over the vehicles."""
    n = q.shape[0]
    q = _c(q, np.float64); p = _c(p, np.float64); adj = _c(adj, np.uint8)
    P = _c(P, np.uint16)
    C = np.zeros((n, n), np.float32); Rt = np.zeros((n, 6)); g = np.zeros(1)
    lib().orc_prices_gap(n, _p(q, ct.c_double), _p(p, ct.c_double), _p(adj, ct.c_uint8),
                         _p(P, ct.c_uint16), _p(C, ct.c_float), _p(Rt, ct.c_double),
                         _p(g, ct.c_double))
    return C, Rt, float(g[0])


def umeyama2_gap(src, dst):
    src = _c(src, np.float64); dst = _c(dst, np.float64)
    R = np.zeros(4); t = np.zeros(2); g = np.zeros(1)
    lib().orc_umeyama2_gap(src.shape[0], _p(src, ct.c_double), _p(dst, ct.c_double),
                           _p(R, ct.c_double), _p(t, ct.c_double), 0, _p(g, ct.c_double))
    return R.reshape(2, 2), t, float(g[0])


def cbaa_margin(C, adj, P, early_exit=True):
    """orc_cbaa_m: (who, price, eff, gap) with gap the f64 decision gap of the
    CBAA comparisons (include/aclswarm_amd.h, margin)."""
    n = C.shape[0]
    C = _c(C, np.float32); adj = _c(adj, np.uint8); P = _c(P, np.uint16)
    who = np.zeros((n, n), np.int32); pr = np.zeros((n, n), np.float32)
    m = np.zeros(2, np.float32)
    eff = lib().orc_cbaa_m(n, _p(C, ct.c_float), _p(adj, ct.c_uint8), _p(P, ct.c_uint16),
                           int(early_exit), _p(who, ct.c_int32), _p(pr, ct.c_float),
                           _p(m, ct.c_float))
    return who, pr, eff, float(lib().orc_margin_gap(_p(m, ct.c_float)))


def cbaa(C, adj, P, early_exit=True):
    n = C.shape[0]
    C = _c(C, np.float32); adj = _c(adj, np.uint8); P = _c(P, np.uint16)
    who = np.zeros((n, n), np.int32); pr = np.zeros((n, n), np.float32)
    eff = lib().orc_cbaa(n, _p(C, ct.c_float), _p(adj, ct.c_uint8), _p(P, ct.c_uint16),
                         int(early_exit), _p(who, ct.c_int32), _p(pr, ct.c_float))
    return who, pr, eff


def pdist(p):
    n = p.shape[0]
    p = _c(p, np.float64)
    dxy = np.zeros((n, n)); dz = np.zeros((n, n))
    lib().orc_pdist(n, _p(p, ct.c_double), _p(dxy, ct.c_double), _p(dz, ct.c_double))
    return dxy, dz


def control(v, q, vel_v, Pt, adj, gains, p, g=None):
    n = q.shape[0]
    g = g or default_gains()
    dxy, dz = pdist(p)
    q = _c(q, np.float64); vel_v = _c(vel_v, np.float64); Pt = _c(Pt, np.uint16)
    adj = _c(adj, np.uint8); gains = _c(gains, np.float64)
    u = np.zeros(3)
    lib().orc_control(n, v, _p(q, ct.c_double), _p(vel_v, ct.c_double),
                      _p(Pt, ct.c_uint16), _p(adj, ct.c_uint8), _p(gains, ct.c_double),
                      _p(dxy, ct.c_double), _p(dz, ct.c_double), ct.byref(g),
                      _p(u, ct.c_double))
    return u


def saturate(cmd, s=None):
    s = s or default_safety()
    c = _c(cmd, np.float64).copy()
    lib().orc_saturate(ct.byref(s), _p(c, ct.c_double))
    return c


def collision_avoidance(v, q, cmd, s=None):
    s = s or default_safety()
    q = _c(q, np.float64)
    c = _c(cmd, np.float64).copy()
    mod = lib().orc_collision_avoidance(q.shape[0], v, _p(q, ct.c_double),
                                        ct.byref(s), _p(c, ct.c_double))
    return c, bool(mod)


def solve(q, vel, p, adj, gains, P_in, g=None, s=None, early_exit=True, P_rows=None):
    """One swarm. gains dense [3n][3n] row-major. P_rows (optional [n][n]):
    row v = vehicle v's own assignment as formation point -> vehicle
    (orc_solve_rows; acl_solve_args_t::P_rows)."""
    n = q.shape[0]
    g = g or default_gains(); s = s or default_safety()
    q = _c(q, np.float64); vel = _c(vel, np.float64); p = _c(p, np.float64)
    adj = _c(adj, np.uint8); gains = _c(gains, np.float64); P_in = _c(P_in, np.uint16)
    P_out = np.zeros(n, np.uint16); st = SwarmStatus()
    u = np.zeros((n, 3)); us = np.zeros((n, 3)); ca = np.zeros(n, np.uint8)
    who = np.zeros((n, n), np.uint16)
    gm = np.zeros(1)
    rows = None if P_rows is None else _c(P_rows, np.uint16)
    lib().orc_solve_rows(n, _p(q, ct.c_double), _p(vel, ct.c_double), _p(p, ct.c_double),
                         _p(adj, ct.c_uint8), _p(gains, ct.c_double), _p(P_in, ct.c_uint16),
                         None if rows is None else _p(rows, ct.c_uint16),
                         ct.byref(g), ct.byref(s), int(early_exit), _p(P_out, ct.c_uint16),
                         ct.byref(st), _p(u, ct.c_double), _p(us, ct.c_double),
                         _p(ca, ct.c_uint8), _p(who, ct.c_uint16), _p(gm, ct.c_double))
    status = {k: getattr(st, k) for k, _ in SwarmStatus._fields_}
    return dict(P_out=P_out, status=status, u=u, u_safe=us, ca=ca, who=who,
                gate_margin=float(gm[0]))


def solve_batch(fidx, q, vel, p, adj, gains, P_in, nthreads=1, g=None, s=None,
                early_exit=True, margin=True):
    """B swarms; p [F][n][3], adj [F][n][n], gains [F][3n][3n]. Returns outputs and
    the wall time (s). margin=False skips the decision-margin bookkeeping
    (the CPU baseline times the reference's work only)."""
    B, n = q.shape[0], q.shape[1]
    g = g or default_gains(); s = s or default_safety()
    fidx = _c(fidx, np.int32); q = _c(q, np.float64); vel = _c(vel, np.float64)
    p = _c(p, np.float64); adj = _c(adj, np.uint8); gains = _c(gains, np.float64)
    P_in = _c(P_in, np.uint16)
    P_out = np.zeros((B, n), np.uint16); st = np.zeros(B, STATUS_DTYPE)
    u = np.zeros((B, n, 3)); us = np.zeros((B, n, 3)); ca = np.zeros((B, n), np.uint8)
    t = lib().orc_solve_batch(B, n, nthreads, _p(fidx, ct.c_int32), _p(q, ct.c_double),
                              _p(vel, ct.c_double), _p(p, ct.c_double), _p(adj, ct.c_uint8),
                              _p(gains, ct.c_double), _p(P_in, ct.c_uint16), ct.byref(g),
                              ct.byref(s), int(early_exit), _p(P_out, ct.c_uint16),
                              st.ctypes.data_as(ct.c_void_p), _p(u, ct.c_double),
                              _p(us, ct.c_double), _p(ca, ct.c_uint8), int(bool(margin)))
    return dict(P_out=P_out, status=st, u=u, u_safe=us, ca=ca), t


def lsap(C):
    """orc_lsap: SciPy's linear_sum_assignment restated (square, minimise).
    Returns col4row (int32) or None when SciPy would raise."""
    C = _c(C, np.float64)
    n = C.shape[0]
    out = np.empty(n, np.int32)
    rc = lib().orc_lsap(n, _p(C, ct.c_double), _p(out, ct.c_int32))
    return None if rc else out


def hungarian(q, p, P_last=None, P_cmp=None):
    """orc_hungarian: assignment.py:94-137 for one swarm. q, p [n][3].
    Returns (P_opt u16, cost[2], Rt[4], status)."""
    q = _c(q, np.float64); p = _c(p, np.float64)
    n = q.shape[0]
    Pl = None if P_last is None else _c(P_last, np.uint16)
    Pc = None if P_cmp is None else _c(P_cmp, np.uint16)
    P = np.empty(n, np.uint16)
    cost = np.empty(2, np.float64)
    Rt = np.full(4, np.nan)
    st = lib().orc_hungarian(n, _p(q, ct.c_double), _p(p, ct.c_double),
                             None if Pl is None else _p(Pl, ct.c_uint16),
                             None if Pc is None else _p(Pc, ct.c_uint16),
                             _p(P, ct.c_uint16), _p(cost, ct.c_double), _p(Rt, ct.c_double))
    return P, cost, Rt, st
