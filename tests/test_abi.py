"""CPU suite: the C-ABI library loads, exports every declared symbol, its host
helpers are correct, and argument errors are reported without a GPU."""
import ctypes as ct
import os
import re

import numpy as np
import pytest

import helpers as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "aclswarm_amd.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(acl_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from aclswarm_amd import _lib as L
    lib = L.lib()
    syms = _declared_symbols()
    assert len(syms) >= 17
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(L.EXPORTS)


def test_defaults_match_reference_values():
    from aclswarm_amd import _lib as L
    g = L.default_gains()  # coordination.launch:32-39
    assert (g.K1_xy, g.K2_xy, g.K1_z, g.K2_z, g.e_xy_thr, g.e_z_thr, g.kp, g.kd) == \
        (0.1, 0.1, 0.5, 0.3, 0.3, 0.1, 1.5, 0.5)
    s = L.default_safety()  # safety.cpp:49-52
    assert (s.max_vel_xy, s.max_vel_z, s.d_avoid_thresh, s.r_keep_out) == (0.5, 0.3, 1.5, 1.2)
    a = L.default_admm_params()  # solver.h:18-31
    assert (a.thrSparseZero, a.thrPlanar, a.epsEig, a.mu, a.thresh, a.threshTr, a.maxItr) == \
        (1e-8, 1e-2, 1e-5, 1.0, 1e-4, 0.10, 10)
    assert a.basis == 0   # ACL_ADMM_BASIS_LINPACK: codegen parity by default
    assert ct.sizeof(L.AdmmParams) == 64  # basis sits in maxItr's old tail padding
    assert L.lib().acl_max_vehicles() == 512


def test_pack_adjacency_and_gains():
    from aclswarm_amd import engine
    pts, adj, gains, _ = H.swarm6()
    for f in range(3):
        A = adj[f].copy()
        A[2, 2] = 1  # a diagonal entry is an edge of the control law
        p, bits, planes, E = engine.pack_formation_host(pts[f], A, gains[f])
        n = 6
        assert E == int(A.sum())
        for i in range(n):
            for j in range(n):
                assert bool((int(bits[i, 0]) >> j) & 1) == bool(A[i, j])
        e = 0
        for i in range(n):
            for j in range(n):
                if A[i, j]:
                    blk = gains[f][3 * i:3 * i + 3, 3 * j:3 * j + 3]
                    np.testing.assert_array_equal(planes.reshape(9, E)[:, e], blk.reshape(9))
                    e += 1
    # n > 64: two words per row
    rng = np.random.RandomState(0)
    n = 100
    A = (rng.uniform(size=(n, n)) < 0.9).astype(np.uint8)
    _, bits, _, E = engine.pack_formation_host(np.zeros((n, 3)), A, None)
    assert bits.shape == (n, 2) and E == int(A.sum())
    for i in range(0, n, 7):
        row = [(int(bits[i, j // 64]) >> (j % 64)) & 1 for j in range(n)]
        assert row == list(A[i])


def test_solve_batch_argument_errors_without_gpu():
    from aclswarm_amd import _lib as L
    lib = L.lib()
    F = L.Formations(0, 1, None, None, None, None)
    a = L.SolveArgs()
    a.B = 1
    rc = lib.acl_solve_batch(ct.byref(F), ct.byref(a), None)
    assert rc == 1 and b"n out of range" in lib.acl_last_error()
    F.n = 513
    assert lib.acl_solve_batch(ct.byref(F), ct.byref(a), None) == 1
    F.n = 10
    assert lib.acl_solve_batch(ct.byref(F), ct.byref(a), None) == 1  # NULL pointers
    assert b"NULL" in lib.acl_last_error()
    a.B = 0
    assert lib.acl_solve_batch(ct.byref(F), ct.byref(a), None) == 0  # empty batch
    a.B = -1
    assert lib.acl_solve_batch(ct.byref(F), ct.byref(a), None) == 1
    assert lib.acl_solve_batch(None, ct.byref(a), None) == 1


def test_tile_gains_argument_errors_without_gpu():
    from aclswarm_amd import _lib as L
    lib = L.lib()
    out = ct.c_void_p(0x1000)  # never dereferenced: every call below fails its checks
    F = L.Formations(100, 1, None, None, None, None, 9)
    assert lib.acl_tile_gains(ct.byref(F), out, None) == 1
    assert b"gain_planes must be 5" in lib.acl_last_error()
    F.gain_planes = 5
    F.n = 129
    assert lib.acl_tile_gains(ct.byref(F), out, None) == 1
    assert b"n out of range" in lib.acl_last_error()
    F.n = 100
    assert lib.acl_tile_gains(ct.byref(F), out, None) == 1
    assert b"NULL" in lib.acl_last_error()
    F.n_formations = 0
    assert lib.acl_tile_gains(ct.byref(F), out, None) == 0  # nothing to do
    assert lib.acl_tile_gains(None, out, None) == 1
    assert lib.acl_tile_gains(ct.byref(F), None, None) == 1
    assert ct.sizeof(L.Formations) == 56  # gains_tiled appended after gain_planes


def test_status_record_is_16_bytes():
    from aclswarm_amd import _lib as L
    assert L.STATUS_DTYPE.itemsize == 16
    assert L.STATUS_DTYPE.fields["margin"][1] == 12  # f32 decision margin at byte 12


def test_abi_version_and_formations_init():
    """ABI 11 (ABI 5: gains_tiled in acl_formations_t, margin in the status,
    gate margins, the episode's auction latency and pending state; ABI 6:
    acl_admm_params_t.basis; ABI 7: acl_solve_args_t.skip_margin, appended;
    ABI 8: acl_solve_args_t.P_rows / P_rows_on, appended; ABI 9:
    acl_episode_params_t.assignment appended, the trial entry points; ABI 10:
    acl_solve_args_t.ws_persistent, appended; ABI 11: acl_cbaa_step_batch):
    acl_formations_init zero-fills the struct so no optional pointer
    is left as garbage; the solve rejects an empty formation table."""
    from aclswarm_amd import _lib as L
    with open(os.path.join(ROOT, "include", "aclswarm_amd.h")) as f:
        assert "#define ACL_ABI_VERSION 11" in f.read()
    lib = L.lib()
    assert lib.acl_abi_version() == 11 == L.ABI_VERSION  # the load-time check's inputs
    assert L.EpisodeParams.assignment.offset == L.EpisodeParams.avg_active_ca_thr.offset + 8
    assert L.SolveArgs.skip_margin.offset == L.SolveArgs.gate_margin.offset + 8
    assert L.SolveArgs.P_rows.offset == L.SolveArgs.skip_margin.offset + 8  # (4 B padding)
    assert L.SolveArgs.P_rows_on.offset == L.SolveArgs.P_rows.offset + 8
    assert L.SolveArgs.ws_persistent.offset == L.SolveArgs.P_rows_on.offset + 8
    F = L.Formations()
    ct.memset(ct.byref(F), 0xAB, ct.sizeof(F))
    lib.acl_formations_init(ct.byref(F), 100, 7)
    assert (F.n, F.n_formations, F.gain_planes) == (100, 7, 9)
    assert not F.p and not F.adj and not F.gains and not F.gain_off and not F.gains_tiled
    a = L.SolveArgs()
    a.B = 1
    a.fidx = a.q = a.P_in = a.P_out = a.status = a.workspace = 8  # never dereferenced
    F.p = F.adj = 8
    F.n_formations = 0
    assert lib.acl_solve_batch(ct.byref(F), ct.byref(a), None) == 1
    assert b"n_formations" in lib.acl_last_error()


def test_cpp_facade_compiles_and_exports():
    """include/aclswarm_amd.hpp (Auctioneer / DistCntrl / admm::Solver facade)
    compiles warning-free as C++17 and the built exerciser exports facade_run."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for src in ("facade_driver.cpp", "exchange_asan_main.cpp"):
        subprocess.check_call(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                               "-I" + os.path.join(root, "include"), os.path.join(root, "tests", src)])
    from aclswarm_amd import build
    so = build.build_driver()
    assert hasattr(ct.CDLL(so), "facade_run")


def test_gain_planes_detection_and_packing():
    """acl_gain_planes / acl_pack_gains_planes: the 5-entry record layout exists only
    for blocks with bit-exact +0.0 at (0,2), (1,2), (2,0), (2,1) (the ADMM
    assembly, solver.cpp:49-77); its per-edge records hold (0,0) (0,1) (1,0)
    (1,1) (2,2) of the 9-plane layout."""
    from aclswarm_amd import _lib as L
    from aclswarm_amd import engine
    lib = L.lib()
    rng = np.random.RandomState(3)
    n = 12
    A = (rng.rand(n, n) < 0.5).astype(np.uint8)
    np.fill_diagonal(A, 0)
    G = H.synth_gains(rng, A)
    pts = rng.rand(n, 3)
    assert engine.gain_planes_host(A, G) == 5
    _, _, g9, E = engine.pack_formation_host(pts, A, G, 9)
    _, _, g5, E5 = engine.pack_formation_host(pts, A, G, 5)
    assert E == E5 == int(A.sum())
    np.testing.assert_array_equal(g5.reshape(E, 5).T, g9.reshape(9, E)[[0, 1, 3, 4, 8]])
    # the real formations.yaml gains (ADMM outputs) have the structure
    _, adj6, gains6, _ = H.swarm6()
    assert all(engine.gain_planes_host(a, g) == 5 for a, g in zip(adj6, gains6))
    # a nonzero or a -0.0 in a structural-zero slot of an edge block -> 9
    i, j = map(int, np.argwhere(A)[0])
    for val in (1e-300, -0.0):
        G2 = G.copy()
        G2[3 * i + 2, 3 * j] = val
        assert engine.gain_planes_host(A, G2) == 9
        with pytest.raises(RuntimeError):
            engine.pack_formation_host(pts, A, G2, 5)
    # a non-edge block is never read
    k, l = map(int, np.argwhere(A == 0)[1])
    G3 = G.copy()
    G3[3 * k, 3 * l + 2] = 7.0
    assert engine.gain_planes_host(A, G3) == 5
    assert lib.acl_pack_gains_planes(n, None, None, 7, None) == 1


def test_codegen_entry_points_export_and_reject_bad_shapes_without_gpu():
    """include/aclswarm_amd_codegen.h: the generated library's ADMM entry
    points with their C++ names (the ones aclswarm/src/admm.cpp links), and a
    driver built against include/codegen_admm/ (-Werror); a malformed call
    (Qs 2 x n) leaves an empty result without touching the GPU."""
    from aclswarm_amd import _lib as L
    from aclswarm_amd import build
    lib = L.lib()
    build.build_driver()
    cg = ct.CDLL(build.CODEGEN_OUT)
    syms = ("_Z16ADMMGainDesign3DPK15emxArray_real_TS1_PS_",
            "_Z27ADMMGainDesign3D_initializev", "_Z26ADMMGainDesign3D_terminatev",
            "_Z14emxInit_real_TPP15emxArray_real_Ti", "_Z14emxFree_real_TPP15emxArray_real_T",
            "_Z23emxCreateWrapper_real_TPdii", "_Z22emxDestroyArray_real_TP15emxArray_real_T")
    for sym in syms:
        assert hasattr(cg, sym), sym
        # the generic Coder names stay out of the core library's exports
        assert not hasattr(lib, sym), sym
    drv = ct.CDLL(build.CG_DRIVER)
    assert drv.codegen_bad_call(5) == 0
    assert b"3 x n" in lib.acl_last_error()
