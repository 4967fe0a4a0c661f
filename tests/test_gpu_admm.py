"""GPU parity of the batched ADMM gain design (SURVEY.md rows a15-a19, config
C5) through the C ABI (acl_admm_solve_batch).

Bar (BASELINE.json north_star): ADMM gains within 1e-5 relative (fp64) of
the reference. The golden gains are the reference's own codegen ADMM outputs
(tests/golden/admm_golden.npz, made by tests/golden/make_admm_fixtures.py);
iteration counts must equal the CPU restatement's (oracle/admm_oracle.py).
"""
import numpy as np
import pytest

import admm_cases as AC
import admm_oracle as O
import helpers as H

pytestmark = pytest.mark.gpu

REL_TOL = 1e-5  # north_star: ADMM gains within 1e-5 relative (fp64)
CASES = AC.load()


def _gpu(ps, adjs, basis=None):
    import torch
    from aclswarm_amd import engine
    dev = torch.device("cuda:0")
    pts = torch.from_numpy(np.ascontiguousarray(np.stack(ps), dtype=np.float64)).to(dev)
    adj = torch.from_numpy(np.ascontiguousarray(np.stack(adjs), dtype=np.float64)).to(dev)
    A, its = engine.admm_design(pts, adj, basis=basis)
    torch.cuda.synchronize()
    return A.cpu().numpy(), its.cpu().numpy()


@pytest.mark.parametrize("n", sorted({c["p"].shape[0] for c in CASES}))
def test_admm_matches_reference_golden(n):
    """All golden formations of one size in one batched call."""
    cs = [c for c in CASES if c["p"].shape[0] == n]
    A, its = _gpu([c["p"] for c in cs], [c["adj"].astype(np.float64) for c in cs])
    for k, c in enumerate(cs):
        ref = AC.assemble(c["Axy"], c["Az"])
        err = AC.rel_err(A[k], ref)
        assert err < REL_TOL, (c["name"], err)
        assert (its[k] > 0).all(), (c["name"], its[k])


@pytest.mark.parametrize("n", [3, 5, 6, 9, 20])
def test_admm_iterations_match_oracle(n):
    cs = [c for c in CASES if c["p"].shape[0] == n]
    if not cs:
        pytest.skip("no fixture of this size")
    A, its = _gpu([c["p"] for c in cs], [c["adj"].astype(np.float64) for c in cs])
    for k, c in enumerate(cs):
        Ao, ito = O.design_3d(c["p"], c["adj"])
        assert tuple(int(x) for x in its[k]) == tuple(ito), (c["name"], its[k], ito)
        assert AC.rel_err(A[k], Ao) < REL_TOL


def test_admm_test_admm_goldens():
    """aclswarm/test/test_admm.cpp:10-80: the two MATLAB 12 x 12 matrices."""
    d = H.load_json("admm_test_admm.json")
    A, _ = _gpu([np.array(c["p"]) for c in d["cases"]],
                [np.array(c["adj"], dtype=np.float64) for c in d["cases"]])
    for k, c in enumerate(d["cases"]):
        assert np.linalg.norm(A[k] - np.array(c["A"])) < d["tol"]


def test_admm_complex_basis_nine_agent():
    """ACL_ADMM_BASIS_COMPLEX (acl_admm_params_t.basis = 1): the nine-agent
    formation of aclswarm/test/test_admm.cpp:84-187 meets both of that test's
    assertions at 1e-8 (zero non-edge blocks, [a b 0; -b a 0; 0 0 c] blocks),
    the MATLAB 12 x 12 matrices (:10-80) still match, and every result equals
    the oracle's complex-basis design (1e-5 relative, same iteration counts)
    on a batch mixing the fixture sizes. The default basis is covered by the
    codegen-parity tests above; its nine-agent violation is recorded in
    tests/test_admm.py::test_nine_agent_codegen_basis_recorded."""
    from test_admm import nine_agent_violations
    d = H.load_json("admm_nine_agent.json")
    g = H.load_json("admm_test_admm.json")
    adj9 = np.array(d["adj"], dtype=np.float64)
    A, its = _gpu([np.array(d["p"])], [adj9], basis=O.BASIS_COMPLEX)
    zs, worst = nine_agent_violations(A[0], adj9)
    assert abs(zs) < d["tol"] and worst < d["tol"], (zs, worst)
    A, its = _gpu([np.array(c["p"]) for c in g["cases"]],
                  [np.array(c["adj"], dtype=np.float64) for c in g["cases"]],
                  basis=O.BASIS_COMPLEX)
    for k, c in enumerate(g["cases"]):
        assert np.linalg.norm(A[k] - np.array(c["A"])) < g["tol"]
    for n in (5, 9, 20):
        cs = [c for c in CASES if c["p"].shape[0] == n][:8]
        A, its = _gpu([c["p"] for c in cs], [c["adj"].astype(np.float64) for c in cs],
                      basis=O.BASIS_COMPLEX)
        for k, c in enumerate(cs):
            Ao, ito = O.design_3d(c["p"], c["adj"], basis=O.BASIS_COMPLEX)
            assert AC.rel_err(A[k], Ao) < REL_TOL, (c["name"], AC.rel_err(A[k], Ao))
            assert tuple(int(x) for x in its[k]) == tuple(ito), (c["name"], its[k], ito)


def test_admm_mixed_batch_properties():
    """A batch mixing planar and 3-D generator formations (n = 20): each
    result equals the oracle's and keeps the reference's properties (trace,
    symmetry, the formation in the kernel)."""
    P20, A20 = H.simform("simform20_nc")
    ps, adjs = [], []
    for f in range(6):
        p = np.array(P20[f, 0], dtype=np.float64)
        if f % 2:
            p[:, 2] = 1.5  # planar: the z kernel is [1] (3D.m:30-46)
        ps.append(p)
        adjs.append(np.asarray(A20[f], dtype=np.float64))
    A, its = _gpu(ps, adjs)
    for k in range(len(ps)):
        Ao, ito = O.design_3d(ps[k], adjs[k])
        assert AC.rel_err(A[k], Ao) < REL_TOL, k
        assert tuple(int(x) for x in its[k]) == tuple(ito)
        n = ps[k].shape[0]
        flat = np.std(ps[k][:, 2], ddof=1) < 1e-2
        assert abs(np.trace(A[k]) + (2 * (n - 2) + n - (1 if flat else 2))) < 1e-6
        np.testing.assert_allclose(A[k], A[k].T, atol=1e-9)


def test_admm_abi_errors():
    import ctypes as ct
    from aclswarm_amd import _lib as L
    lib = L.lib()
    prm = L.default_admm_params()
    assert lib.acl_admm_solve_batch(1, 2, None, None, None, None, ct.byref(prm), None) != 0
    assert lib.acl_admm_solve_batch(0, 10, None, None, None, None, ct.byref(prm), None) == 0


def _psd_ref(W, eps):
    """The reference's projection: keep the eigenvalues > eps (solver.cpp:296-316,
    ADMMGainDesign2D.m:430-445; admm_oracle.Part.run's eigh form)."""
    d, V = np.linalg.eigh(W)
    pos = d > eps
    return (V[:, pos] * d[pos]) @ V[:, pos].T


def _spectrum_case(rng, N, near, eps=1e-5):
    """Symmetric N x N W with |W|_2 = 1 and eigenvalues at eps +- near (and
    eps exactly when near == 0), the rest spread over [-1, 1]."""
    lam = rng.uniform(-1.0, 1.0, N)
    lam[0], lam[1] = 1.0, -1.0
    lam[2], lam[3] = eps + near, eps - near
    Q, _ = np.linalg.qr(rng.normal(size=(N, N)))
    W = (Q * lam) @ Q.T
    return 0.5 * (W + W.T)


def _psd_gpu(Ws, eps, force):
    import ctypes as ct
    import torch
    from aclswarm_amd import _lib as L
    dev = torch.device("cuda:0")
    nm, N = len(Ws), Ws[0].shape[0]
    W = torch.from_numpy(np.stack([np.asfortranarray(w).T.copy() for w in Ws])).to(dev)
    S = torch.empty_like(W)
    used = (ct.c_int * nm)()
    rc = L.lib().acl_internal_psd_project(nm, N, ct.c_void_p(W.data_ptr()), eps,
                                          ct.c_void_p(S.data_ptr()), int(force), used)
    assert rc == 0
    # column-major device matrices: transpose back (symmetric anyway)
    return [m.T for m in S.cpu().numpy()], list(used)


@pytest.mark.parametrize("N", [40, 392])
def test_psd_projection_near_eps(N):
    """The ADMM PSD step on spectra with eigenvalues near epsEig, against the
    eigendecomposition projection the reference uses. 1e-3 |W| away: the
    Newton-Schulz sign converges (slowly) and is used; 1e-12 |W| away: it
    cannot converge in 64 steps and the Jacobi eigensolver fallback makes the
    projection; both within 1e-9 |W| (a misclassified eigenvalue would cost
    ~1e-5; the pair eps +- 1e-12 is a near-degenerate pair whose eigenvectors
    are determined only to ~1e-16 / 2e-12, in any eigensolver, so the kept
    one's direction carries ~1e-11 of the projection). The fallback forced
    on every spectrum agrees too."""
    rng = np.random.RandomState(900 + N)
    eps = 1e-5
    Ws = [_spectrum_case(rng, N, 1e-3), _spectrum_case(rng, N, 1e-12),
          _spectrum_case(rng, N, 0.3)]
    S, used = _psd_gpu(Ws, eps, force=False)
    assert used == [0, 1, 0], used
    for k, W in enumerate(Ws):
        err = np.abs(S[k] - _psd_ref(W, eps)).max()
        assert err <= 1e-9, (k, err)
    S2, used2 = _psd_gpu(Ws, eps, force=True)
    assert used2 == [1, 1, 1], used2
    for k, W in enumerate(Ws):
        err = np.abs(S2[k] - _psd_ref(W, eps)).max()
        assert err <= (1e-9 if k == 1 else 1e-12), (k, err)


@pytest.mark.parametrize("N", [40, 392])
def test_psd_projection_tight_bound(N):
    """Spectra where the Newton-Schulz start's eigenvalue bound is exact: a
    diagonal W has spectral radius = |W - eps I|_inf, so the largest
    |eigenvalue| of Z0 is the kNsScale bound and the first scaled update sits
    at its cap (a |x| = 0.98 sqrt 3); with eigenvalues +-1, eps +- 1e-3 and a
    cluster near 0 every sign still comes out right (the Newton-Schulz path,
    no fallback), within 1e-9 |W| of the eigendecomposition projection; a
    rotated copy of the same spectrum agrees too."""
    rng = np.random.RandomState(77 + N)
    eps = 1e-5
    lam = rng.uniform(-1.0, 1.0, N)
    lam[0], lam[1] = 1.0, -1.0
    lam[2], lam[3] = eps + 1e-3, eps - 1e-3
    lam[4:8] = rng.uniform(-0.05, 0.05, 4)
    D = np.diag(lam)
    Q, _ = np.linalg.qr(rng.normal(size=(N, N)))
    R = (Q * lam) @ Q.T
    Ws = [D, 0.5 * (R + R.T)]
    S, used = _psd_gpu(Ws, eps, force=False)
    assert used == [0, 0], used
    for k, W in enumerate(Ws):
        err = np.abs(S[k] - _psd_ref(W, eps)).max()
        assert err <= 1e-9, (k, err)


def test_admm_c5_full_batch():
    """Config C5 at its size: F = 1024 generator formations (n = 100,
    L = 40, noncomplete; the bench's formations, seeds 0..1023) in one
    acl_admm_solve_batch call, which runs them as one pass of
    ACL_ADMM_CHUNK = 1024 formations (csrc/admm.hip; smaller chunk builds
    reuse the workspace between passes). Every formation: finite,
    symmetric, the trace identity of the reference's design (trace of the
    gain matrix = -(2 (n - 2) + n - 2) for a 3-D formation), both designs
    converged (positive iteration counts). Formations across the batch (0,
    511, 512, 1023 and four random ones) against the CPU restatement: gains
    within 1e-5 relative, equal iteration counts."""
    import torch
    from aclswarm_amd import engine, workload
    dev = torch.device("cuda:0")
    F, n = 1024, 100
    pts, adjb = workload.reference_formations(F, n, 40.0, False, 0, dev)
    A, its = engine.admm_design(pts, adjb.to(torch.float64))
    torch.cuda.synchronize()
    A = A.cpu().numpy()
    its = its.cpu().numpy()
    p = pts.cpu().numpy()
    adj = adjb.cpu().numpy().astype(np.float64)
    assert np.isfinite(A).all()
    assert (its > 0).all(), np.argwhere(its <= 0)[:8]
    sym = np.abs(A - A.transpose(0, 2, 1)).max(axis=(1, 2))
    assert sym.max() < 1e-9, (int(sym.argmax()), sym.max())
    flat = np.std(p[:, :, 2], axis=1, ddof=1) < 1e-2
    want = -(2 * (n - 2) + n - np.where(flat, 1, 2))
    tr = np.trace(A, axis1=1, axis2=2)
    assert np.abs(tr - want).max() < 1e-6, np.abs(tr - want).max()
    rng = np.random.RandomState(1024)
    sample = [0, 511, 512, 1023] + list(rng.randint(1, 511, 2)) + list(rng.randint(513, 1023, 2))
    for f in sample:
        Ao, ito = O.design_3d(p[f], adj[f])
        assert AC.rel_err(A[f], Ao) < REL_TOL, (f, AC.rel_err(A[f], Ao))
        assert tuple(int(x) for x in its[f]) == tuple(ito), (f, its[f], ito)


@pytest.mark.parametrize("basis", [O.BASIS_LINPACK, O.BASIS_COMPLEX])
def test_admm_deterministic(basis):
    """Two calls on the same 64 generator formations (n = 20, noncomplete)
    give bit-identical gains and iteration counts: every sum the outputs
    depend on runs in a fixed order (the wave sums of the basis, the
    per-diagonal-tile trace partials that scale the Newton-Schulz updates,
    summed in tile order); the atomically accumulated sums (|Z^2 - I|_F^2,
    sum |dX|, tr X22) only feed stop decisions."""
    import torch
    from aclswarm_amd import engine, workload
    dev = torch.device("cuda:0")
    pts, adjb = workload.reference_formations(64, 20, 40.0, False, 4096, dev)
    adj = adjb.to(torch.float64)
    A1, i1 = engine.admm_design(pts, adj, basis=basis)
    A2, i2 = engine.admm_design(pts, adj, basis=basis)
    torch.cuda.synchronize()
    assert torch.equal(i1, i2)
    assert torch.equal(A1.view(torch.int64), A2.view(torch.int64))
    assert torch.isfinite(A1).all()


def test_admm_passes_halve_when_workspace_does_not_fit():
    """A batch whose workspace does not fit the device runs in passes of
    fewer formations (halved until a pass fits) instead of failing: with the
    test hook capping workspace allocations, 24 formations at n = 40 run in
    passes of 3 and give the gains and iteration counts of one pass,
    bit for bit."""
    import torch
    from aclswarm_amd import _lib, engine, workload
    dev = torch.device("cuda:0")
    pts, adjb = workload.reference_formations(24, 40, 40.0, False, 11, dev)
    adj = adjb.to(torch.float64)
    A1, i1 = engine.admm_design(pts, adj)
    torch.cuda.synchronize()
    L = _lib.lib()
    # the one-pass workspace (arena0 + arena1) of 24 formations is tens of
    # MB here; 8 MB forces several halvings
    L.acl_internal_admm_mem_cap(8 << 20)
    try:
        A2, i2 = engine.admm_design(pts, adj)
        torch.cuda.synchronize()
    finally:
        L.acl_internal_admm_mem_cap(0)
    assert torch.equal(i1, i2)
    assert torch.equal(A1.view(torch.int64), A2.view(torch.int64))
    # a cap no single formation fits still fails loudly
    L.acl_internal_admm_mem_cap(1 << 10)
    try:
        with pytest.raises(RuntimeError):
            engine.admm_design(pts[:2], adj[:2])
    finally:
        L.acl_internal_admm_mem_cap(0)


def test_admm_large_n_global_cholesky():
    """Eight generator formations at n = 160 (seeds 7..14, L = 60,
    noncomplete): three of them have more than 197 graph rows in the 2-D
    design (Gram systems of 253, 309 and 215), past the LDS Cholesky, so the
    batch factors in global memory (chol_kernel); the sign iteration's parts
    have 8 diagonal tiles (the scaled and quintic updates' trace partials)
    and the post and W passes 20 x 20 blocks. Gains within 1e-5 relative of
    the CPU restatement, equal iteration counts."""
    import torch
    from aclswarm_amd import engine, workload
    dev = torch.device("cuda:0")
    F, n = 8, 160
    pts, adjb = workload.reference_formations(F, n, 60.0, False, 7, dev)
    A, its = engine.admm_design(pts, adjb.to(torch.float64))
    torch.cuda.synchronize()
    A = A.cpu().numpy()
    its = its.cpu().numpy()
    p = pts.cpu().numpy()
    adj = adjb.cpu().numpy().astype(np.float64)
    nonedges = ((adj == 0).sum(axis=(1, 2)) - n) // 2
    assert (2 * nonedges + 1 > 198).sum() >= 3, nonedges
    assert np.isfinite(A).all()
    for f in range(F):
        Ao, ito = O.design_3d(p[f], adj[f])
        assert AC.rel_err(A[f], Ao) < REL_TOL, (f, AC.rel_err(A[f], Ao))
        assert tuple(int(x) for x in its[f]) == tuple(ito), (f, its[f], ito)
