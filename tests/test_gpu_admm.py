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


def _gpu(ps, adjs):
    import torch
    from aclswarm_amd import engine
    dev = torch.device("cuda:0")
    pts = torch.from_numpy(np.ascontiguousarray(np.stack(ps), dtype=np.float64)).to(dev)
    adj = torch.from_numpy(np.ascontiguousarray(np.stack(adjs), dtype=np.float64)).to(dev)
    A, its = engine.admm_design(pts, adj)
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
