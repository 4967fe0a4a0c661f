"""CPU suite for the ADMM gain design: the oracle
restatement against the reference's own outputs, and the properties
aclswarm/test/test_admm.cpp asserts."""
import numpy as np
import pytest

import admm_cases as AC
import admm_oracle as O
import helpers as H

CASES = AC.load()
TOL = 1e-9          # oracle vs reference, relative to max |A| (both fp64)


def _small(c):
    return c["p"].shape[0] <= 20


@pytest.mark.parametrize("case", [c for c in CASES if _small(c)], ids=lambda c: c["name"])
def test_oracle_matches_reference(case):
    A, its = O.design_3d(case["p"], case["adj"])
    ref = AC.assemble(case["Axy"], case["Az"])
    assert AC.rel_err(A, ref) < TOL
    assert 1 <= its[0] <= 10 and 1 <= its[1] <= 10


@pytest.mark.slow
def test_oracle_matches_reference_n100():
    c = [c for c in CASES if c["name"] == "nc100_s0"][0]
    A, _ = O.design_3d(c["p"], c["adj"])
    assert AC.rel_err(A, AC.assemble(c["Axy"], c["Az"])) < TOL


def test_test_admm_goldens():
    """aclswarm/test/test_admm.cpp:10-80 (the two MATLAB 12x12 matrices)."""
    d = H.load_json("admm_test_admm.json")
    for c in d["cases"]:
        A, _ = O.design_3d(np.array(c["p"]), np.array(c["adj"]))
        assert np.linalg.norm(A - np.array(c["A"])) < d["tol"]


@pytest.mark.parametrize("case", [c for c in CASES if _small(c)], ids=lambda c: c["name"])
def test_reference_properties(case):
    """Trace, symmetry and kernel of the reference's own output: trace is
    -(2(n-2) + n - dimker) (the trVal constraints), the formation lies in the
    kernel (A p = 0 per axis block), A is symmetric."""
    p, n = case["p"], case["p"].shape[0]
    A = AC.assemble(case["Axy"], case["Az"])
    flat = np.std(p[:, 2], ddof=1) < 1e-2
    assert abs(np.trace(A) + (2 * (n - 2) + n - (1 if flat else 2))) < 1e-8
    np.testing.assert_allclose(A, A.T, atol=1e-9)
    np.testing.assert_allclose(case["Axy"] @ p[:, :2].reshape(-1), 0, atol=1e-8)
    np.testing.assert_allclose(case["Axy"] @ np.tile([1.0, 0.0], n), 0, atol=1e-8)
    np.testing.assert_allclose(case["Az"] @ np.ones(n), 0, atol=1e-8)


def test_linpack_basis_is_orthonormal_complement():
    rng = np.random.RandomState(3)
    for n in (3, 7, 20):
        N = O.kernel_2d(rng.uniform(-5, 5, (n, 2)))
        Q = O.linpack_complement(N)
        np.testing.assert_allclose(Q.T @ Q, np.eye(2 * n - 4), atol=1e-13)
        np.testing.assert_allclose(N.T @ Q, 0, atol=1e-12)
    Q = O.linpack_complement(O.kernel_z(np.ones(5)))
    np.testing.assert_allclose(Q.sum(axis=0), 0, atol=1e-14)


def test_reference_lib_when_built():
    """When oracle/_ref is built (build container), the reference itself
    reproduces the fixtures bit-for-bit."""
    import pyadmm_ref as R
    if not R.available():
        pytest.skip("oracle/_ref not built")
    for c in CASES:
        if c["p"].shape[0] > 20:
            continue
        A = R.solve(c["p"], c["adj"])
        assert AC.rel_err(A, AC.assemble(c["Axy"], c["Az"])) == 0.0


def nine_agent_violations(A, adj):
    """The two assertions of aclswarm/test/test_admm.cpp:84-187, as numbers:
    (sum over the non-edge 3x3 blocks, :113-122) and the largest violation of
    the one-sided block-structure checks (:165-171)."""
    n = adj.shape[0]
    adjbar = np.abs(adj - 1.0) - np.eye(n)
    zero_sum = float((np.kron(adjbar, np.ones((3, 3))) * A).sum())
    worst = 0.0
    for i in range(n):
        for j in range(n):
            b = A[3 * i:3 * i + 3, 3 * j:3 * j + 3]
            v = (b[0, 0] - b[1, 1], b[1, 0] + b[0, 1], b[0, 2], b[2, 0], b[1, 2], b[2, 1])
            worst = max(worst, max(v))
    return zero_sum, worst


def test_nine_agent_codegen_basis_recorded():
    """Codegen semantics (the default LINPACK basis) do NOT meet
    test_admm.cpp:84-187: the reference's codegen ADMM gives the same
    violations (oracle == libadmm_ref on the fixtures). Recorded, not hidden:
    the zero-block sum is ~9.4e-2 and the structure is broken by ~7.6e-2."""
    d = H.load_json("admm_nine_agent.json")
    A, _ = O.design_3d(np.array(d["p"]), np.array(d["adj"], dtype=np.float64))
    zs, worst = nine_agent_violations(A, np.array(d["adj"], dtype=np.float64))
    assert abs(zs - 9.383e-2) < 1e-4 and abs(worst - 7.622e-2) < 1e-4


def test_nine_agent_complex_basis_meets_test_admm():
    """ACL_ADMM_BASIS_COMPLEX meets both nine-agent assertions at the test's
    1e-8 and still reproduces the MATLAB 12x12 matrices (test_admm.cpp:10-80)
    and the fixed traces (:191-227)."""
    d = H.load_json("admm_nine_agent.json")
    adj = np.array(d["adj"], dtype=np.float64)
    A, _ = O.design_3d(np.array(d["p"]), adj, basis=O.BASIS_COMPLEX)
    zs, worst = nine_agent_violations(A, adj)
    assert abs(zs) < d["tol"] and worst < d["tol"]
    g = H.load_json("admm_test_admm.json")
    for c in g["cases"]:
        A, _ = O.design_3d(np.array(c["p"]), np.array(c["adj"]), basis=O.BASIS_COMPLEX)
        assert np.linalg.norm(A - np.array(c["A"])) < g["tol"]
    rng = np.random.RandomState(0)
    for sparse in (False, True):
        a = np.ones((20, 20)) - np.eye(20)
        if sparse:
            a[0, 5] = a[5, 0] = a[3, 15] = a[15, 3] = 0
        A, _ = O.design_3d(rng.uniform(-5, 5, (20, 3)), a, basis=O.BASIS_COMPLEX)
        assert abs(np.trace(A) + 3 * 18) < 1e-8


def test_complex_basis_is_structured_orthonormal_complement():
    rng = np.random.RandomState(5)
    for n in (3, 4, 9, 31):
        p = rng.uniform(-5, 5, (n, 2))
        Q = O.complex_complement(p)
        np.testing.assert_allclose(Q.T @ Q, np.eye(2 * n - 4), atol=1e-13)
        np.testing.assert_allclose(O.kernel_2d(p).T @ Q, 0, atol=1e-12)
        J = np.kron(np.eye(n), [[0.0, -1.0], [1.0, 0.0]])     # multiplication by i
        np.testing.assert_allclose(J @ Q[:, 0::2], Q[:, 1::2], atol=1e-15)
    # degenerate: all agents at one point (z parallel to 1) -> H2 from the
    # residual of 1 alone, still an orthonormal complement
    Q = O.complex_complement(np.ones((5, 2)))
    np.testing.assert_allclose(Q.T @ Q, np.eye(6), atol=1e-13)
