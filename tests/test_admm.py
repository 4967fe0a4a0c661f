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
