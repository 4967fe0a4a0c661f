"""GPU: the codegen-compatible ADMM entry points (include/aclswarm_amd_codegen.h)
driven as the reference's ADMM wrapper drives the generated library
(aclswarm/src/admm.cpp:13-48; tests/codegen_driver.cpp): the gain matrix is
acl_admm_solve_batch's for the same formation bit for bit, and within 1e-5
of the reference codegen's own outputs (tests/golden/admm_golden.npz)."""
import ctypes as ct

import numpy as np
import pytest

import admm_cases as AC
from test_gpu_admm import _gpu

pytestmark = pytest.mark.gpu

CASES = AC.load()


def _driver():
    from aclswarm_amd import build
    build.build_driver()
    lib = ct.CDLL(build.CG_DRIVER)
    lib.codegen_run.restype = ct.c_int
    lib.codegen_run.argtypes = [ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p]
    return lib


@pytest.mark.parametrize("k", range(0, len(CASES), max(1, len(CASES) // 6)))
def test_codegen_entry_point_equals_batched_design(cuda, k):
    # (`cuda` first: torch brings its own HIP runtime, which must be the
    # process's first to initialise the device; the library then shares it)
    c = CASES[k]
    p = np.ascontiguousarray(c["p"], dtype=np.float64)
    n = p.shape[0]
    adj = np.ascontiguousarray(c["adj"] != 0, dtype=np.uint8)
    g = np.zeros((3 * n) * (3 * n), np.float64)
    dims = np.zeros(2, np.int32)
    lib = _driver()
    rows = lib.codegen_run(n, p.ctypes.data, adj.ctypes.data, g.ctypes.data, dims.ctypes.data)
    assert rows == 3 * n and tuple(dims) == (3 * n, 3 * n)
    G = g.reshape(3 * n, 3 * n).T  # column-major GainMat -> [r][c]
    A, its = _gpu([p], [adj.astype(np.float64)])
    np.testing.assert_array_equal(G, A[0])
    assert AC.rel_err(G, AC.assemble(c["Axy"], c["Az"])) < 1e-5, c["name"]
