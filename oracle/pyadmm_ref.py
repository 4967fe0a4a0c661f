"""ctypes binding of the reference's own MATLAB-Coder ADMM -- TEST INFRASTRUCTURE.

oracle/_ref/libadmm_ref.so is compiled by `make -C oracle ref` from
aclswarm/lib/codegen_admm/ADMMGainDesign3D/*.cpp (+ vendored CXSparse) where
they lie in the reference tree, plus oracle/admm_ref_shim.cpp. It is the
ADMM parity oracle: codegen semantics of
matlab/Helpers/ADMMGainDesign{3D,2D}.m. Only tests/, smoke() and bench.py's
cpu_baseline leg may use it.
"""
import ctypes as ct
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_LIB = os.path.join(HERE, "_ref", "libadmm_ref.so")
_lib = None


def available():
    return os.path.exists(REF_LIB)


def lib():
    global _lib
    if _lib is None:
        if not available():
            raise RuntimeError(f"{REF_LIB} missing: run `make -C oracle ref` "
                               "where /root/reference is mounted")
        L = ct.CDLL(REF_LIB)
        L.admm_ref_solve.argtypes = [ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_void_p,
                                     ct.c_int]
        L.admm_ref_solve.restype = ct.c_int
        _lib = L
    return _lib


def solve(p, adj, prune=True):
    """ADMM::calculateFormationGains (aclswarm/src/admm.cpp:32-51).

    p: n x 3 formation points (PtsMat), adj: n x n 0/1. Returns the 3n x 3n
    gain matrix (|a| < 1e-10 zeroed when prune, admm.cpp:50)."""
    p = np.asarray(p, dtype=np.float64)
    n = p.shape[0]
    pts = np.asfortranarray(p.T)                 # 3 x n column-major
    A = np.asfortranarray(np.asarray(adj, dtype=np.float64))
    out = np.zeros((3 * n, 3 * n), dtype=np.float64, order="F")
    rc = lib().admm_ref_solve(n, pts.ctypes.data, A.ctypes.data, out.ctypes.data,
                              1 if prune else 0)
    if rc != 0:
        raise RuntimeError("reference ADMM returned an unexpected shape")
    return np.ascontiguousarray(out)
