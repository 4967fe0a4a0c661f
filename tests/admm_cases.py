"""ADMM golden cases (tests/golden/admm_golden.npz, made by
tests/golden/make_admm_fixtures.py from the reference's own codegen ADMM)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    z = np.load(os.path.join(GOLDEN, "admm_golden.npz"), allow_pickle=False)
    cases = []
    for name in z["names"]:
        name = str(name)
        cases.append({"name": name, "p": z[name + "/p"], "adj": z[name + "/adj"],
                      "Axy": z[name + "/Axy"], "Az": z[name + "/Az"]})
    return cases


def assemble(Axy, Az):
    """The 3n x 3n gain matrix from its xy and z parts (ADMMGainDesign3D.m:412-420)."""
    n = Az.shape[0]
    A = np.zeros((3 * n, 3 * n))
    for i in range(n):
        for j in range(n):
            A[3 * i:3 * i + 2, 3 * j:3 * j + 2] = Axy[2 * i:2 * i + 2, 2 * j:2 * j + 2]
    A[2::3, 2::3] = Az
    return A


def rel_err(A, B):
    return float(np.abs(A - B).max() / max(np.abs(B).max(), 1e-300))
