#!/usr/bin/env python3
"""Diagnostic: Newton-Schulz update counts of the ADMM PSD projection on the
C5 designs' spectra (csrc/admm.hip kNsCap). Captures every W the CPU
restatement (oracle/admm_oracle.py, test infrastructure) projects for the
first SEEDS generator formations (n = 100, L = 40, noncomplete, complex
basis) and runs the sign iteration on W's eigenvalues (the updates act on
each eigenvalue separately): unscaled from Z0 = (W - eps I) / (|.|_inf / 1.5),
and with the per-update rescaling a = sqrt(dim / tr Z^2), capped as the
kernel caps it, a = 1 on the last update; and with the quintic final update
for a check in [1e-12, 1e-8) dim (kNsTolQ)."""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from oracle import admm_oracle as A  # noqa: E402
from oracle.formation_gen_oracle import generate_formation_group  # noqa: E402

SEEDS = int(sys.argv[1]) if len(sys.argv) > 1 else 6
EPS, TOL, SCALE, CAP = 1e-5, 1e-12, 1.5, 0.98 * np.sqrt(3.0)
spectra = []
_eigh = np.linalg.eigh


def _capture(W):
    d, V = _eigh(W)
    z = W - EPS * np.eye(len(W))
    spectra.append((d - EPS) / (np.abs(z).sum(0).max() / SCALE))
    return d, V


A.np.linalg.eigh = _capture
for seed in range(SEEDS):
    adj, forms, _ = generate_formation_group(seed, 100, False, 40.0, 40.0, 2.0, 2.0)
    A.design_3d(np.array(forms[0], dtype=float), np.array(adj, dtype=float),
                basis=A.BASIS_COMPLEX)


TOLQ = 1e-8  # kNsTolQ: the quintic final update's band [TOL, TOLQ)


def updates(x, scaled, quintic=False):
    """-> (updates, products, largest | |sign| - 1 |): products counts the
    Z^2 checks and the update products (two for a quintic update)."""
    k, g, bound = 0, 0, SCALE
    while True:
        g += 1  # Y = Z^2 and its check
        err = ((x * x - 1.0) ** 2).sum()
        conv = err < TOL * len(x)
        if quintic and not conv and err < TOLQ * len(x):
            y = x * x
            x = x * (15.0 - 10.0 * y + 3.0 * y * y) / 8.0
            return k + 1, g + 2, np.abs(np.abs(x) - 1.0).max()
        a = 1.0
        if scaled and not conv:
            a = min(np.sqrt(len(x) / (x * x).sum()), CAP / bound)
        y = a * x
        x = 1.5 * y - 0.5 * y ** 3
        k, g, bound = k + 1, g + 1, 1.0
        if conv or k >= 64:
            return k, g, np.abs(np.abs(x) - 1.0).max()


for name, scaled, quintic in (("unscaled", False, False), ("scaled", True, False),
                              ("scaled+quintic", True, True)):
    r = [updates(x.copy(), scaled, quintic) for x in spectra]
    k = np.array([a for a, _, _ in r])
    g = np.array([b for _, b, _ in r])
    print(f"{name:15s} projections {len(k)}: updates mean {k.mean():.2f} max {k.max()}, "
          f"products mean {g.mean():.2f} max {g.max()}, "
          f"max | |sign| - 1 | {max(e for _, _, e in r):.1e}")
