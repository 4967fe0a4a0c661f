#!/usr/bin/env python3
"""Diagnostic: Newton-Schulz update counts of the ADMM PSD projection on the
C5 designs' spectra (csrc/admm.hip kNsCap). Captures every W the CPU
restatement (oracle/admm_oracle.py, test infrastructure) projects for the
first SEEDS generator formations (n = 100, L = 40, noncomplete, complex
basis) and runs the sign iteration on W's eigenvalues (the updates act on
each eigenvalue separately): unscaled from Z0 = (W - eps I) / (|.|_inf / 1.5),
and with the per-update rescaling a = sqrt(dim / tr Z^2), capped as the
kernel caps it, a = 1 on the last update."""
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


def updates(x, scaled):
    k, bound = 0, SCALE
    while True:
        conv = ((x * x - 1.0) ** 2).sum() < TOL * len(x)
        a = 1.0
        if scaled and not conv:
            a = min(np.sqrt(len(x) / (x * x).sum()), CAP / bound)
        y = a * x
        x = 1.5 * y - 0.5 * y ** 3
        k, bound = k + 1, 1.0
        if conv or k >= 64:
            return k, np.abs(np.abs(x) - 1.0).max()


for scaled in (False, True):
    r = [updates(x.copy(), scaled) for x in spectra]
    k = np.array([a for a, _ in r])
    print(f"{'scaled' if scaled else 'unscaled':9s} projections {len(k)}: updates mean {k.mean():.2f} "
          f"max {k.max()}  histogram { {int(a): int(b) for a, b in zip(*np.unique(k, return_counts=True))} }  "
          f"max | |sign| - 1 | {max(e for _, e in r):.1e}")
