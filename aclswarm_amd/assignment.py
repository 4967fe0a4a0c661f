"""Drop-in for aclswarm/src/aclswarm/assignment.py (the centralized
comparator), computed on the GPU by acl_hungarian_batch.

Same names, argument meaning and return values as the reference:
  find_optimal_assignment(q, p, last=None) -> (P list, paligned)   (:94-137)
  align(q, p) -> paligned                                           (:55-92)
with q, p as d x n numpy arrays (d = 3). The batched form
find_optimal_assignments(q[B][n][3], p[F][n][3], fidx, last, P_cmp) works on
device tensors for many swarms at once. Errors follow the reference's
dependencies: a `last` that is not a permutation raises ValueError (the
reference would silently misalign), a NaN / -inf cost or an infeasible
matrix raises ValueError as scipy's linear_sum_assignment does.
There is no CPU fallback: without the HIP library these raise.
"""
import numpy as np
import torch

from . import _lib as L
from . import engine


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("aclswarm_amd.assignment: no GPU (the comparator runs on the MI355X)")
    return torch.device("cuda", torch.cuda.current_device())


def find_optimal_assignments(q, p, fidx, last=None, P_cmp=None, stream=None):
    """Batched find_optimal_assignment on device tensors: q [B][n][3] f64,
    p [F][n][3] f64, fidx [B] i32, last / P_cmp [B][n] int16 (uint16 bits)
    or None. Returns engine.hungarian's dict (P_opt, cost, status, align_Rt)."""
    n = int(q.shape[1])
    F = int(p.shape[0])
    W = (n + 63) // 64
    dev = q.device
    T = engine.FormationTable(n, p.contiguous(), torch.zeros((F, n, W), dtype=torch.int64, device=dev),
                              torch.zeros(9, dtype=torch.float64, device=dev),
                              torch.zeros(F, dtype=torch.int64, device=dev), 9)
    return engine.hungarian(T, fidx, q.contiguous(), last, P_cmp, want_Rt=True, stream=stream)


def _one(q, p, last):
    q = np.asarray(q, np.float64)
    p = np.asarray(p, np.float64)
    if q.ndim != 2 or q.shape != p.shape or q.shape[0] not in (2, 3):
        raise ValueError("q and p must be d x n arrays of the same shape (d = 2 or 3)")
    d, n = q.shape
    q3 = np.zeros((n, 3)); q3[:, :d] = q.T
    p3 = np.zeros((n, 3)); p3[:, :d] = p.T
    dev = _device()
    lastt = None
    if last is not None:
        lastt = torch.from_numpy(np.asarray(last, np.uint16).reshape(1, n).view(np.int16)).to(dev)
    out = find_optimal_assignments(torch.from_numpy(q3).reshape(1, n, 3).to(dev),
                                   torch.from_numpy(p3).reshape(1, n, 3).to(dev),
                                   torch.zeros(1, dtype=torch.int32, device=dev), lastt)
    st = int(out["status"].item())
    if st & L.HUNG_BAD_INPUT:
        raise ValueError("last is not a permutation of 0..n-1")
    if st & L.HUNG_NONFINITE:
        raise ValueError("cost matrix is infeasible or contains NaN / -inf")
    c, s, tx, ty = out["align_Rt"][0].cpu().numpy()
    pal = np.empty_like(p)
    pal[0] = (c * p[0] - s * p[1]) + tx
    pal[1] = (s * p[0] + c * p[1]) + ty
    if d == 3:
        pal[2] = p[2]
    P = out["P_opt"][0].cpu().numpy().view(np.uint16).astype(np.int64)
    return P.tolist(), pal


def find_optimal_assignment(q, p, last=None):
    """assignment.py:94-137: (P, paligned), P[vehid] = formation point."""
    return _one(q, p, last)


def align(q, p):
    """assignment.py:55-92: the formation p aligned onto q (2-D Arun, z kept)."""
    return _one(q, p, None)[1]
