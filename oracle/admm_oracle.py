"""CPU restatement of the ADMM formation-gain design -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module; the product path (aclswarm_amd, HIP) never imports it.

What it restates: the MATLAB-Coder ADMM the reference ships
(aclswarm/lib/codegen_admm/ADMMGainDesign3D, spec in
aclswarm/matlab/Helpers/ADMMGainDesign{3D,2D}.m), i.e. SURVEY.md rows a15-a19
with codegen semantics (App. C):
  * kernel N = [q, qbar, ex, ey] (2-D, ADMMGainDesign2D.m:36-49) and
    [qz, 1] or [1] when std(qz) < 1e-2 (ADMMGainDesign3D.m:30-46);
  * Q = trailing columns of U from LINPACK dsvdc (codegen svd1.cpp b_svd /
    d_svd); only the Householder phase determines those columns;
  * SDP standard form (ADMMGainDesign2D.m:72-330, 3D.m:60-300) with trivial
    z-constraint removal (3D.m:85-90, threshold 100*eps);
  * ADMM loop (2D.m:420-455, 3D.m:360-395): mu=1, epsEig=1e-5, thresh=1e-4,
    threshTr=10 (abs, percent), maxItr=10, then the S=0 projection.

How (the restatement, also the design of the HIP path): the y-update
y = (A A^T)^-1 (A vec(C-S-muX) + mu b) followed by W = C - A^T y - mu X and
symmetrisation equals, for symmetric C, S, X,
    W = S + (I - P)(M) - mu x_b,          M = C - S - mu X,
where P projects onto the symmetric part of A's row space. That space splits
into blocks: X11 -> traceless symmetric; X12 -> everything; X22 -> the
structure rows T (2-D only: 2x2 blocks [a b; -b a]) plus span{I, H_k},
H_k = P_struct(sym(q_a q_b^T)) for each graph row (q_a = row a of Q). So
    (I-P)(M)11 = tr(M11)/s * I,  (I-P)(M)12 = 0,
    (I-P)(M)22 = P_V(M22) = P_struct(M22) - c0 I - P_struct(sym(Q^T C Q)),
with Gamma c = r, r_k = <H_k, M22>, Gamma the (K+1)^2 Gram matrix of {I, H_k}
(closed form from the row Gram of Q), C sparse with c_k at (a_k, b_k); x_b =
[0 I; I 0] + blkdiag(0, h_b), h_b the minimum-norm point of the affine
X22 constraints (Gamma c_b = s e_0). Parity against the reference itself
(oracle/_ref/libadmm_ref.so) is checked in tests/test_admm.py.
"""
import math

import numpy as np

EPS = np.finfo(np.float64).eps


# ---------------------------------------------------------------- kernel basis
TINY = 1.0020841800044864e-292      # codegen's reciprocal-scaling guard


def _nrm2(x):
    """codegen xnrm2/b_xnrm2 (xnrm2.cpp): scaled sequential 2-norm."""
    if len(x) == 1:
        return abs(x[0])
    y = 0.0
    scale = 3.3121686421112381e-170
    for v in x:
        a = abs(v)
        if a > scale:
            t = scale / a
            y = y * t * t + 1.0
            scale = a
        else:
            t = a / scale
            y += t * t
    return scale * math.sqrt(y)


def _dot(x, y):
    d = 0.0
    for a, b in zip(x, y):
        d += a * b
    return d


def linpack_complement(N):
    """U(:, p+1:n) of the codegen's LINPACK dsvdc (svd1.cpp b_svd:27-330 for
    p=4, d_svd:601-870 for p<=2): the left Householder reflectors of the
    bidiagonalisation -- with dsvdc's right reflectors, which change later
    columns when p > 2 -- applied to the trailing identity columns (the QR
    sweep that follows only touches columns <= p).

    The arithmetic is replayed in the codegen's exact order (sequential dots,
    scaled norms, multiply by the reciprocal): for the 2-D kernel
    [q, qbar, ex, ey] the first right reflector's sign is decided by the sign
    of A(1,2) = -(q . qbar)/|q|, which is pure rounding noise (q is exactly
    orthogonal to qbar), and Q -- and with it the structure-constrained
    design -- depends on that sign."""
    A = np.array(N, dtype=np.float64, copy=True)
    n, p = A.shape
    nct = min(n - 1, p)
    nrt = max(0, min(p - 2, n))
    s = np.zeros(p)
    e = np.zeros(p)
    U = np.zeros((n, n))
    for q in range(max(nct, nrt)):
        apply = False
        if q < nct:
            nrm = _nrm2(A[q:, q].tolist())
            if nrm > 0.0:
                apply = True
                r = -nrm if A[q, q] < 0.0 else nrm
                if abs(r) >= TINY:
                    A[q:, q] *= 1.0 / r
                else:
                    A[q:, q] /= r
                A[q, q] += 1.0
                s[q] = -r
            else:
                s[q] = 0.0
        for jj in range(q + 1, p):
            if apply:
                t = -(_dot(A[q:, q].tolist(), A[q:, jj].tolist()) / A[q, q])
                if t != 0.0:
                    A[q:, jj] += t * A[q:, q]
            e[jj] = A[q, jj]
        if q < nct:
            U[q:, q] = A[q:, q]
        if q < nrt:
            nrm = _nrm2(e[q + 1:].tolist()) if p - q - 1 > 1 else abs(e[q + 1])
            if nrm == 0.0:
                e[q] = 0.0
            else:
                e[q] = -nrm if e[q + 1] < 0.0 else nrm
                if abs(e[q]) >= TINY:
                    e[q + 1:] *= 1.0 / e[q]
                else:
                    e[q + 1:] /= e[q]
                e[q + 1] += 1.0
                e[q] = -e[q]
                if q + 2 <= n:
                    work = np.zeros(n)
                    for jj in range(q + 1, p):
                        if e[jj] != 0.0:
                            work[q + 1:] += e[jj] * A[q + 1:, jj]
                    for jj in range(q + 1, p):
                        a = -e[jj] / e[q + 1]
                        if a != 0.0:
                            A[q + 1:, jj] += a * work[q + 1:]
    for jj in range(nct, n):
        U[jj, jj] = 1.0
    for q in range(nct - 1, -1, -1):
        if s[q] != 0.0:
            u = U[q:, q].tolist()
            for jj in range(max(q + 1, p), n):
                t = -(_dot(u, U[q:, jj].tolist()) / u[0])
                if t != 0.0:
                    U[q:, jj] += t * U[q:, q]
    return U[:, p:]


def kernel_2d(p_xy):
    """N = [qs, qsbar, one1, one2] (ADMMGainDesign2D.m:36-49); qs = Qs(:)
    interleaves x, y per agent."""
    n = p_xy.shape[0]
    qs = np.asarray(p_xy, dtype=np.float64).reshape(-1)
    qsbar = np.zeros(2 * n)
    qsbar[0::2] = -qs[1::2]
    qsbar[1::2] = qs[0::2]
    one1 = np.zeros(2 * n)
    one1[0::2] = 1.0
    one2 = np.zeros(2 * n)
    one2[1::2] = 1.0
    return np.stack([qs, qsbar, one1, one2], axis=1)


def complex_complement(p_xy):
    """The ACL_ADMM_BASIS_COMPLEX basis of the 2-D part (not in the
    reference): an orthonormal basis of the complement of the same kernel
    span{qs, qsbar, one1, one2}, built complex-structured. With z = x + iy the
    kernel is the complex span of {z, 1}; two complex Householder reflectors
    H1, H2 triangularise [z, 1] (H = I - beta v v^H, beta = 2/|v|^2,
    alpha = -phase(x0)|x|), w_k = H1 H2 e_k (k = 2..n-1) span the complex
    complement, and each w_k gives the real column pair (emb(w_k),
    emb(i w_k)), emb interleaving (Re, Im) per agent. A Q of that form
    commutes with the 2x2 [a b; -b a] structure, so the design's output is
    complex-linear and meets the graph rows exactly -- the properties
    aclswarm/test/test_admm.cpp:84-187 assert, which the codegen's LINPACK
    basis (rounding-noise sign choice, linpack_complement) violates by
    ~1e-1 on that test's formation. Any complex-structured orthonormal basis
    gives the same design up to rounding (the SDP and ADMM iterates are
    equivariant under complex-unitary changes of basis). Restates
    admm.hip basis_kernel's basis == 1 branch (the same operations; the
    kernel sums v1^H w as a wave tree, numpy's vdot pairwise)."""
    p_xy = np.asarray(p_xy, dtype=np.float64)
    n = p_xy.shape[0]
    z = p_xy[:, 0] + 1j * p_xy[:, 1]

    def reflector(x):
        nrm = math.sqrt(float(np.sum(x.real * x.real + x.imag * x.imag)))
        if nrm == 0.0:
            return None, 0.0
        a0 = abs(x[0])
        ph = x[0] / a0 if a0 > 0.0 else 1.0
        v = x.copy()
        v[0] += ph * nrm                   # x0 - alpha, alpha = -ph |x|
        vv = float(np.sum(v.real * v.real + v.imag * v.imag))
        return v, 2.0 / vv

    v1, b1 = reflector(z)
    y = np.ones(n, dtype=np.complex128)
    if v1 is not None:
        y = y - b1 * v1 * np.vdot(v1, y)
    v2, b2 = reflector(y[1:])
    W = np.zeros((n, n - 2), dtype=np.complex128)
    for k in range(2, n):
        w = np.zeros(n, dtype=np.complex128)
        w[k] = 1.0
        if v2 is not None:
            w[1:] -= b2 * v2 * np.conj(v2[k - 1])
        if v1 is not None:
            w -= b1 * v1 * np.vdot(v1, w)
        W[:, k - 2] = w
    Q = np.zeros((2 * n, 2 * (n - 2)))
    Q[0::2, 0::2] = W.real
    Q[1::2, 0::2] = W.imag
    Q[0::2, 1::2] = -W.imag
    Q[1::2, 1::2] = W.real
    return Q


def kernel_z(qz):
    """[qz, 1], or [1] for a planar formation: std(qz) < 1e-2 with MATLAB's
    n-1 normalisation (ADMMGainDesign3D.m:30-46, codegen 3D.cpp:196)."""
    n = qz.shape[0]
    sd = np.std(qz, ddof=1) if n > 1 else 0.0
    if sd < 1e-2:
        return np.ones((n, 1))
    return np.stack([qz, np.ones(n)], axis=1)


def nonedges(adj):
    """[idxRow, idxCol] = find(triu(~adj - diag)) in MATLAB column-major order."""
    a = np.asarray(adj) != 0
    n = a.shape[0]
    out = []
    for j in range(n):
        for i in range(j):
            if not a[i, j]:
                out.append((i, j))
    return out


# ---------------------------------------------------------------- projections
def p_struct(M):
    """Orthogonal projection of a symmetric 2m x 2m matrix onto block
    [a b; -b a] structure (the complement of the structure rows,
    ADMMGainDesign2D.m:221-265)."""
    s = M.shape[0]
    B = M.reshape(s // 2, 2, s // 2, 2)
    a = 0.5 * (B[:, 0, :, 0] + B[:, 1, :, 1])
    b = 0.5 * (B[:, 0, :, 1] - B[:, 1, :, 0])
    out = np.empty_like(B)
    out[:, 0, :, 0] = a
    out[:, 1, :, 1] = a
    out[:, 0, :, 1] = b
    out[:, 1, :, 0] = -b
    return out.reshape(s, s)


def _pivoted_cholesky(G, rel_tol=1e-10):
    """Cholesky of the Gram matrix over a maximal independent subset of its
    rows, in order (a row is dropped when its residual pivot is below
    rel_tol * its diagonal): returns (kept indices, lower factor)."""
    keep = []
    L = np.zeros((0, 0))
    for k in range(G.shape[0]):
        if keep:
            l = np.linalg.solve(L, G[keep, k])
            d = G[k, k] - l @ l
        else:
            l = np.zeros(0)
            d = G[k, k]
        if d <= rel_tol * G[k, k]:
            continue
        m = len(keep)
        L2 = np.zeros((m + 1, m + 1))
        L2[:m, :m] = L
        L2[m, :m] = l
        L2[m, m] = math.sqrt(d)
        L = L2
        keep.append(k)
    return np.array(keep, dtype=np.int64), L


class Part:
    """One ADMM sub-problem (the 2-D xy design or the 1-D z design)."""

    def __init__(self, Q, pairs, structured):
        self.Q = Q
        self.s = Q.shape[1]
        self.pairs = pairs            # graph rows: (a, b) -> (Q X22 Q^T)[a, b] = 0
        self.structured = structured
        K = len(pairs)
        G = Q @ Q.T                   # row Gram of Q
        Gam = np.zeros((K + 1, K + 1))
        Gam[0, 0] = self.s
        if structured:
            Qc = Q[:, 0::2] + 1j * Q[:, 1::2]     # complexified rows
            Psi = Qc @ Qc.conj().T                # <x, y> = sum x_I conj(y_I)
            for k, (a, b) in enumerate(pairs):
                Gam[0, k + 1] = Gam[k + 1, 0] = G[a, b]
                for l, (c, d) in enumerate(pairs):
                    t = (Psi[a, c] * Psi[d, b] + Psi[a, d] * Psi[c, b]
                         + Psi[b, c] * Psi[d, a] + Psi[b, d] * Psi[c, a])
                    Gam[k + 1, l + 1] = 2.0 * t.real / 16.0
        else:
            for k, (a, b) in enumerate(pairs):
                Gam[0, k + 1] = Gam[k + 1, 0] = G[a, b]
                for l, (c, d) in enumerate(pairs):
                    Gam[k + 1, l + 1] = 0.5 * (G[a, c] * G[b, d] + G[a, d] * G[b, c])
        self.Gam = Gam
        rhs = np.zeros(K + 1)
        rhs[0] = self.s
        # The graph rows can be linearly dependent (e.g. swarm6_3d formation 1),
        # making A A^T singular; A^T y -- the projection -- is unique anyway,
        # so any consistent solve gives it (codegen: LU, QR fallback,
        # sparse.cpp:735-741). Pivoted Cholesky dropping dependent rows here.
        self.keep, self.L = _pivoted_cholesky(Gam)
        self.hb = self.combine(self.gsolve(rhs))

    def gsolve(self, r):
        c = np.zeros(len(r))
        k = self.keep
        y = np.linalg.solve(self.L, r[k])
        c[k] = np.linalg.solve(self.L.T, y)
        return c

    def ps(self, M):
        return p_struct(M) if self.structured else M

    def combine(self, c):
        """c0 I + P_struct(sym(sum_k c_k q_a q_b^T))."""
        n = self.Q.shape[0]
        Cm = np.zeros((n, n))
        for k, (a, b) in enumerate(self.pairs):
            Cm[a, b] += c[k + 1]
        T = self.Q.T @ Cm @ self.Q
        return c[0] * np.eye(self.s) + self.ps(0.5 * (T + T.T))

    def pv(self, M22):
        """Projection onto the free X22 subspace V."""
        Pm = self.ps(M22)
        R = self.Q @ Pm @ self.Q.T
        r = np.empty(len(self.pairs) + 1)
        r[0] = np.trace(M22)
        for k, (a, b) in enumerate(self.pairs):
            r[k + 1] = R[a, b]
        return Pm - self.combine(self.gsolve(r))

    def run(self, mu=1.0, eps_eig=1e-5, thresh=1e-4, thresh_tr=10.0, max_itr=10):
        s = self.s
        I = np.eye(s)
        X = np.block([[I, I], [I, I]])
        S = np.zeros_like(X)
        C = np.zeros_like(X)
        C[:s, :s] = I
        itr = 0
        for itr in range(1, max_itr + 1):
            M = C - S - mu * X
            W = S.copy()
            W[:s, :s] += (np.trace(M[:s, :s]) / s) * I
            W[:s, s:] -= mu * I
            W[s:, :s] -= mu * I
            W[s:, s:] += self.pv(M[s:, s:]) - mu * self.hb
            W = 0.5 * (W + W.T)
            d, V = np.linalg.eigh(W)
            pos = d > eps_eig
            S = (V[:, pos] * d[pos]) @ V[:, pos].T
            Xold = X
            X = (S - W) / mu
            if np.abs(Xold - X).sum() < thresh:
                break
            if abs(np.trace(X[s:, s:]) - s) / s * 100.0 < thresh_tr:
                break
        X22 = self.hb + self.pv(X[s:, s:] - C[s:, s:] / mu)
        return self.Q @ (-X22) @ self.Q.T, itr


BASIS_LINPACK, BASIS_COMPLEX = 0, 1     # acl_admm_params_t.basis


def design_2d(p_xy, adj, basis=BASIS_LINPACK, **kw):
    if basis == BASIS_COMPLEX and np.asarray(p_xy).shape[0] > 2:
        Q = complex_complement(p_xy)
    else:
        Q = linpack_complement(kernel_2d(p_xy))
    pairs = []
    for (i, j) in nonedges(adj):
        pairs.append((2 * i, 2 * j))
        pairs.append((2 * i + 1, 2 * j))
    return Part(Q, pairs, True).run(**kw)


def design_z(qz, adj, **kw):
    Q = linpack_complement(kernel_z(qz))
    zro = set(np.nonzero(np.abs(Q).sum(axis=1) < 100 * EPS)[0].tolist())
    pairs = [(i, j) for (i, j) in nonedges(adj) if i not in zro and j not in zro]
    return Part(Q, pairs, False).run(**kw)


def design_3d(p, adj, prune=True, basis=BASIS_LINPACK, **kw):
    """ADMMGainDesign3D (+ the |a| < 1e-10 zeroing of admm.cpp:50). p: n x 3.
    basis selects the 2-D complement basis (BASIS_LINPACK = codegen parity,
    BASIS_COMPLEX = complex_complement). Returns (Aopt 3n x 3n,
    (iters_xy, iters_z))."""
    p = np.asarray(p, dtype=np.float64)
    n = p.shape[0]
    Axy, it_xy = design_2d(p[:, :2], adj, basis=basis, **kw)
    Az, it_z = design_z(p[:, 2].copy(), adj, **kw)
    A = np.zeros((3 * n, 3 * n))
    for i in range(n):
        for j in range(n):
            A[3 * i:3 * i + 2, 3 * j:3 * j + 2] = Axy[2 * i:2 * i + 2, 2 * j:2 * j + 2]
            A[3 * i + 2, 3 * j + 2] = Az[i, j]
    if prune:
        A[~(np.abs(A) > 1e-10)] = 0.0
    return A, (it_xy, it_z)
