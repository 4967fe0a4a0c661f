// admm.hip -- batched ADMM formation-gain design for gfx950 (SURVEY.md rows
// a15-a19): admm::Solver::solve (aclswarm/lib/admm/src/solver.cpp:28-79) with
// the semantics of the reference's MATLAB-Coder ADMM
// (aclswarm/lib/codegen_admm, spec aclswarm/matlab/Helpers/ADMMGainDesign{3D,2D}.m),
// the one the reference wrapper calls (aclswarm/src/admm.cpp:32-51).
//
// F formations are solved at once; each formation is two independent
// sub-problems ("parts"): the 2-D xy design (ADMMGainDesign2D) and the 1-D z
// design. A part is an SDP in X = [X11 X12; X12' X22] (2s x 2s) solved by at
// most maxItr ADMM iterations. The algebra (derivation in oracle/admm_oracle.py
// and DESIGN.md §6) needs no sparse solve:
//
//   W   = S + (I-P)(C - S - mu X) - mu x_b,  (I-P) blockwise closed form:
//         X11 -> tr/s I, X12 -> 0, X22 -> P_V(M22) = Pm - combine(Ginv r),
//         Pm = P_struct(M22), r_k = q_a' Pm q_b  (K graph rows), r_0 = tr M22,
//         combine(c) = c0 I + P_struct(sym(Qa' diag(c) Qb))
//   S   = PSD part of W (eigenvalues > epsEig)
//   X   = (S - W) / mu
//
// and the PSD projection is a matrix-sign function: S = (W + W sign(W - eps I))/2,
// sign() by the Newton-Schulz iteration Z <- 1.5 Z - 0.5 Z Z^2. The W of this
// problem has its spectrum bounded away from zero (>= 3% of |W| on every
// reference fixture), so the iteration converges in ~7-14 steps. Everything
// dense is a batched fp64 GEMM on the matrix cores (gemm_f64.h); the small
// sequential pieces (LINPACK Householder basis, pivoted Cholesky of the
// (K+1)^2 Gram matrix) run one workgroup per part.
//
// Parity: gains within 1e-5 relative of the reference's codegen output
// (observed ~1e-14, tests/test_gpu_admm.py), iteration counts identical.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/aclswarm_amd.h"
#include "gemm_f64.h"

extern "C" acl_status_t acl__set_error(const char* msg);

namespace acl_amd {
namespace admm {

constexpr int kT = 256;         // threads per workgroup of the per-part kernels
constexpr int kMaxN = 1024;     // points per formation
constexpr int kMaxRows = 2047;  // graph rows (K) per part: the Gram system is (K+1)^2
#ifndef ACL_ADMM_CHUNK
#define ACL_ADMM_CHUNK 1024  // formations per pass at most (~16 GB of workspace at N = 100; 512: 4 728 vs 4 846 formations/s at C5)
#endif
constexpr int kNsMax = 64;      // Newton-Schulz iterations before a part is declared failed
constexpr double kNsScale = 1.5;  // Z0 scaling: |W - eps I|_inf / kNsScale (norm_kernel)
// A part's sign iteration has converged when |Z^2 - I|_F^2 < kNsTol * dim;
// one more update follows, so the sign is good to ~kNsTol relative (the
// oracle check: S within 1e-12 relative of the eigendecomposition's on every
// fixture W; 1e-20 cost ~0.9 more updates per projection for 1e-15).
constexpr double kNsTol = 1e-12;
// Quintic final update (fused builds): a part whose check lands in
// [kNsTol, kNsTolQ) dim takes Z <- Z (15 - 10 Z^2 + 3 Z^4) / 8 (third order,
// no sign change: 3x^4 - 10x^2 + 15 has no real root) as its last update --
// two products (T = 3/8 Y^2 - 10/8 Y, then Z T + 15/8 Z) instead of an update,
// another check and a last update (three). On the C5 spectra: 7.69 -> 7.08
// products per projection, largest | |sign| - 1 | 4.1e-11 -> 5.8e-11
// (scripts/ns_scaling_sim.py).
constexpr double kNsTolQ = 1e-8;
// Scaled updates: before each update the part's Z is rescaled by
// a = sqrt(dim / tr Z^2) (its eigenvalues' root mean square to 1; tr Z^2 from
// the product Y = Z^2 the update reads anyway), at most kNsCap / (a bound on
// |eigenvalue|): kNsScale for Z0, 1 after any update (1.5 y - 0.5 y^3 <= 1 on
// [0, sqrt 3]). a |x| < sqrt 3 keeps every eigenvalue's sign, and a >= 1 once
// every |x| <= 1, so no eigenvalue converges slower than unscaled; a = 1 on
// the last update. On the C5 designs' spectra: 4.76 -> 3.85 updates per
// projection, at most 5 instead of 7 (scripts/ns_scaling_sim.py).
constexpr double kNsCap = 1.6974097914174996;  // 0.98 sqrt(3)
constexpr int kTrMax = 64;                      // diagonal tiles per part for the scaled updates
constexpr double kTiny = 1.0020841800044864e-292;  // codegen reciprocal-scaling guard

struct Info {  // written by basis_kernel
  int np, s, K, st;
};

struct Scal {
  double trM11, c0, nrm, err2, diff, tr22;
  int active, inactive, ns_done, ns_final, ns_upd, ns_fail, itr, pad;
  int skip_s0, skip_s1;  // which S product runs: the sign is in N0 (even updates) or N1
  int ns_fail_now;       // this iteration's sign iteration did not converge: Jacobi fallback
  int jacobi;            // iterations whose projection the Jacobi fallback made
  int jacobi_fail;       // ... of which the fallback hit kJacobiSweeps unconverged
  int pad2;
  double trp[kTrMax];    // tr Z^2 partials, one per diagonal tile (GemmJob::trp)
};

struct Part {
  int np, s, K, st;
  const double* Q;
  const unsigned short* pa;
  const unsigned short* pb;
  double *Qa, *Qb, *Qbc, *Yk;
  double *Gam, *Li, *Ginv;
  double *r, *c;
  double *hb, *Pm, *T;
  double *W, *S, *Sr, *X, *N0, *N1, *Y;
  double* cs;  // [nb][2s] column-sum partials of |W - eps I| per 32-row block (w_ut_kernel, in
               // Y), or NULL: norm_kernel reads W
  double *G, *Pre, *Pim;  // setup (alias W, Sr, Y)
  double *A1, *Ap;        // final (alias N0, N1)
  Scal* sc;
};

// ---------------------------------------------------------------------------
// LINPACK dsvdc Householder phase (svd1.cpp b_svd:27-330 / d_svd:601-870), in
// the codegen's exact arithmetic order; see oracle/admm_oracle.py
// linpack_complement for why the order matters (the sign of a reflector is
// decided by rounding noise).
__device__ double nrm2_seq(const double* x, int len, int stride) {
  if (len == 1) return fabs(x[0]);
  double y = 0.0, scale = 3.3121686421112381e-170;
  for (int k = 0; k < len; ++k) {
    const double a = fabs(x[(size_t)k * stride]);
    if (a > scale) {
      const double t = scale / a;
      y = y * t * t + 1.0;
      scale = a;
    } else {
      const double t = a / scale;
      y += t * t;
    }
  }
  return scale * sqrt(y);
}

// One workgroup per part. Kernel basis N (ADMMGainDesign2D.m:36-49,
// ADMMGainDesign3D.m:30-46), Q = trailing columns of the LINPACK U, the zero
// rows of Q (3D.m:85-90) and the graph rows [idxRow, idxCol] = find(triu(~adj))
// in column-major order (2D.m:72-90).
__global__ void __launch_bounds__(kT) basis_kernel(int n, int Fc, int f0, const double* pts,
                                                   const double* adj, double thrPlanar,
                                                   int basis, double* Qbuf, size_t qstride,
                                                   unsigned short* pairbuf, size_t pstride,
                                                   Info* info) {
  extern __shared__ double sm[];
  const int part = blockIdx.x;
  const bool xy = part < Fc;
  const int f = f0 + (xy ? part : part - Fc);
  const int np = xy ? 2 * n : n;
  const int tid = threadIdx.x;
  double* A = sm;                  // np x 4, column-major
  double* work = A + 4 * np;       // np
  double* sv = work + np;          // 4
  double* ev = sv + 4;             // 4
  int* zro = reinterpret_cast<int*>(ev + 4);  // np
  __shared__ int s_p;
  const double* P = pts + (size_t)f * 3 * n;  // 3 x n column-major: (r, i) at r + 3i
  if (tid == 0) {
    int p;
    if (xy) {
      p = 4;
    } else {
      // std(qz) with n-1 normalisation (3D.m:30-46)
      double mean = 0.0;
      for (int i = 0; i < n; ++i) mean += P[2 + 3 * i];
      mean /= n;
      double ss = 0.0;
      for (int i = 0; i < n; ++i) {
        const double d = P[2 + 3 * i] - mean;
        ss += d * d;
      }
      const double sd = n > 1 ? sqrt(ss / (n - 1)) : 0.0;
      p = sd < thrPlanar ? 1 : 2;
    }
    s_p = p;
  }
  __syncthreads();
  const int p = s_p;
  for (int i = tid; i < np; i += kT) {
    if (xy) {
      const int a = i >> 1, c = i & 1;
      const double x = P[3 * a], y = P[3 * a + 1];
      A[i] = c ? y : x;                 // qs
      A[np + i] = c ? x : -y;           // qsbar
      A[2 * np + i] = c ? 0.0 : 1.0;    // one1
      A[3 * np + i] = c ? 1.0 : 0.0;    // one2
    } else if (p == 1) {
      A[i] = 1.0;
    } else {
      A[i] = P[2 + 3 * i];
      A[np + i] = 1.0;
    }
  }
  __syncthreads();
  const int nct = min(np - 1, p);
  const int nrt = max(0, min(p - 2, np));
  const int s = np - p;
  double* Q = Qbuf + (size_t)part * qstride;
  if (xy && basis == ACL_ADMM_BASIS_COMPLEX && n > 2) {
    // Complex-structured complement (oracle complex_complement): reflectors
    // H1, H2 triangularise [z, 1] (z = x + iy), w_k = H1 H2 e_k, columns
    // (emb(w_k), emb(i w_k)). v1, v2 interleaved (re, im) per agent in A.
    double* v1 = A;            // n complex
    double* v2 = A + 2 * n;    // n complex, v2[0] = 0 (H2 acts on agents 1..n-1)
    if (tid == 0) {
      double b1 = 0.0, b2 = 0.0;
      for (int c = 0; c < 2; ++c) {
        double* v = c ? v2 : v1;
        const int i0 = c;      // first agent the reflector acts on
        for (int i = 0; i < 2 * n; ++i) v[i] = 0.0;
        if (c == 0) {
          for (int i = 0; i < n; ++i) { v[2 * i] = P[3 * i]; v[2 * i + 1] = P[3 * i + 1]; }
        } else {
          // y = H1 1 restricted to agents 1..n-1
          double yr = 0.0, yi = 0.0;   // v1^H 1
          for (int i = 0; i < n; ++i) { yr += v1[2 * i]; yi -= v1[2 * i + 1]; }
          for (int i = 1; i < n; ++i) {
            const double vr = v1[2 * i], vi = v1[2 * i + 1];
            v[2 * i] = 1.0 - b1 * (vr * yr - vi * yi);
            v[2 * i + 1] = -b1 * (vr * yi + vi * yr);
          }
        }
        double ss = 0.0;
        for (int i = i0; i < n; ++i) ss += v[2 * i] * v[2 * i] + v[2 * i + 1] * v[2 * i + 1];
        const double nrm = sqrt(ss);
        double b = 0.0;
        if (nrm != 0.0) {
          const double xr = v[2 * i0], xi = v[2 * i0 + 1];
          const double a0 = sqrt(xr * xr + xi * xi);
          const double pr = a0 > 0.0 ? xr / a0 : 1.0, pi = a0 > 0.0 ? xi / a0 : 0.0;
          v[2 * i0] += pr * nrm;           // x0 - alpha, alpha = -phase(x0) |x|
          v[2 * i0 + 1] += pi * nrm;
          double vv = 0.0;
          for (int i = i0; i < n; ++i) vv += v[2 * i] * v[2 * i] + v[2 * i + 1] * v[2 * i + 1];
          b = 2.0 / vv;
        }
        if (c == 0) b1 = b; else b2 = b;
      }
      sv[0] = b1; sv[1] = b2;
    }
    __syncthreads();
    const double b1 = sv[0], b2 = sv[1];
    // a wave per column pair, lanes over agents: w = H2 e_k, then
    // w -= b1 v1 (v1^H w) with the dot product as a wave sum
    const int lane = tid & 63, wv = tid >> 6;
    for (int k = 2 + wv; k < n; k += kT / 64) {
      double* u = Q + (size_t)(2 * (k - 2)) * np;       // emb(w)
      double* ui = u + np;                              // emb(i w)
      // H2 e_k = e_k - b2 v2 conj(v2_k)
      const double cr = v2[2 * k], ci = -v2[2 * k + 1];
      auto h2 = [&](int i, double& wr, double& wi) {
        const double vr = v2[2 * i], vi = v2[2 * i + 1];
        wr = (i == k ? 1.0 : 0.0) - b2 * (vr * cr - vi * ci);
        wi = -b2 * (vr * ci + vi * cr);
      };
      double dr = 0.0, di = 0.0;
      for (int i = lane; i < n; i += 64) {
        double wr, wi;
        h2(i, wr, wi);
        const double vr = v1[2 * i], vi = v1[2 * i + 1];
        dr += vr * wr + vi * wi;
        di += vr * wi - vi * wr;
      }
      for (int o = 32; o > 0; o >>= 1) {
        dr += __shfl_xor(dr, o, 64);
        di += __shfl_xor(di, o, 64);
      }
      for (int i = lane; i < n; i += 64) {
        double wr, wi;
        h2(i, wr, wi);
        const double vr = v1[2 * i], vi = v1[2 * i + 1];
        const double xr = wr - b1 * (vr * dr - vi * di);
        const double xi = wi - b1 * (vr * di + vi * dr);
        u[2 * i] = xr; u[2 * i + 1] = xi;
        ui[2 * i] = -xi; ui[2 * i + 1] = xr;
      }
    }
  } else {
  if (tid == 0) {
    for (int q = 0; q < max(nct, nrt); ++q) {
      bool apply = false;
      double* Aq = A + (size_t)q * np;
      if (q < nct) {
        const double nrm = nrm2_seq(Aq + q, np - q, 1);
        if (nrm > 0.0) {
          apply = true;
          const double r = Aq[q] < 0.0 ? -nrm : nrm;
          if (fabs(r) >= kTiny) {
            const double rr = 1.0 / r;
            for (int i = q; i < np; ++i) Aq[i] *= rr;
          } else {
            for (int i = q; i < np; ++i) Aq[i] /= r;
          }
          Aq[q] += 1.0;
          sv[q] = -r;
        } else {
          sv[q] = 0.0;
        }
      }
      for (int jj = q + 1; jj < p; ++jj) {
        double* Aj = A + (size_t)jj * np;
        if (apply) {
          double d = 0.0;
          for (int i = q; i < np; ++i) d += Aq[i] * Aj[i];
          const double t = -(d / Aq[q]);
          if (t != 0.0)
            for (int i = q; i < np; ++i) Aj[i] += t * Aq[i];
        }
        ev[jj] = Aj[q];
      }
      if (q < nrt) {
        const int len = p - q - 1;
        const double nrm = len > 1 ? nrm2_seq(ev + q + 1, len, 1) : fabs(ev[q + 1]);
        if (nrm == 0.0) {
          ev[q] = 0.0;
        } else {
          ev[q] = ev[q + 1] < 0.0 ? -nrm : nrm;
          if (fabs(ev[q]) >= kTiny) {
            const double rr = 1.0 / ev[q];
            for (int k = q + 1; k < p; ++k) ev[k] *= rr;
          } else {
            for (int k = q + 1; k < p; ++k) ev[k] /= ev[q];
          }
          ev[q + 1] += 1.0;
          ev[q] = -ev[q];
          if (q + 2 <= np) {
            for (int i = q + 1; i < np; ++i) work[i] = 0.0;
            for (int jj = q + 1; jj < p; ++jj)
              if (ev[jj] != 0.0)
                for (int i = q + 1; i < np; ++i) work[i] += ev[jj] * A[(size_t)jj * np + i];
            for (int jj = q + 1; jj < p; ++jj) {
              const double a = -ev[jj] / ev[q + 1];
              if (a != 0.0)
                for (int i = q + 1; i < np; ++i) A[(size_t)jj * np + i] += a * work[i];
            }
          }
        }
      }
    }
  }
  __syncthreads();
  // U(:, p:np) = H_0 ... H_{nct-1} e_jj; U(q:, q) is A(q:, q) after step q
  // (later steps never touch column q). A wave per column, each element on
  // one lane throughout (i = lane + 64 m), the reflector dot products as wave
  // sums (the factorisation above, whose rounding decides the reflectors'
  // signs, keeps the codegen's serial order).
  {
    const int lane = tid & 63, wv = tid >> 6;
    for (int jj = p + wv; jj < np; jj += kT / 64) {
      double* u = Q + (size_t)(jj - p) * np;
      for (int i = lane; i < np; i += 64) u[i] = (i == jj) ? 1.0 : 0.0;
      for (int q = nct - 1; q >= 0; --q) {
        if (sv[q] == 0.0) continue;
        const double* h = A + (size_t)q * np;
        double d = 0.0;
        for (int i = lane; i < np; i += 64)
          if (i >= q) d += h[i] * u[i];
        for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
        const double t = -(d / h[q]);
        if (t != 0.0)
          for (int i = lane; i < np; i += 64)
            if (i >= q) u[i] += t * h[i];
      }
    }
  }
  }
  __syncthreads();
  if (!xy) {
    // rows of Q that are numerically zero drop their graph rows (3D.m:85-90)
    for (int r = tid; r < np; r += kT) {
      double a = 0.0;
      for (int j = 0; j < s; ++j) a += fabs(Q[r + (size_t)j * np]);
      zro[r] = a < 100.0 * 2.220446049250313e-16;
    }
    __syncthreads();
  }
  // graph rows: per-column counts, prefix, then each column writes its rows
  int* cnt = zro + np;  // n + 1
  const double* Ad = adj + (size_t)f * n * n;
  for (int j = tid; j < n; j += kT) {
    int c = 0;
    if (xy || !zro[j])
      for (int i = 0; i < j; ++i)
        if (Ad[i + (size_t)j * n] == 0.0 && (xy || !zro[i])) c += xy ? 2 : 1;
    cnt[j + 1] = c;
  }
  __syncthreads();
  if (tid == 0) {
    cnt[0] = 0;
    for (int j = 0; j < n; ++j) cnt[j + 1] += cnt[j];
    Info in;
    in.np = np; in.s = s; in.K = cnt[n]; in.st = xy ? 1 : 0;
    info[part] = in;
  }
  __syncthreads();
  unsigned short* pr = pairbuf + (size_t)part * pstride;
  for (int j = tid; j < n; j += kT) {
    int K = cnt[j];
    if (!(xy || !zro[j])) continue;
    for (int i = 0; i < j; ++i) {
      if (Ad[i + (size_t)j * n] != 0.0 || !(xy || !zro[i])) continue;
      if (xy) {
        if (K + 2 <= kMaxRows) {
          pr[2 * K] = (unsigned short)(2 * i); pr[2 * K + 1] = (unsigned short)(2 * j);
          pr[2 * K + 2] = (unsigned short)(2 * i + 1); pr[2 * K + 3] = (unsigned short)(2 * j);
        }
        K += 2;
      } else {
        if (K + 1 <= kMaxRows) {
          pr[2 * K] = (unsigned short)i; pr[2 * K + 1] = (unsigned short)j;
        }
        K += 1;
      }
    }
  }
}

// Qa = rows a_k of Q, Qb = rows b_k (K x s, ld K)
__global__ void __launch_bounds__(kT) gather_kernel(const Part* parts) {
  const Part& P = parts[blockIdx.y];
  const int K = P.K, s = P.s;
  for (int e = blockIdx.x * kT + threadIdx.x; e < K * s; e += gridDim.x * kT) {
    const int k = e % K, j = e / K;
    P.Qa[e] = P.Q[P.pa[2 * k] + (size_t)j * P.np];
    P.Qb[e] = P.Q[P.pa[2 * k + 1] + (size_t)j * P.np];
  }
}

// Gram matrix of {I, H_k} in the X22 space (admm_oracle.Part.__init__):
// structured: 2 Re(Psi_ac Psi_db + Psi_ad Psi_cb + Psi_bc Psi_da + Psi_bd Psi_ca)/16
// with Psi = Qc Qc^H (Qc = complexified rows of Q), plain: (G_ac G_bd + G_ad G_bc)/2.
__global__ void __launch_bounds__(kT) gamma_kernel(const Part* parts) {
  const Part& P = parts[blockIdx.y];
  const int K1 = P.K + 1, np = P.np;
  for (int e = blockIdx.x * kT + threadIdx.x; e < K1 * K1; e += gridDim.x * kT) {
    const int r = e % K1, c = e / K1;
    double v;
    if (r == 0 && c == 0) {
      v = (double)P.s;
    } else if (r == 0 || c == 0) {
      const int k = (r == 0 ? c : r) - 1;
      v = P.G[P.pa[2 * k] + (size_t)P.pa[2 * k + 1] * np];
    } else {
      const int a = P.pa[2 * (r - 1)], b = P.pa[2 * (r - 1) + 1];
      const int cc = P.pa[2 * (c - 1)], d = P.pa[2 * (c - 1) + 1];
      if (P.st) {
        auto re = [&](int x, int y) { return P.Pre[x + (size_t)y * np]; };
        auto im = [&](int x, int y) { return P.Pim[x + (size_t)y * np]; };
        auto cm = [&](int x1, int y1, int x2, int y2) {
          return re(x1, y1) * re(x2, y2) - im(x1, y1) * im(x2, y2);
        };
        const double t = cm(a, cc, d, b) + cm(a, d, cc, b) + cm(b, cc, d, a) + cm(b, d, cc, a);
        v = 2.0 * t / 16.0;
      } else {
        auto g = [&](int x, int y) { return P.G[x + (size_t)y * np]; };
        v = 0.5 * (g(a, cc) * g(b, d) + g(a, d) * g(b, cc));
      }
    }
    P.Gam[e] = v;
  }
}

// Pivoted Cholesky of Gamma (rows whose Schur pivot is <= 1e-10 of their
// diagonal are dependent graph rows and dropped, as admm_oracle's
// _pivoted_cholesky), then Li = L^-1 on the kept rows (zero elsewhere), so
// Ginv = Li' Li is the solve the codegen's LU/QR performs (sparse.cpp:735-741).
__global__ void __launch_bounds__(kT) chol_kernel(const Part* parts) {
  const Part& P = parts[blockIdx.x];
  const int K1 = P.K + 1;
  const int tid = threadIdx.x;
  __shared__ double d0[kMaxRows + 1];
  __shared__ unsigned char keep[kMaxRows + 1];
  __shared__ int s_keep;
  double* L = P.Li;  // factor in place (lower)
  for (int e = tid; e < K1 * K1; e += kT) L[e] = P.Gam[e];
  for (int k = tid; k < K1; k += kT) d0[k] = P.Gam[k + (size_t)k * K1];
  __syncthreads();
  for (int k = 0; k < K1; ++k) {
    if (tid == 0) {
      const double d = L[k + (size_t)k * K1];
      s_keep = d > 1e-10 * d0[k];
      keep[k] = (unsigned char)s_keep;
      if (s_keep) L[k + (size_t)k * K1] = sqrt(d);
    }
    __syncthreads();
    const bool kp = s_keep;
    const double piv = L[k + (size_t)k * K1];
    for (int i = k + 1 + tid; i < K1; i += kT) {
      double& x = L[i + (size_t)k * K1];
      x = kp ? x / piv : 0.0;
    }
    if (!kp && tid == 0) L[k + (size_t)k * K1] = 0.0;
    __syncthreads();
    if (kp) {
      // trailing update, every (i, j), k < j <= i, in one parallel pass (each
      // element still takes its updates in k order: the same roundings as a
      // column-by-column sweep, without its K1^2 / 2 serial steps)
      const int m = K1 - k - 1;
      for (int e = tid; e < m * m; e += kT) {
        const int jj = e / m, ii = e - jj * m;
        if (ii < jj) continue;
        const int j = k + 1 + jj, i = k + 1 + ii;
        const double ljk = L[j + (size_t)k * K1];
        if (ljk == 0.0) continue;
        L[i + (size_t)j * K1] -= L[i + (size_t)k * K1] * ljk;
      }
    }
    __syncthreads();
  }
  // forward substitution, one column of L^-1 per thread (into Gam)
  for (int c = tid; c < K1; c += kT) {
    double* x = P.Gam + (size_t)c * K1;
    for (int i = 0; i < K1; ++i) {
      if (i < c || !keep[c] || !keep[i]) {
        x[i] = 0.0;
        continue;
      }
      double acc = (i == c) ? 1.0 : 0.0;
      for (int m = c; m < i; ++m) acc -= L[i + (size_t)m * K1] * x[m];
      x[i] = acc / L[i + (size_t)i * K1];
    }
  }
}

// chol_kernel with the factor in LDS as a packed lower triangle (column j,
// rows j..K1-1, at pk(j) - j + i), for systems whose triangle fits
// (chol_lds_bytes <= 160 KiB: K1 <= 198). Every element takes the same
// operations in the same order as in chol_kernel (pivot test, scale, the
// trailing updates in k order, each row's substitution sum in m order), so
// L^-1 is bit-identical. One barrier per column step: every wave takes the
// pivot and the scaled column k itself (lanes over rows, in registers) and
// wave 0 stores column k one step late (no later step reads it). The
// substitution: a wave per column of L^-1, lanes over its rows, the running
// sums in registers (no round trips through the global column).
constexpr int kCholT = 512;
constexpr int kCholRows = 4;  // rows per lane: K1 <= 256
inline size_t chol_lds_bytes(int K1) {
  return ((size_t)K1 * (K1 + 1) / 2 + (size_t)K1) * sizeof(double) + (size_t)K1 + 16;
}
constexpr size_t kCholLdsMax = 160 * 1024;
// the register columns hold 64 kCholRows rows: every K1 the LDS budget admits
// must fit them (a larger budget needs more rows per lane, or rows past
// 64 kCholRows would be skipped silently)
static_assert(((size_t)64 * kCholRows + 1) * (64 * kCholRows + 2) / 2 * sizeof(double) > kCholLdsMax,
              "chol_lds_kernel: the LDS budget admits K1 > 64 * kCholRows");
inline bool chol_lds_fits(int K1) {
  return K1 <= 64 * kCholRows && chol_lds_bytes(K1) <= kCholLdsMax;
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__global__ void __launch_bounds__(kCholT) chol_lds_kernel(const Part* parts) {
  extern __shared__ double lsm[];
  const Part& P = parts[blockIdx.x];
  const int K1 = P.K + 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int kW = kCholT / 64;
  double* Lp = lsm;
  double* d0 = Lp + (size_t)K1 * (K1 + 1) / 2;
  unsigned char* keep = reinterpret_cast<unsigned char*>(d0 + K1);
  // column j of L: col(j)[i] = L[i, j], i >= j
  auto col = [&](int j) { return Lp + ((size_t)j * K1 - (size_t)j * (j - 1) / 2) - j; };
  for (int j = wave; j < K1; j += kW) {
    const double* g = P.Gam + (size_t)j * K1;
    double* c = col(j);
    for (int i = j + lane; i < K1; i += 64) c[i] = g[i];
  }
  for (int k = tid; k < K1; k += kCholT) d0[k] = P.Gam[k + (size_t)k * K1];
  __syncthreads();
  double lk[kCholRows];    // scaled column k, rows k + 1 + lane + 64 t
  double piv = 0.0;
  bool kp = false;
  for (int k = 0; k < K1; ++k) {
    if (wave == 0 && k > 0) {  // column k - 1, held since the last step
      double* cp = col(k - 1);
      if (lane == 0) cp[k - 1] = kp ? piv : 0.0;
#pragma unroll
      for (int t = 0; t < kCholRows; ++t) {
        const int i = k + lane + 64 * t;
        if (i < K1) cp[i] = lk[t];
      }
    }
    const double* ck = col(k);
    const double d = ck[k];
    kp = d > 1e-10 * d0[k];
    piv = kp ? sqrt(d) : 0.0;
    if (tid == 0) keep[k] = (unsigned char)kp;
#pragma unroll
    for (int t = 0; t < kCholRows; ++t) {
      const int i = k + 1 + lane + 64 * t;
      lk[t] = (i < K1 && kp) ? ck[i] / piv : 0.0;
    }
    if (kp) {
      for (int j = k + 1 + wave; j < K1; j += kW) {
        const int r = j - k - 1;  // row j's lane and slot
        double v = lk[0];
#pragma unroll
        for (int t = 1; t < kCholRows; ++t) v = (r >> 6) == t ? lk[t] : v;
        const double ljk = readlane_f64(v, r & 63);
        if (ljk == 0.0) continue;
        double* cj = col(j);
#pragma unroll
        for (int t = 0; t < kCholRows; ++t) {
          const int i = k + 1 + lane + 64 * t;
          if (i >= j && i < K1) cj[i] -= lk[t] * ljk;
        }
      }
    }
    __syncthreads();
  }
  if (wave == 0) {  // the last column
    double* cp = col(K1 - 1);
    if (lane == 0) cp[K1 - 1] = kp ? piv : 0.0;
  }
  __syncthreads();
  // L^-1 column c: x_i = (delta_ic - sum_{m=c}^{i-1} L[i, m] x_m) / L[i, i]
  // (0 above c, in dropped rows and for a dropped c), rows i = lane + 64 t
  for (int c = wave; c < K1; c += kW) {
    double x[kCholRows];
#pragma unroll
    for (int t = 0; t < kCholRows; ++t) x[t] = (lane + 64 * t == c) ? 1.0 : 0.0;
    const bool kc = keep[c];
    if (kc) {
      for (int m = c; m < K1; ++m) {
        const int tm = m >> 6, lm = m & 63;
        double a = x[0];
#pragma unroll
        for (int t = 1; t < kCholRows; ++t) a = tm == t ? x[t] : a;
        const double* cm = col(m);
        const double xm = readlane_f64(keep[m] ? a / cm[m] : 0.0, lm);
#pragma unroll
        for (int t = 0; t < kCholRows; ++t) {
          const int i = lane + 64 * t;
          if (i == m) x[t] = xm;
          else if (i > m && i < K1) x[t] -= cm[i] * xm;
        }
      }
    }
    double* g = P.Gam + (size_t)c * K1;
#pragma unroll
    for (int t = 0; t < kCholRows; ++t) {
      const int i = lane + 64 * t;
      if (i < K1) g[i] = (kc && i >= c) ? x[t] : 0.0;
    }
  }
}

// P_struct of a 2m x 2m block: element (i, j) of the projection of M onto
// [a b; -b a] blocks (ADMMGainDesign2D.m:221-265).
template <typename F>
__device__ __forceinline__ double pstruct_at(int st, int i, int j, F M) {
  if (!st) return M(i, j);
  const int I = i & ~1, Jb = j & ~1;
  if ((i & 1) == (j & 1)) return 0.5 * (M(I, Jb) + M(I + 1, Jb + 1));
  const double b = 0.5 * (M(I, Jb + 1) - M(I + 1, Jb));
  return (i & 1) ? -b : b;
}

// Pm = P_struct(M22), M22 = aS S22 + aX X22 (iteration: aS = -1, aX = -mu;
// final projection: aS = 0, aX = 1).
__global__ void __launch_bounds__(kT) pm_kernel(const Part* parts, double aS, double aX,
                                                int only_active) {
  const Part& P = parts[blockIdx.y];
  if (only_active && !P.sc->active) return;
  const int s = P.s, n2 = 2 * s;
  auto M = [&](int i, int j) {
    const size_t e = (size_t)(s + i) + (size_t)(s + j) * n2;
    return (aS != 0.0 ? aS * P.S[e] : 0.0) + aX * P.X[e];
  };
  for (int e = blockIdx.x * kT + threadIdx.x; e < s * s; e += gridDim.x * kT) {
    const int i = e % s, j = e / s;
    P.Pm[e] = pstruct_at(P.st, i, j, M);
  }
}

__device__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += red[k];
  return t;  // valid in thread 0
}

// r_0 = tr M22, r_k = q_a' Pm q_b = (Qa Pm)_k . Qb_k;  c = Ginv r;
// Qbc = diag(c_1..K) Qb; also tr M11 (iteration mode).
// mode 0: hb (r = s e_0), 1: iteration, 2: final projection.
__global__ void __launch_bounds__(kT) rc_kernel(const Part* parts, int mode, double mu) {
  const Part& P = parts[blockIdx.x];
  if (mode == 1 && !P.sc->active) return;
  const int s = P.s, n2 = 2 * s, K = P.K, K1 = K + 1;
  const int tid = threadIdx.x;
  __shared__ double red[kT / 64];
  __shared__ double rr[kMaxRows + 1];
  __shared__ double cc[kMaxRows + 1];
  double t11 = 0.0, t22 = 0.0;
  if (mode != 0) {
    for (int i = tid; i < s; i += kT) {
      const size_t d1 = (size_t)i * (n2 + 1), d2 = (size_t)(s + i) * (n2 + 1);
      if (mode == 1) {
        t11 += 1.0 - P.S[d1] - mu * P.X[d1];
        t22 += -P.S[d2] - mu * P.X[d2];
      } else {
        t22 += P.X[d2];
      }
    }
  }
  const double T11 = block_sum(t11, red);
  const double T22 = block_sum(t22, red);
  if (tid == 0) {
    rr[0] = (mode == 0) ? (double)s : T22;
    if (mode == 1) P.sc->trM11 = T11;
  }
  // the row dot products and the Ginv product as kAcc interleaved partial
  // sums (independent load chains; added in a fixed order: deterministic)
  constexpr int kAcc = 8;
  for (int k = tid; k < K; k += kT) {
    double a = 0.0;
    if (mode != 0) {
      double pa[kAcc] = {};
      int j = 0;
      for (; j + kAcc <= s; j += kAcc)
#pragma unroll
        for (int u = 0; u < kAcc; ++u)
          pa[u] += P.Yk[k + (size_t)(j + u) * K] * P.Qb[k + (size_t)(j + u) * K];
      for (; j < s; ++j) pa[0] += P.Yk[k + (size_t)j * K] * P.Qb[k + (size_t)j * K];
#pragma unroll
      for (int u = 0; u < kAcc; ++u) a += pa[u];
    }
    rr[k + 1] = a;
  }
  __syncthreads();
  for (int i = tid; i < K1; i += kT) {
    double pa[kAcc] = {};
    int m = 0;
    for (; m + kAcc <= K1; m += kAcc)
#pragma unroll
      for (int u = 0; u < kAcc; ++u) pa[u] += P.Ginv[i + (size_t)(m + u) * K1] * rr[m + u];
    for (; m < K1; ++m) pa[0] += P.Ginv[i + (size_t)m * K1] * rr[m];
    double a = 0.0;
#pragma unroll
    for (int u = 0; u < kAcc; ++u) a += pa[u];
    P.c[i] = a;
    cc[i] = a;
  }
  __syncthreads();
  for (int e = tid; e < K * s; e += kT) P.Qbc[e] = cc[1 + e % K] * P.Qb[e];
  if (tid == 0) P.sc->c0 = cc[0];
}

// combine(c) at (i, j) = c0 delta_ij + P_struct(sym(T))(i, j)
__device__ __forceinline__ double combine_at(const Part& P, double c0, int i, int j) {
  const int s = P.s;
  auto sym = [&](int x, int y) { return 0.5 * (P.T[x + (size_t)y * s] + P.T[y + (size_t)x * s]); };
  return (i == j ? c0 : 0.0) + pstruct_at(P.st, i, j, sym);
}

// hb = combine(Ginv s e_0) (minimum-norm point of the affine X22 constraints)
// and the ADMM start: X = [I I; I I], S = 0 (2D.m:420-430).
__global__ void __launch_bounds__(kT) init_kernel(const Part* parts) {
  const Part& P = parts[blockIdx.y];
  const int s = P.s, n2 = 2 * s;
  const double c0 = P.c[0];
  for (int e = blockIdx.x * kT + threadIdx.x; e < n2 * n2; e += gridDim.x * kT) {
    const int i = e % n2, j = e / n2;
    if (i < s && j < s) P.hb[i + (size_t)j * s] = combine_at(P, c0, i, j);
    P.X[e] = (i % s == j % s) ? 1.0 : 0.0;
    P.S[e] = 0.0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    Scal z = {};
    z.active = 1;
    *P.sc = z;
  }
}

// W = sym(S + (I-P)(C - S - mu X) - mu x_b) (admm_oracle.Part.run), element
// (i, j) before the sym. raw(j, i) == raw(i, j) bit for bit: S, Pm, hb and
// combine are symmetric element for element (each is built from symmetric
// operands by the same operations in the same order, or as 0.5 (a + b) of a
// transposed pair), so sym(raw) = 0.5 (x + x) = x exactly.
__device__ __forceinline__ double w_raw(const Part& P, double trs, double c0, double mu, int i,
                                        int j) {
  const int s = P.s, n2 = 2 * s;
  double w = P.S[i + (size_t)j * n2];
  if (i < s && j < s) {
    if (i == j) w += trs;
  } else if (i >= s && j >= s) {
    const int a = i - s, b = j - s;
    w += P.Pm[a + (size_t)b * s] - combine_at(P, c0, a, b) - mu * P.hb[a + (size_t)b * s];
  } else if (i % s == j % s) {
    w -= mu;
  }
  return w;
}

// W by 32 x 32 blocks of the upper triangle (W symmetric element for element,
// above): the block's raw values, the mirror block through LDS (coalesced),
// and the column sums of |W - eps I| for norm_kernel as per-block-row
// partials cs[b n2 + j] (block row b = rows 32 b .. 32 b + 31; a block off
// the diagonal also gives its mirror's, from its row sums), which
// norm_kernel adds in block order (deterministic).
constexpr int kWB = 32;
__global__ void __launch_bounds__(256) w_ut_kernel(const Part* parts, double mu, double eps) {
  const Part& P = parts[blockIdx.y];
  if (!P.sc->active) return;
  const int s = P.s, n2 = 2 * s;
  const int nb = (n2 + kWB - 1) / kWB;
  int t = blockIdx.x;
  if (t >= nb * (nb + 1) / 2) return;
  int bj = 0;
  while (t > bj) { t -= bj + 1; ++bj; }
  const int bi = t;
  const int i0 = bi * kWB, j0 = bj * kWB;
  const bool dgb = bi == bj;
  const double trs = P.sc->trM11 / s, c0 = P.sc->c0;
  __shared__ double tw[kWB][kWB + 1];
  __shared__ double rs[8][kWB];
  const int tid = threadIdx.x, li = tid & 31, lg = tid >> 5;
  double rsum = 0.0;  // this thread's part of row i0 + li (the mirror's column)
#pragma unroll
  for (int m = 0; m < kWB / 8; ++m) {
    const int c = lg + 8 * m, i = i0 + li, j = j0 + c;
    double av = 0.0;
    if (i < n2 && j < n2) {
      const double w = w_raw(P, trs, c0, mu, i, j);
      P.W[i + (size_t)j * n2] = w;
      tw[c][li] = w;
      av = fabs(w - (i == j ? eps : 0.0));
    }
    rsum += av;
    // column j0 + c over the block's 32 rows: the half-wave's lanes (li)
    double cv = av;
    for (int o = 16; o > 0; o >>= 1) cv += __shfl_xor(cv, o, 32);
    if (li == 0 && j < n2) P.cs[(size_t)bi * n2 + j] = cv;
  }
  if (!dgb) {  // workgroup-uniform
    rs[lg][li] = rsum;
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kWB / 8; ++m) {
      const int c = lg + 8 * m, j = j0 + li, i = i0 + c;
      if (j < n2 && i < n2) P.W[j + (size_t)i * n2] = tw[li][c];
    }
    if (lg == 0 && i0 + li < n2) {
      double a = 0.0;
#pragma unroll
      for (int g = 0; g < 8; ++g) a += rs[g][li];
      P.cs[(size_t)bj * n2 + i0 + li] = a;  // mirror: row block bj, column i0 + li
    }
  }
}

// |W - eps I|_inf (= |.|_1, W symmetric: contiguous column sums); resets the
// Newton-Schulz state of active parts.
__global__ void __launch_bounds__(kT) norm_kernel(const Part* parts, double eps) {
  const Part& P = parts[blockIdx.x];
  Scal& sc = *P.sc;
  if (!sc.active) {
    if (threadIdx.x == 0) { sc.ns_done = 1; sc.inactive = 1; }
    return;
  }
  const int n2 = 2 * P.s;
  __shared__ double red[kT / 64];
  double mx = 0.0;
  for (int j = threadIdx.x; j < n2; j += kT) {
    double a = 0.0;
    if (P.cs) {  // per-block-row partials left by w_ut_kernel, in block order
      const int nbw = (n2 + kWB - 1) / kWB;
      for (int b = 0; b < nbw; ++b) a += P.cs[(size_t)b * n2 + j];
    } else {
      const double* col = P.W + (size_t)j * n2;
      for (int i = 0; i < n2; ++i) a += fabs(col[i] - (i == j ? eps : 0.0));
    }
    mx = fmax(mx, a);
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_down(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = 0.0;
    for (int k = 0; k < kT / 64; ++k) m = fmax(m, red[k]);
    // Z0 = (W - eps I) / (|.|_inf / kNsScale): the spectral radius is at most
    // the inf-norm, so every |eigenvalue| of Z0 is <= kNsScale < sqrt(3) and
    // Newton-Schulz converges; measured on the C5 designs the spectrum lies in
    // [0.37, 1] of the radius and the radius at 0.67-0.75 of the inf-norm, so
    // kNsScale = 1.5 starts the eigenvalues nearer 1 (about 20% fewer steps)
    sc.nrm = m > 0.0 ? m / kNsScale : 1.0;
    sc.ns_done = 0; sc.ns_final = 0; sc.ns_upd = 0; sc.inactive = 0; sc.ns_fail_now = 0;
  }
}

// N0 = (W - eps I) / |W - eps I|_inf
__global__ void __launch_bounds__(kT) nsinit_kernel(const Part* parts, double eps) {
  const Part& P = parts[blockIdx.y];
  if (!P.sc->active) return;
  const int n2 = 2 * P.s;
  const double inv = 1.0 / P.sc->nrm;
  for (int e = blockIdx.x * kT + threadIdx.x; e < n2 * n2; e += gridDim.x * kT) {
    const int i = e % n2, j = e / n2;
    P.N0[e] = (P.W[e] - (i == j ? eps : 0.0)) * inv;
  }
}

// |Z^2 - I|_F^2 -> ns_final when converged (the update that follows is the last)
__global__ void __launch_bounds__(kT) nserr_kernel(const Part* parts) {
  const Part& P = parts[blockIdx.y];
  Scal& sc = *P.sc;
  if (sc.ns_done) return;
  const int n2 = 2 * P.s;
  __shared__ double red[kT / 64];
  double a = 0.0;
  for (int e = blockIdx.x * kT + threadIdx.x; e < n2 * n2; e += gridDim.x * kT) {
    const int i = e % n2, j = e / n2;
    const double d = P.Y[e] - (i == j ? 1.0 : 0.0);
    a += d * d;
  }
  const double t = block_sum(a, red);
  if (threadIdx.x == 0) atomicAdd(&sc.err2, t);
}

// after the update GEMM: count it, finish converged parts, count the rest
// remaining[0]: parts still iterating; remaining[2]: active parts whose sign
// iteration failed (the host skips psd_jacobi_kernel when none did)
__global__ void __launch_bounds__(1024) nsstep_kernel(const Part* parts, int nparts, int last,
                                                      double tol, int* remaining) {
  __shared__ int cnt, fails;
  if (threadIdx.x == 0) { cnt = 0; fails = 0; }
  __syncthreads();
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) {
    Scal& sc = *parts[p].sc;
    if (sc.ns_done) {
      if (!sc.inactive && sc.ns_fail_now) atomicAdd(&fails, 1);
      continue;
    }
    sc.ns_upd += 1;
    const int n2 = 2 * parts[p].s;
    if (sc.err2 < tol * n2 || sc.ns_upd >= kNsMax || !(sc.err2 == sc.err2)) {
      sc.ns_done = 1;
      if (!(sc.err2 < tol * n2)) sc.ns_fail_now = 1;
    } else if (last) {
      sc.ns_done = 1;
      sc.ns_fail_now = 1;
    }
    sc.err2 = 0.0;
    if (!sc.ns_done) atomicAdd(&cnt, 1);
    else if (sc.ns_fail_now) atomicAdd(&fails, 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) { remaining[0] = cnt; remaining[2] = fails; }
}

// the sign lives in N0 after an even number of updates, N1 after an odd one:
// the S product of each part reads the one that holds it (two job lists,
// each skipping the other parity's parts) instead of a copy N1 -> N0
__global__ void __launch_bounds__(1024) nsparity_kernel(const Part* parts, int nparts) {
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) {
    Scal& sc = *parts[p].sc;
    const int odd = sc.ns_upd & 1;
    const int skip = !sc.active || sc.ns_fail_now;  // no sign: psd_jacobi_kernel writes Sr
    sc.skip_s0 = (skip || odd) ? 1 : 0;
    sc.skip_s1 = (skip || !odd) ? 1 : 0;
  }
}

// test hook (acl_internal_psd_project): every active part takes the fallback
__global__ void __launch_bounds__(1024) force_jacobi_kernel(const Part* parts, int nparts) {
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) parts[p].sc->ns_fail_now = 1;
}

// ---------------------------------------------------------------------------
// PSD projection fallback: S = sum over lambda > eps of lambda v v^T from a
// parallel two-sided Jacobi eigensolver (one workgroup per part), for the
// parts whose Newton-Schulz sign iteration did not converge in kNsMax steps:
// an eigenvalue of W at (or within ~1e-11 |W| of) eps, where sign(W - eps I)
// is ill-conditioned. The reference decides that projection with its
// eigensolver (admm::Solver: SelfAdjointEigenSolver, solver.cpp:296-316; the
// codegen: eig -> schur, eig.cpp:24, ADMMGainDesign2D.m:430-445); so does
// this, eigenvalue by eigenvalue.
//
// Pairing: the circle method. In step t (0 .. N-2) index 0 meets 1 + t and,
// for k = 1 .. N/2 - 1, 1 + (t + k) % (N - 1) meets 1 + (t - k) % (N - 1);
// the N/2 rotations of a step are disjoint, so A <- J^T A J is one pass over
// the 2 x 2 blocks (block (k, l) <- R_k^T A_kl R_l for k <= l, mirrored: A
// stays symmetric bit for bit) and V <- V J one pass over V's column pairs.
// Rotation (Golub & Van Loan, sym.schur2): tau = (a_qq - a_pp) / (2 a_pq),
// t = sign(tau) / (|tau| + sqrt(1 + tau^2)), c = 1 / sqrt(1 + t^2), s = t c.
// Sweeps until the off-diagonal mass is below (1e-15 |A|_F)^2 (at most
// kJacobiSweeps). Workspace: A in N0, V in N1; the result goes to Sr, full
// and symmetric, where the S product would have put it.
constexpr int kJT = 1024;
constexpr int kJacobiSweeps = 40;

__device__ __forceinline__ double block_sum_all(double v, double* red) {
  const double t = block_sum(v, red);
  __syncthreads();
  if (threadIdx.x == 0) red[0] = t;
  __syncthreads();
  const double r = red[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(kJT) psd_jacobi_kernel(const Part* parts, double eps) {
  const Part& P = parts[blockIdx.x];
  Scal& sc = *P.sc;
  if (!sc.active || !sc.ns_fail_now) return;
  const int N = 2 * P.s, m = N / 2, N1 = N - 1;
  extern __shared__ __attribute__((aligned(16))) double jsm[];
  double* cs = jsm;                                  // [m][2] c, s
  double* lam = jsm + 2 * m;                         // [N] eigenvalues kept (> eps), else 0
  int* pq = reinterpret_cast<int*>(jsm + 2 * m + N); // [m][2] the step's pairs
  __shared__ double red[kJT / 64];
  double* A = P.N0;
  double* V = P.N1;
  const int tid = threadIdx.x;
  double fro = 0.0;
  for (int e = tid; e < N * N; e += kJT) {
    const double w = P.W[e];
    A[e] = w;
    V[e] = (e % N == e / N) ? 1.0 : 0.0;
    fro += w * w;
  }
  const double tol = 1e-30 * block_sum_all(fro, red);  // (1e-15 |A|_F)^2
  __syncthreads();
  bool conv = false;
  for (int sweep = 0; sweep <= kJacobiSweeps; ++sweep) {
    double off = 0.0;
    for (int e = tid; e < N * N; e += kJT) {
      const int i = e % N, j = e / N;
      if (i != j) off += A[e] * A[e];
    }
    const double o = block_sum_all(off, red);
    if (!(o > tol)) {              // (NaN: stop, the result is NaN -- not converged)
      conv = o == o;
      break;
    }
    if (sweep == kJacobiSweeps) break;   // off-diagonal mass left: reported below
    for (int t = 0; t < N1; ++t) {
      for (int k = tid; k < m; k += kJT) {
        int p, q;
        if (k == 0) { p = 0; q = 1 + t; }
        else { p = 1 + (t + k) % N1; q = 1 + (t - k + N1) % N1; }
        const double app = A[p + (size_t)p * N], aqq = A[q + (size_t)q * N];
        const double apq = A[p + (size_t)q * N];
        double c = 1.0, sn = 0.0;
        if (apq != 0.0) {
          const double tau = (aqq - app) / (2.0 * apq);
          const double tt = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
          c = 1.0 / sqrt(1.0 + tt * tt);
          sn = tt * c;
        }
        cs[2 * k] = c; cs[2 * k + 1] = sn;
        pq[2 * k] = p; pq[2 * k + 1] = q;
      }
      __syncthreads();
      // A <- J^T A J, block by block (k <= l)
      const int nblk = m * (m + 1) / 2;
      for (int bidx = tid; bidx < nblk; bidx += kJT) {
        // bidx -> (k, l), k <= l, row by row of the upper triangle
        int k = (int)((2.0 * m + 1.0 - sqrt((2.0 * m + 1.0) * (2.0 * m + 1.0) - 8.0 * bidx)) / 2.0);
        while (k > 0 && k * (2 * m - k + 1) / 2 > bidx) --k;
        while ((k + 1) * (2 * m - k) / 2 <= bidx) ++k;
        const int l = k + bidx - k * (2 * m - k + 1) / 2;
        const int pk = pq[2 * k], qk = pq[2 * k + 1], pl = pq[2 * l], ql = pq[2 * l + 1];
        const double ck = cs[2 * k], sk = cs[2 * k + 1], cl = cs[2 * l], sl = cs[2 * l + 1];
        const double x00 = A[pk + (size_t)pl * N], x01 = A[pk + (size_t)ql * N];
        const double x10 = A[qk + (size_t)pl * N], x11 = A[qk + (size_t)ql * N];
        // M = X R_l, Y = R_k^T M, R = [c s; -s c]
        const double m00 = cl * x00 - sl * x01, m01 = sl * x00 + cl * x01;
        const double m10 = cl * x10 - sl * x11, m11 = sl * x10 + cl * x11;
        double y00 = ck * m00 - sk * m10, y01 = ck * m01 - sk * m11;
        double y10 = sk * m00 + ck * m10, y11 = sk * m01 + ck * m11;
        if (k == l) {  // the annihilated entry
          y01 = 0.0;
          y10 = 0.0;
        }
        A[pk + (size_t)pl * N] = y00; A[pk + (size_t)ql * N] = y01;
        A[qk + (size_t)pl * N] = y10; A[qk + (size_t)ql * N] = y11;
        if (k != l) {
          A[pl + (size_t)pk * N] = y00; A[ql + (size_t)pk * N] = y01;
          A[pl + (size_t)qk * N] = y10; A[ql + (size_t)qk * N] = y11;
        }
      }
      // V <- V J: rows i, column pairs k
      for (int e = tid; e < N * m; e += kJT) {
        const int i = e % N, k = e / N;
        const int p = pq[2 * k], q = pq[2 * k + 1];
        const double c = cs[2 * k], sn = cs[2 * k + 1];
        const double vp = V[i + (size_t)p * N], vq = V[i + (size_t)q * N];
        V[i + (size_t)p * N] = c * vp - sn * vq;
        V[i + (size_t)q * N] = sn * vp + c * vq;
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < N; i += kJT) {
    const double l = A[i + (size_t)i * N];
    lam[i] = l > eps ? l : 0.0;  // the eigenvalues the projection keeps
  }
  __syncthreads();
  // Sr = V diag(lam) V^T, upper triangle computed, mirrored
  for (int e = tid; e < N * N; e += kJT) {
    const int i = e % N, j = e / N;
    if (i > j) continue;
    double a = 0.0;
    for (int k = 0; k < N; ++k)
      if (lam[k] != 0.0) a += V[i + (size_t)k * N] * lam[k] * V[j + (size_t)k * N];
    P.Sr[i + (size_t)j * N] = a;
    P.Sr[j + (size_t)i * N] = a;
  }
  if (tid == 0) {
    sc.jacobi += 1;
    if (!conv) sc.jacobi_fail += 1;
  }
}

// S = sym(Sr), Sr = (W + W sign)/2 from the S products (or the Jacobi
// fallback); X = (S - W)/mu; sum |X_old - X|, tr X22. A tile of the S
// products off the diagonal (tile size `tile`) is stored mirrored, so there
// sym(Sr) = Sr bit for bit; a diagonal tile's element is 0.5 (Sr_ij + Sr_ji).
// By 32 x 32 blocks of the upper triangle: Sr, W and X are symmetric element
// for element (the S products and the fallback store mirrored, W by
// construction, X = (S - W) / mu), so a block and its mirror share S, X and
// X_old: the block is read (Sr's mirror block too, through LDS, where it
// meets a diagonal tile) and S, X are written to both, the mirror through the
// LDS tile (coalesced); sum |dX| counts an off-diagonal pair twice.
// pmf: the block's elements of the X22 quadrant also give the next
// iteration's Pm = P_struct(M22), M22 = -S22 - mu X22 (pm_kernel's expression
// on the S, X just written, the same bits), so no pm launch re-reads S and X.
// A structured part's 2 x 2 groups (s even, the host checks) never straddle a
// 32-aligned block, and P_struct of the symmetric M22 is symmetric bit for bit
// (0.5 (x + y) of a mirrored pair; the odd terms negate as x - y = -(y - x)),
// so the mirror block gets the same values.
constexpr int kPB = 32;
__global__ void __launch_bounds__(256) post_ut_kernel(const Part* parts, double mu, int tile,
                                                      int pmf) {
  const Part& P = parts[blockIdx.y];
  if (!P.sc->active) return;
  const int s = P.s, n2 = 2 * s;
  const int nb = (n2 + kPB - 1) / kPB;
  int t = blockIdx.x;
  if (t >= nb * (nb + 1) / 2) return;
  int bj = 0;
  while (t > bj) { t -= bj + 1; ++bj; }
  const int bi = t;
  const int i0 = bi * kPB, j0 = bj * kPB;
  __shared__ double ts[kPB][kPB + 1];  // Sr mirror block, then S of the block
  __shared__ double tx[kPB][kPB + 1];  // X of the block
  __shared__ double red[4];
  const int tid = threadIdx.x, li = tid & 31, lg = tid >> 5;
  const bool dgb = bi == bj;
  const int ie = min(i0 + kPB, n2) - 1, je = min(j0 + kPB, n2) - 1;
  const bool meets = i0 / tile <= je / tile && j0 / tile <= ie / tile;
  if (meets) {  // ts[r][c] = Sr(j0 + r, i0 + c)
#pragma unroll
    for (int m = 0; m < kPB / 8; ++m) {
      const int c = lg + 8 * m, gr = j0 + li, gc = i0 + c;
      ts[li][c] = (gr < n2 && gc < n2) ? P.Sr[gr + (size_t)gc * n2] : 0.0;
    }
  }
  __syncthreads();
  const double imu = 1.0 / mu;
  double dsum = 0.0, tr = 0.0;
#pragma unroll
  for (int m = 0; m < kPB / 8; ++m) {
    const int c = lg + 8 * m, i = i0 + li, j = j0 + c;
    if (i < n2 && j < n2) {
      const size_t e = i + (size_t)j * n2;
      const double a = P.Sr[e];
      const double Sv = (i / tile != j / tile) ? a : 0.5 * (a + ts[c][li]);
      const double Xn = (Sv - P.W[e]) * imu;
      const double d = fabs(P.X[e] - Xn);
      if (dgb) {
        dsum += d;
        if (i == j && i >= s) tr += Xn;
      } else {
        dsum += 2.0 * d;
      }
      P.S[e] = Sv;
      P.X[e] = Xn;
      ts[c][li] = Sv;  // this thread's own slot (read above)
      tx[c][li] = Xn;
    }
  }
  // the block meets the X22 quadrant (workgroup-uniform)
  const bool pmb = pmf && i0 + kPB > s && j0 + kPB > s;
  if (!dgb || pmb) __syncthreads();
  if (!dgb) {  // workgroup-uniform: the mirror block, rows j coalesced
#pragma unroll
    for (int m = 0; m < kPB / 8; ++m) {
      const int c = lg + 8 * m, j = j0 + li, i = i0 + c;
      if (j < n2 && i < n2) {
        const size_t et = j + (size_t)i * n2;
        P.S[et] = ts[li][c];
        P.X[et] = tx[li][c];
      }
    }
  }
  if (pmb) {
    __shared__ double tp[kPB][kPB + 1];  // Pm of the block
    // M22 at block-local (row r, column c): pm_kernel's (-1 S) + (-mu X)
    auto Mv = [&](int r, int c) { return (-1.0 * ts[c][r]) + (-mu * tx[c][r]); };
#pragma unroll
    for (int m = 0; m < kPB / 8; ++m) {
      const int c = lg + 8 * m, i = i0 + li, j = j0 + c;
      if (i < n2 && j < n2 && i >= s && j >= s) {
        const int a = i - s, b = j - s;
        double v;
        if (!P.st) {
          v = Mv(li, c);
        } else {  // pstruct_at: the group's rows li - (a & 1) + {0, 1}, columns likewise
          const int r0 = li - (a & 1), c0 = c - (b & 1);
          if ((a & 1) == (b & 1)) {
            v = 0.5 * (Mv(r0, c0) + Mv(r0 + 1, c0 + 1));
          } else {
            const double bb = 0.5 * (Mv(r0, c0 + 1) - Mv(r0 + 1, c0));
            v = (a & 1) ? -bb : bb;
          }
        }
        P.Pm[a + (size_t)b * s] = v;
        tp[c][li] = v;
      }
    }
    if (!dgb) {
      __syncthreads();
#pragma unroll
      for (int m = 0; m < kPB / 8; ++m) {
        const int c = lg + 8 * m, j = j0 + li, i = i0 + c;
        if (j < n2 && i < n2 && i >= s && j >= s)
          P.Pm[(j - s) + (size_t)(i - s) * s] = tp[li][c];
      }
    }
  }
  const double D = block_sum(dsum, red);
  const double Tt = block_sum(tr, red);
  if (threadIdx.x == 0) {
    atomicAdd(&P.sc->diff, D);
    if (Tt != 0.0) atomicAdd(&P.sc->tr22, Tt);
  }
}

// stop rules (ADMMGainDesign2D.m:450-455, 3D.m:386-388): sum|dX| < thresh or
// |tr X22 - s|/s < threshTr
__global__ void __launch_bounds__(1024) check_kernel(const Part* parts, int nparts, double thresh,
                                                     double threshTr, int* remaining) {
  __shared__ int cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) {
    Scal& sc = *parts[p].sc;
    if (!sc.active) continue;
    sc.itr += 1;
    const double s = parts[p].s;
    if (sc.diff < thresh || fabs(sc.tr22 - s) / s < threshTr) sc.active = 0;
    sc.diff = 0.0;
    sc.tr22 = 0.0;
    if (sc.active) atomicAdd(&cnt, 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) *remaining = cnt;
}

// final projection: X22f = hb + P_V(X22) = hb + Pm - combine(c), into Sr
__global__ void __launch_bounds__(kT) x22f_kernel(const Part* parts) {
  const Part& P = parts[blockIdx.y];
  const int s = P.s;
  const double c0 = P.c[0];
  for (int e = blockIdx.x * kT + threadIdx.x; e < s * s; e += gridDim.x * kT) {
    const int i = e % s, j = e / s;
    P.Sr[e] = P.hb[e] + P.Pm[e] - combine_at(P, c0, i, j);
  }
}

// gains (3n x 3n column-major) from Axy (2n x 2n) and Az (n x n), |a| <= 1e-10
// zeroed (aclswarm/src/admm.cpp:49-50); iteration counts.
__global__ void __launch_bounds__(kT) assemble_kernel(const Part* parts, int n, int Fc, int f0,
                                                      double* gains, int32_t* iters) {
  const int fl = blockIdx.y;
  const Part& Pxy = parts[fl];
  const Part& Pz = parts[Fc + fl];
  const int N3 = 3 * n;
  double* G = gains + (size_t)(f0 + fl) * N3 * N3;
  for (int e = blockIdx.x * kT + threadIdx.x; e < N3 * N3; e += gridDim.x * kT) {
    const int R = e % N3, C = e / N3;
    const int i = R / 3, a = R % 3, j = C / 3, b = C % 3;
    double v = 0.0;
    if (a < 2 && b < 2) v = Pxy.Ap[(2 * i + a) + (size_t)(2 * j + b) * (2 * n)];
    else if (a == 2 && b == 2) v = Pz.Ap[i + (size_t)j * n];
    G[e] = (fabs(v) > 1e-10) ? v : 0.0;
  }
  if (iters && blockIdx.x == 0 && threadIdx.x == 0) {
    // negative: some PSD projection was resolved by neither the sign
    // iteration nor kJacobiSweeps Jacobi sweeps (the gains are unreliable)
    iters[2 * (f0 + fl)] = Pxy.sc->jacobi_fail ? -Pxy.sc->itr : Pxy.sc->itr;
    iters[2 * (f0 + fl) + 1] = Pz.sc->jacobi_fail ? -Pz.sc->itr : Pz.sc->itr;
  }
}

// ---------------------------------------------------------------------------
// host side

// test hook (acl_internal_admm_mem_cap): workspace allocations above this many
// bytes fail as out of memory (0 = no cap), to exercise the halving retry
size_t g_mem_cap = 0;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t b) {
    if (g_mem_cap && b > g_mem_cap) return hipErrorOutOfMemory;
    if (b <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, b);
    if (e == hipSuccess) bytes = b;
    return e;
  }
};

struct Ctx {
  DevBuf arena0, arena1, jobs, parts;
  int* h_cnt = nullptr;  // pinned
  int* d_cnt = nullptr;
  size_t jacobi_lds = 64 * 1024;  // psd_jacobi_kernel's dynamic-LDS limit as set
};
Ctx g_ctx[16];
unsigned long long* g_flops = nullptr;  // diagnostic GEMM flop counter (device)

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
inline int grid1(long long work) { return std::max(1, std::min(cdiv(work, kT), 1024)); }

// GEMM job lists: one device array of NP descriptors per kind
// J_NSYF / J_NSUF: the first Newton-Schulz step, reading Z0 = (W - eps I) /
// nrm from W through the GEMM's operand transform (no pass that writes N0)
enum {
  J_G, J_PRE1, J_PRE2, J_PIM1, J_PIM2, J_GINV, J_T, J_YK, J_NSY0, J_NSU0, J_NSY1, J_NSU1,
  J_S, J_S1, J_A1, J_AP, J_NSYF, J_NSUF, J_NST, J_COUNT
};

struct JobLists {
  GemmJob* dj = nullptr;  // device: J_COUNT x NP
  int NP = 0;
  int njob[J_COUNT] = {};
  int mx[J_COUNT][2] = {};
  // the kind's operands may be staged by LDS-DMA (gemm_f64.h): 16-byte
  // aligned operands, even leading dimensions and sizes,
  // 32-bit byte offsets (checked on the host over every job of the kind)
  bool dma[J_COUNT] = {};
  void check_dma(const GemmJob* jobs) {
    for (int k = 0; k < J_COUNT; ++k) {
      bool ok = njob[k] > 0;
      for (int i = 0; ok && i < njob[k]; ++i) {
        const GemmJob& j = jobs[(size_t)k * NP + i];
        const uintptr_t al = (uintptr_t)j.A | (uintptr_t)j.B | (uintptr_t)j.qB;
        ok = (j.tmask & ~7) == 0 && (al & 15) == 0 && ((j.lda | j.ldb | j.m | j.k) & 1) == 0 &&
             (long long)j.lda * j.k * 8 < (1ll << 30) && (long long)j.ldb * j.n * 8 < (1ll << 30);
      }
      dma[k] = ok;
    }
  }
  // symmetric products (exact arithmetic): G = Q Q^T, the Newton-Schulz
  // Z^2 and Z Z^2 (polynomials in one symmetric Z commute), W sign(W)
  static bool sym(int kind) {
    return kind == J_G || kind == J_NSY0 || kind == J_NSU0 || kind == J_NSY1 ||
           kind == J_NSU1 || kind == J_S || kind == J_S1 || kind == J_NSYF || kind == J_NSUF ||
           kind == J_NST;
  }
  hipError_t run(int kind, bool ta, bool tb, hipStream_t st) const {
    return gemm_f64(ta, tb, dj + (size_t)kind * NP, njob[kind], mx[kind][0], mx[kind][1], st,
                    g_flops, sym(kind) && mx[kind][0] == mx[kind][1], dma[kind]);
  }
};

// The Newton-Schulz and S products of one part (dimension n2): Y = Z^2 (with
// |Y - I|_F^2 and the tr Y partials when fused), Z <- Z (3 - Y) / 2 scaled
// (kNsCap), the first step reading Z0 = (W - eps I) / nrm through the operand
// transform, S = (W + W sign) / 2 from the parity's sign buffer.
template <class Add>
void add_sign_jobs(Add& add, const Part& P, int n2, double eps, bool fuse) {
  const int* nsd = &P.sc->ns_done;
  double* e2 = fuse ? &P.sc->err2 : nullptr;
  const int ntr = (n2 + gemm_tile_size() - 1) / gemm_tile_size();
  const bool scaled = fuse && ntr <= kTrMax;
  auto y = [&](GemmJob j) {
    if (scaled) j.trp = P.sc->trp;
    return j;
  };
  auto u = [&](GemmJob j, double cap) {
    if (scaled) {
      j.nsp = P.sc->trp;
      j.nserr = &P.sc->err2;
      j.nsn = ntr;
      j.nscap = cap;
      j.nstol = kNsTol * n2;
      j.qB = P.Sr;  // T (J_NST), in the quintic band
      j.qlo = kNsTol * n2;
      j.qhi = kNsTolQ * n2;
      j.qalpha = 1.0;
      j.qbeta = 1.875;
    }
    return j;
  };
  if (scaled) {  // T = 3/8 Y Y - 10/8 Y into Sr (free until the S products), quintic band only
    GemmJob t{P.Y, P.Y, P.Y, P.Sr, n2, n2, n2, n2, n2, n2, n2, 0.375, -1.25, &P.sc->ns_done};
    t.gerr = &P.sc->err2;
    t.glo = kNsTol * n2;
    t.ghi = kNsTolQ * n2;
    add(J_NST, t);
  }
  const int N = n2;
  add(J_NSY0, y({P.N0, P.N0, nullptr, P.Y, N, N, N, N, N, N, N, 1.0, 0.0, nsd, e2}));
  add(J_NSU0, u({P.N0, P.Y, P.N0, P.N1, N, N, N, N, N, N, N, -0.5, 1.5, nsd}, kNsCap));
  add(J_NSYF, y({P.W, P.W, nullptr, P.Y, N, N, N, N, N, N, N, 1.0, 0.0, nsd, e2, &P.sc->nrm, eps, 3}));
  add(J_NSUF, u({P.W, P.Y, P.W, P.N1, N, N, N, N, N, N, N, -0.5, 1.5, nsd, nullptr, &P.sc->nrm, eps, 5},
                kNsCap / kNsScale));
  add(J_NSY1, y({P.N1, P.N1, nullptr, P.Y, N, N, N, N, N, N, N, 1.0, 0.0, nsd, e2}));
  add(J_NSU1, u({P.N1, P.Y, P.N1, P.N0, N, N, N, N, N, N, N, -0.5, 1.5, nsd}, kNsCap));
  add(J_S, {P.W, P.N0, P.W, P.Sr, N, N, N, N, N, N, N, 0.5, 0.5, &P.sc->skip_s0});
  add(J_S1, {P.W, P.N1, P.W, P.Sr, N, N, N, N, N, N, N, 0.5, 0.5, &P.sc->skip_s1});
}

// The PSD part of every active part's W (eigenvalues > eps) into Sr: the
// Newton-Schulz sign iteration on the matrix cores (S = (W + W sign(W - eps
// I)) / 2), then psd_jacobi_kernel for the parts it did not resolve
// (force_jacobi: for every part, a test hook). Synchronises the stream to
// stop the sign iteration once every part has converged.
hipError_t psd_project(const JobLists& J, Part* dp, int NP, int n2max, double eps, bool fuse_err,
                       bool force_jacobi, Ctx& X, hipStream_t st) {
  const dim3 gW(grid1((long long)n2max * n2max), NP);
  hipLaunchKernelGGL(norm_kernel, dim3(NP), dim3(kT), 0, st, dp, eps);
  // the default GEMM forms Z0 = (W - eps I) / nrm while staging step 0's
  // operands (J_NSYF / J_NSUF); other tiles (diagnostic builds) write N0 first
  const bool tr = gemm_tile() == 80;
  if (!tr) hipLaunchKernelGGL(nsinit_kernel, gW, dim3(kT), 0, st, dp, eps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // every part has the scaled and quintic jobs when fused and no part has
  // more than kTrMax diagonal tiles (add_sign_jobs): then a check in the
  // quintic band ends the iteration too
  const double tol =
      (fuse_err && (n2max + gemm_tile_size() - 1) / gemm_tile_size() <= kTrMax) ? kNsTolQ : kNsTol;
  for (int it = 0; it < kNsMax; ++it) {
    const bool odd = it & 1;
    const bool first = tr && it == 0;
    if ((e = J.run(first ? J_NSYF : (odd ? J_NSY1 : J_NSY0), false, false, st)) != hipSuccess)
      return e;
    if (!fuse_err)
      hipLaunchKernelGGL(nserr_kernel, dim3(std::min(grid1((long long)n2max * n2max), 64), NP),
                         dim3(kT), 0, st, dp);
    // the quintic band's T (no jobs unless add_sign_jobs made them; each
    // gated on its part's check)
    if ((e = J.run(J_NST, false, false, st)) != hipSuccess) return e;
    if ((e = J.run(first ? J_NSUF : (odd ? J_NSU1 : J_NSU0), false, false, st)) != hipSuccess)
      return e;
    hipLaunchKernelGGL(nsstep_kernel, dim3(1), dim3(1024), 0, st, dp, NP,
                       it == kNsMax - 1 ? 1 : 0, tol, X.d_cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (it >= 5) {  // [0] still iterating, [2] failed (d_cnt[1] is check_kernel's)
      if ((e = hipMemcpyAsync(X.h_cnt, X.d_cnt, 3 * sizeof(int), hipMemcpyDeviceToHost, st)) !=
          hipSuccess)
        return e;
      if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
      if (*X.h_cnt == 0) break;
    }
  }
  if (force_jacobi) hipLaunchKernelGGL(force_jacobi_kernel, dim3(1), dim3(1024), 0, st, dp, NP);
  hipLaunchKernelGGL(nsparity_kernel, dim3(1), dim3(1024), 0, st, dp, NP);
  if ((e = J.run(J_S, false, false, st)) != hipSuccess) return e;
  if ((e = J.run(J_S1, false, false, st)) != hipSuccess) return e;
  // the fallback only when some part needs it (the last readback's count)
  if (!force_jacobi && X.h_cnt[2] == 0) return hipSuccess;
  const size_t jlds = (size_t)20 * n2max;
  if (jlds > X.jacobi_lds) {
    if ((e = hipFuncSetAttribute((const void*)psd_jacobi_kernel,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)jlds)) !=
        hipSuccess)
      return e;
    X.jacobi_lds = jlds;
  }
  hipLaunchKernelGGL(psd_jacobi_kernel, dim3(NP), dim3(kJT), jlds, st, dp, eps);
  return hipGetLastError();
}

}  // namespace admm
}  // namespace acl_amd

extern "C" acl_status_t acl_admm_solve_batch(int32_t F, int32_t n, const double* pts,
                                             const double* adj, double* gains, int32_t* iters,
                                             const acl_admm_params_t* params, void* stream) {
  using namespace acl_amd;
  using namespace acl_amd::admm;
  if (F < 0) return acl__set_error("acl_admm_solve_batch: F < 0");
  if (F == 0) return ACL_OK;
  if (n < 3 || n > kMaxN) {
    acl__set_error("acl_admm_solve_batch: n out of range [3, 1024]");
    return ACL_ERR_UNSUPPORTED;
  }
  if (!pts || !adj || !gains) return acl__set_error("acl_admm_solve_batch: null pointer");
  acl_admm_params_t prm;
  if (params) prm = *params;
  else acl_default_admm_params(&prm);
  if (prm.basis != ACL_ADMM_BASIS_LINPACK && prm.basis != ACL_ADMM_BASIS_COMPLEX)
    return acl__set_error("acl_admm_solve_batch: params->basis must be ACL_ADMM_BASIS_*");
  const hipStream_t st = (hipStream_t)stream;
  int dev = 0;
  (void)hipGetDevice(&dev);
  Ctx& X = g_ctx[dev & 15];
  if (!X.h_cnt) {
    if (hipHostMalloc((void**)&X.h_cnt, sizeof(int) * 4) != hipSuccess ||
        hipMalloc((void**)&X.d_cnt, sizeof(int) * 4) != hipSuccess)
      return acl__set_error("acl_admm_solve_batch: allocation failed");
  }
  auto hipfail = [&](hipError_t e, const char* what) -> acl_status_t {
    static thread_local char buf[256];
    snprintf(buf, sizeof buf, "acl_admm_solve_batch: %s: %s", what, hipGetErrorString(e));
    acl__set_error(buf);
    return ACL_ERR_HIP;
  };
#define ACL_HIP(call, what)                  \
  do {                                       \
    hipError_t e_ = (call);                  \
    if (e_ != hipSuccess) return hipfail(e_, what); \
  } while (0)

  // Formations per pass: at most ACL_ADMM_CHUNK; a pass whose workspace does
  // not fit the device (the per-part arena grows with the graph rows K and
  // the complement dimension s) is retried with half as many formations.
  int chunk = std::min(F, ACL_ADMM_CHUNK);
  auto oom_retry = [&](hipError_t e, int Fc) {
    if (e != hipErrorOutOfMemory || Fc <= 1) return false;
    (void)hipGetLastError();  // clear the failed allocation's error
    chunk = Fc / 2;
    return true;
  };
  const int np_max = 2 * n;
  const size_t qstride = (size_t)np_max * np_max;
  const size_t kcap = (size_t)n * (n - 1);  // xy graph rows at most
  const size_t pstride = 2 * std::min(kcap, (size_t)kMaxRows);
  for (int f0 = 0; f0 < F;) {
    const int Fc = std::min(chunk, F - f0);
    const int NP = 2 * Fc;
    // ---- phase 0: basis and graph rows
    const size_t a0 = NP * qstride * sizeof(double) + NP * pstride * sizeof(unsigned short) +
                      NP * sizeof(Info) + 256;
    {
      const hipError_t e0 = X.arena0.ensure(a0);
      if (oom_retry(e0, Fc)) continue;
      ACL_HIP(e0, "hipMalloc");
    }
    double* Qbuf = (double*)X.arena0.p;
    unsigned short* pairbuf = (unsigned short*)(Qbuf + NP * qstride);
    Info* d_info = (Info*)(((uintptr_t)(pairbuf + NP * pstride) + 15) & ~(uintptr_t)15);
    const size_t lds = (size_t)(4 * np_max + np_max + 8) * sizeof(double) + (np_max + n + 1) * sizeof(int);
    if (lds > 48 * 1024)
      ACL_HIP(hipFuncSetAttribute((const void*)basis_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
              "hipFuncSetAttribute");
    hipLaunchKernelGGL(basis_kernel, dim3(NP), dim3(kT), lds, st, n, Fc, f0, pts, adj,
                       prm.thrPlanar, prm.basis, Qbuf, qstride, pairbuf, pstride, d_info);
    ACL_HIP(hipGetLastError(), "basis_kernel");
    std::vector<Info> info(NP);
    ACL_HIP(hipMemcpyAsync(info.data(), d_info, NP * sizeof(Info), hipMemcpyDeviceToHost, st),
            "hipMemcpyAsync");
    ACL_HIP(hipStreamSynchronize(st), "hipStreamSynchronize");
    int Kmax = 0;
    for (const Info& in : info) Kmax = std::max(Kmax, in.K);
    if (Kmax > kMaxRows) {
      acl__set_error("acl_admm_solve_batch: more than 2047 graph rows (non-edges) in one part");
      return ACL_ERR_UNSUPPORTED;
    }
    // ---- carve per-part buffers
    std::vector<Part> hp(NP);
    size_t off = 0;
    auto take = [&](size_t nd) {
      const size_t o = off;
      off += (nd + 31) & ~(size_t)31;
      return o;
    };
    std::vector<size_t> offs;
    offs.reserve(NP * 24);
    for (int p = 0; p < NP; ++p) {
      const Info& in = info[p];
      const size_t s = in.s, K = in.K, K1 = K + 1, n2 = 2 * s, npp = in.np;
      const size_t big = std::max(n2 * n2, npp * npp);
      offs.push_back(take(K * s));      // Qa
      offs.push_back(take(K * s));      // Qb
      offs.push_back(take(K * s));      // Qbc
      offs.push_back(take(K * s));      // Yk
      offs.push_back(take(K1 * K1));    // Gam
      offs.push_back(take(K1 * K1));    // Li
      offs.push_back(take(K1 * K1));    // Ginv
      offs.push_back(take(K1));         // r
      offs.push_back(take(K1));         // c
      offs.push_back(take(s * s));      // hb
      offs.push_back(take(s * s));      // Pm
      offs.push_back(take(s * s));      // T
      offs.push_back(take(big));        // W / G
      offs.push_back(take(n2 * n2));    // S
      offs.push_back(take(big));        // Sr / Pre
      offs.push_back(take(n2 * n2));    // X
      offs.push_back(take(big));        // N0 / A1
      offs.push_back(take(big));        // N1 / Ap
      offs.push_back(take(big));        // Y / Pim
      offs.push_back(take(n2));         // cs
    }
    const size_t nd_parts = off;
    const size_t scal_off = nd_parts * sizeof(double);
    const size_t a1 = scal_off + NP * sizeof(Scal) + 256;
    {
      const hipError_t e1 = X.arena1.ensure(a1);
      if (oom_retry(e1, Fc)) continue;
      ACL_HIP(e1, "hipMalloc (ADMM workspace)");
    }
    double* base = (double*)X.arena1.p;
    Scal* scal = (Scal*)((char*)X.arena1.p + scal_off);
    for (int p = 0; p < NP; ++p) {
      const Info& in = info[p];
      Part& P = hp[p];
      P.np = in.np; P.s = in.s; P.K = in.K; P.st = in.st;
      P.Q = Qbuf + p * qstride;
      P.pa = pairbuf + p * pstride;
      P.pb = P.pa + 1;
      const size_t* o = &offs[(size_t)p * 20];
      P.Qa = base + o[0]; P.Qb = base + o[1]; P.Qbc = base + o[2]; P.Yk = base + o[3];
      P.Gam = base + o[4]; P.Li = base + o[5]; P.Ginv = base + o[6];
      P.r = base + o[7]; P.c = base + o[8];
      P.hb = base + o[9]; P.Pm = base + o[10]; P.T = base + o[11];
      P.W = base + o[12]; P.S = base + o[13]; P.Sr = base + o[14]; P.X = base + o[15];
      P.N0 = base + o[16]; P.N1 = base + o[17]; P.Y = base + o[18];
      P.cs = P.Y;  // w_ut_kernel's column-sum partials (nb x 2s; Y is free until the sign iteration)
      P.G = P.W; P.Pre = P.Sr; P.Pim = P.Y;
      P.A1 = P.N0; P.Ap = P.N1;
      P.sc = scal + p;
    }
    // ---- GEMM job lists
    std::vector<GemmJob> jobs((size_t)J_COUNT * NP);
    JobLists JL;
    JL.NP = NP;
    auto add = [&](int kind, const GemmJob& j) {
      jobs[(size_t)kind * NP + JL.njob[kind]++] = j;
      JL.mx[kind][0] = std::max(JL.mx[kind][0], j.m);
      JL.mx[kind][1] = std::max(JL.mx[kind][1], j.n);
    };
    // the default GEMM kernel (the four-wave 80 tile) fuses nserr_kernel's
    // |Y - I|_F^2 into the epilogue of the Newton-Schulz product Y = Z^2
    const bool fuse_err = gemm_tile() == 80;
    for (int p = 0; p < NP; ++p) {
      const Part& P = hp[p];
      const int s = P.s, K = P.K, K1 = K + 1, np = P.np, n2 = 2 * s;
      add(J_G, {P.Q, P.Q, nullptr, P.G, np, np, s, np, np, np, np, 1.0, 0.0, nullptr});
      if (P.st) {
        const int h = s / 2;
        add(J_PRE1, {P.Q, P.Q, nullptr, P.Pre, np, np, h, 2 * np, 2 * np, np, np, 1.0, 0.0, nullptr});
        add(J_PRE2, {P.Q + np, P.Q + np, P.Pre, P.Pre, np, np, h, 2 * np, 2 * np, np, np, 1.0, 1.0, nullptr});
        add(J_PIM1, {P.Q + np, P.Q, nullptr, P.Pim, np, np, h, 2 * np, 2 * np, np, np, 1.0, 0.0, nullptr});
        add(J_PIM2, {P.Q, P.Q + np, P.Pim, P.Pim, np, np, h, 2 * np, 2 * np, np, np, -1.0, 1.0, nullptr});
      }
      add(J_GINV, {P.Gam, P.Gam, nullptr, P.Ginv, K1, K1, K1, K1, K1, K1, K1, 1.0, 0.0, nullptr});
      add(J_T, {P.Qa, P.Qbc, nullptr, P.T, s, s, K, std::max(K, 1), std::max(K, 1), s, s, 1.0, 0.0, nullptr});
      add(J_YK, {P.Qa, P.Pm, nullptr, P.Yk, K, s, s, std::max(K, 1), s, std::max(K, 1), std::max(K, 1), 1.0, 0.0, nullptr});
      // (err2: the default GEMM kernel accumulates |Y - I|_F^2, nserr_kernel's sum)
      add_sign_jobs(add, P, n2, prm.epsEig, fuse_err);
      add(J_A1, {P.Q, P.Sr, nullptr, P.A1, np, s, s, np, s, np, np, 1.0, 0.0, nullptr});
      add(J_AP, {P.A1, P.Q, nullptr, P.Ap, np, np, s, np, np, np, np, -1.0, 0.0, nullptr});
    }
    ACL_HIP(X.jobs.ensure(jobs.size() * sizeof(GemmJob)), "hipMalloc");
    ACL_HIP(X.parts.ensure(NP * sizeof(Part)), "hipMalloc");
    GemmJob* dj = (GemmJob*)X.jobs.p;
    Part* dp = (Part*)X.parts.p;
    ACL_HIP(hipMemcpyAsync(dj, jobs.data(), jobs.size() * sizeof(GemmJob), hipMemcpyHostToDevice, st),
            "hipMemcpyAsync");
    ACL_HIP(hipMemcpyAsync(dp, hp.data(), NP * sizeof(Part), hipMemcpyHostToDevice, st),
            "hipMemcpyAsync");
    JL.dj = dj;
    JL.check_dma(jobs.data());
    auto gemm = [&](int kind, bool ta, bool tb) -> hipError_t { return JL.run(kind, ta, tb, st); };
    int max_s = 0, max_np = 0, maxK1 = 1;
    for (const Info& in : info) {
      max_s = std::max(max_s, in.s);
      max_np = std::max(max_np, in.np);
      maxK1 = std::max(maxK1, in.K + 1);
    }
    const int n2max = 2 * max_s;
    const dim3 gS(grid1((long long)max_s * max_s), NP), gW(grid1((long long)n2max * n2max), NP);
    // ---- setup
    hipLaunchKernelGGL(gather_kernel, dim3(grid1((long long)Kmax * max_s), NP), dim3(kT), 0, st, dp);
    ACL_HIP(gemm(J_G, false, true), "gemm G");
    ACL_HIP(gemm(J_PRE1, false, true), "gemm Pre");
    ACL_HIP(gemm(J_PRE2, false, true), "gemm Pre");
    ACL_HIP(gemm(J_PIM1, false, true), "gemm Pim");
    ACL_HIP(gemm(J_PIM2, false, true), "gemm Pim");
    hipLaunchKernelGGL(gamma_kernel, dim3(grid1((long long)maxK1 * maxK1), NP), dim3(kT), 0, st, dp);
    if (chol_lds_fits(maxK1)) {
      const size_t cb = chol_lds_bytes(maxK1);
      if (cb > 64 * 1024)
        ACL_HIP(hipFuncSetAttribute((const void*)chol_lds_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)cb),
                "hipFuncSetAttribute");
      hipLaunchKernelGGL(chol_lds_kernel, dim3(NP), dim3(kCholT), cb, st, dp);
    } else {
      hipLaunchKernelGGL(chol_kernel, dim3(NP), dim3(kT), 0, st, dp);
    }
    ACL_HIP(gemm(J_GINV, true, false), "gemm Ginv");
    hipLaunchKernelGGL(rc_kernel, dim3(NP), dim3(kT), 0, st, dp, 0, prm.mu);
    ACL_HIP(gemm(J_T, true, false), "gemm T");
    hipLaunchKernelGGL(init_kernel, gW, dim3(kT), 0, st, dp);
    ACL_HIP(hipGetLastError(), "setup kernels");
    // ---- ADMM iterations
    const double mu = prm.mu, eps = prm.epsEig;
    // the iterations after the first take Pm from the previous post-process
    // (post_ut_kernel's pmf: every structured part's s even)
    bool pm_fused = true;
    for (int p = 0; p < NP; ++p)
      if (info[p].st && (info[p].s & 1)) pm_fused = false;
    for (int itr = 0; itr < prm.maxItr; ++itr) {
      if (itr == 0 || !pm_fused) hipLaunchKernelGGL(pm_kernel, gS, dim3(kT), 0, st, dp, -1.0, -mu, 1);
      ACL_HIP(gemm(J_YK, false, false), "gemm Yk");
      hipLaunchKernelGGL(rc_kernel, dim3(NP), dim3(kT), 0, st, dp, 1, mu);
      ACL_HIP(gemm(J_T, true, false), "gemm T");
      {
        const int nbw = (n2max + kWB - 1) / kWB;
        hipLaunchKernelGGL(w_ut_kernel, dim3(nbw * (nbw + 1) / 2, NP), dim3(256), 0, st, dp, mu, eps);
      }
      ACL_HIP(hipGetLastError(), "iteration kernels");
      ACL_HIP(psd_project(JL, dp, NP, n2max, eps, fuse_err, false, X, st), "PSD projection");
      {
        const int nbp = (n2max + kPB - 1) / kPB;
        hipLaunchKernelGGL(post_ut_kernel, dim3(nbp * (nbp + 1) / 2, NP), dim3(256), 0, st, dp, mu,
                           JobLists::sym(J_S) ? gemm_tile_size() : (1 << 30), pm_fused ? 1 : 0);
      }
      hipLaunchKernelGGL(check_kernel, dim3(1), dim3(1024), 0, st, dp, NP, prm.thresh,
                         prm.threshTr, X.d_cnt + 1);
      ACL_HIP(hipGetLastError(), "iteration kernels");
      ACL_HIP(hipMemcpyAsync(X.h_cnt + 1, X.d_cnt + 1, sizeof(int), hipMemcpyDeviceToHost, st), "copy");
      ACL_HIP(hipStreamSynchronize(st), "sync");
      if (X.h_cnt[1] == 0) break;
    }
    // ---- final projection (S = 0) and the gain matrix
    hipLaunchKernelGGL(pm_kernel, gS, dim3(kT), 0, st, dp, 0.0, 1.0, 0);
    ACL_HIP(gemm(J_YK, false, false), "gemm Yk");
    hipLaunchKernelGGL(rc_kernel, dim3(NP), dim3(kT), 0, st, dp, 2, mu);
    ACL_HIP(gemm(J_T, true, false), "gemm T");
    hipLaunchKernelGGL(x22f_kernel, gS, dim3(kT), 0, st, dp);
    ACL_HIP(gemm(J_A1, false, false), "gemm A1");
    ACL_HIP(gemm(J_AP, false, true), "gemm Ap");
    hipLaunchKernelGGL(assemble_kernel, dim3(grid1(9LL * n * n), Fc), dim3(kT), 0, st, dp, n, Fc,
                       f0, gains, iters);
    ACL_HIP(hipGetLastError(), "final kernels");
    // the next chunk reuses the workspace
    f0 += Fc;
    if (f0 < F) ACL_HIP(hipStreamSynchronize(st), "sync");
  }
#undef ACL_HIP
  return ACL_OK;
}

// Test hook (not part of the public ABI; tests/test_gpu_admm.py): ADMM
// workspace allocations above `bytes` fail as out of memory (0 = off), so a
// batch runs in passes of fewer formations, as it does when the device is full.
extern "C" void acl_internal_admm_mem_cap(size_t bytes) { acl_amd::admm::g_mem_cap = bytes; }

// Diagnostic (not part of the public ABI): counts the algorithmic flops of
// every ADMM GEMM tile into *counter (a device pointer; NULL turns it off).
extern "C" void acl_internal_admm_flop_counter(unsigned long long* counter) {
  acl_amd::admm::g_flops = counter;
}

// Test hook (not part of the public ABI; tests/test_gpu_admm.py): the PSD
// projection of nm symmetric N x N matrices W (device, column-major, N even)
// into S = (Sr + Sr^T) / 2 exactly as an ADMM iteration makes it (Newton-
// Schulz on the matrix cores, the Jacobi fallback where the sign iteration
// does not converge; force_jacobi: the fallback for every matrix).
// jacobi_used (host, may be NULL): per matrix, 1 if the fallback made it,
// -1 if the fallback stopped at kJacobiSweeps unconverged.
// Synchronous; returns 0 on success.
extern "C" int acl_internal_psd_project(int nm, int N, const double* W, double eps, double* S,
                                        int force_jacobi, int* jacobi_used) {
  using namespace acl_amd;
  using namespace acl_amd::admm;
  if (nm <= 0 || N < 2 || (N & 1)) return 1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  Ctx& X = g_ctx[dev & 15];
  if (!X.h_cnt) {
    if (hipHostMalloc((void**)&X.h_cnt, sizeof(int) * 4) != hipSuccess ||
        hipMalloc((void**)&X.d_cnt, sizeof(int) * 4) != hipSuccess)
      return 1;
  }
  const size_t NN = (size_t)N * N;
  double* buf = nullptr;
  Scal* sc = nullptr;
  Part* dp = nullptr;
  GemmJob* dj = nullptr;
  if (hipMalloc((void**)&buf, 5 * NN * nm * sizeof(double)) != hipSuccess) return 1;
  if (hipMalloc((void**)&sc, nm * sizeof(Scal)) != hipSuccess) return 1;
  if (hipMalloc((void**)&dp, nm * sizeof(Part)) != hipSuccess) return 1;
  if (hipMalloc((void**)&dj, (size_t)J_COUNT * nm * sizeof(GemmJob)) != hipSuccess) return 1;
  std::vector<Part> hp(nm);
  std::vector<Scal> hs(nm);
  std::vector<GemmJob> jobs((size_t)J_COUNT * nm);
  JobLists JL;
  JL.NP = nm;
  JL.dj = dj;
  auto add = [&](int kind, const GemmJob& j) {
    jobs[(size_t)kind * nm + JL.njob[kind]++] = j;
    JL.mx[kind][0] = std::max(JL.mx[kind][0], j.m);
    JL.mx[kind][1] = std::max(JL.mx[kind][1], j.n);
  };
  const bool fuse_err = gemm_tile() == 80;
  for (int p = 0; p < nm; ++p) {
    Part& P = hp[p];
    P = Part{};
    P.s = N / 2;
    P.W = const_cast<double*>(W) + p * NN;
    P.N0 = buf + (5 * (size_t)p + 0) * NN;
    P.N1 = buf + (5 * (size_t)p + 1) * NN;
    P.Y = buf + (5 * (size_t)p + 2) * NN;
    P.Sr = buf + (5 * (size_t)p + 3) * NN;
    P.sc = sc + p;
    hs[p] = Scal{};
    hs[p].active = 1;
    add_sign_jobs(add, P, N, eps, fuse_err);
  }
  int rc = 1;
  do {
    if (hipMemcpy(dj, jobs.data(), jobs.size() * sizeof(GemmJob), hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipMemcpy(dp, hp.data(), nm * sizeof(Part), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(sc, hs.data(), nm * sizeof(Scal), hipMemcpyHostToDevice) != hipSuccess)
      break;
    if (psd_project(JL, dp, nm, N, eps, fuse_err, force_jacobi != 0, X, 0) != hipSuccess) break;
    if (hipDeviceSynchronize() != hipSuccess) break;
    // S = (Sr + Sr^T) / 2 on the host side of the copy (test hook only)
    std::vector<double> sr(NN);
    bool ok = true;
    for (int p = 0; p < nm && ok; ++p) {
      ok = hipMemcpy(sr.data(), hp[p].Sr, NN * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
      std::vector<double> o(NN);
      for (int j = 0; j < N; ++j)
        for (int i = 0; i < N; ++i)
          o[i + (size_t)j * N] = 0.5 * (sr[i + (size_t)j * N] + sr[j + (size_t)i * N]);
      ok = ok && hipMemcpy(S + p * NN, o.data(), NN * sizeof(double), hipMemcpyHostToDevice) ==
                     hipSuccess;
    }
    if (!ok) break;
    if (jacobi_used) {
      if (hipMemcpy(hs.data(), sc, nm * sizeof(Scal), hipMemcpyDeviceToHost) != hipSuccess) break;
      for (int p = 0; p < nm; ++p) jacobi_used[p] = hs[p].jacobi_fail ? -1 : hs[p].jacobi;
    }
    rc = 0;
  } while (0);
  (void)hipFree(buf);
  (void)hipFree(sc);
  (void)hipFree(dp);
  (void)hipFree(dj);
  return rc;
}
