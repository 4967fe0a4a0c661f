// umeyama_dev.h -- device-side 2-D Umeyama alignment for the CBAA kernel.
//
// Auctioneer::alignFormation (aclswarm/src/auctioneer.cpp:347-415) calls
// Eigen::umeyama(p_xy, q_xy, false) on the vehicle's closed formation
// neighbourhood. Eigen (unpinned, "3.2.2 or later", CMakeLists.txt:30-32) is
// not in the image; DESIGN.md §3 states the Eigen 3.3.4 algorithm this file
// implements. Every expression keeps Eigen's operation order; the library is
// compiled with -ffp-contract=off so no FMA contraction changes a rounding.
// One thread computes one vehicle's (R, t) in registers.
#pragma once

#include <hip/hip_runtime.h>
#include <float.h>

#include "common.h"

namespace acl_amd {

// (shared by align_kernel and align_wide_kernel's alignment sums)
// a_k += v_k in the lanes of `mask` only (the others keep a_k): exec is
// narrowed around the four adds, so non-members cost no selects and leave no
// trace in the sums (Eigen's sums run over the members only)
__device__ __forceinline__ void masked_add4(unsigned long long mask, double& a0, double& a1,
                                            double& a2, double& a3, double v0, double v1,
                                            double v2, double v3) {
  unsigned long long sv;
  asm volatile(
      "s_and_saveexec_b64 %[sv], %[m]\n\t"
      "v_add_f64 %[a0], %[a0], %[v0]\n\t"
      "v_add_f64 %[a1], %[a1], %[v1]\n\t"
      "v_add_f64 %[a2], %[a2], %[v2]\n\t"
      "v_add_f64 %[a3], %[a3], %[v3]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [sv] "=&s"(sv)
      : [m] "s"(mask), [v0] "v"(v0), [v1] "v"(v1), [v2] "v"(v2), [v3] "v"(v3)
      : "scc");  // s_and_saveexec writes SCC
}

// apply_rotation_in_the_plane on the pair (x, y): x' = c x + s y,
// y' = -s x + c y, with Eigen's early return for (c, s) == (1, 0) kept as a
// select (the unrotated values, -0.0 and NaN included): branch-free, so the
// sweep keeps one copy of W, U, V in registers.
__device__ __forceinline__ void rot_pair(double& x, double& y, double c, double s, bool id) {
  const double xn = c * x + s * y;
  const double yn = -s * x + c * y;
  x = id ? x : xn;
  y = id ? y : yn;
}

// MatrixBase::applyOnTheLeft(p, q, (c, s)) on a column-major 2x2: rows p, q
__device__ __forceinline__ void rot_rows(double* W, int p, int q, double c, double s) {
  const bool id = c == 1.0 && s == 0.0;
#pragma unroll
  for (int k = 0; k < 2; ++k) rot_pair(W[p + 2 * k], W[q + 2 * k], c, s, id);
}

// applyOnTheRight(p, q, (c, s)): columns p, q
__device__ __forceinline__ void rot_cols(double* M, int p, int q, double c, double s) {
  const bool id = c == 1.0 && s == 0.0;
#pragma unroll
  for (int k = 0; k < 2; ++k) rot_pair(M[k + 2 * p], M[k + 2 * q], c, s, id);
}

// JacobiRotation::makeJacobi(x, y, z), real case; the deno < DBL_MIN early
// return (identity) as a select.
__device__ __forceinline__ void make_jacobi(double x, double y, double z, double& c, double& s) {
  const double deno = 2.0 * fabs(y);
  const bool tiny = deno < DBL_MIN;
  const double tau = (x - z) / deno;
  const double w = sqrt(tau * tau + 1.0);
  const double t = (tau > 0.0) ? 1.0 / (tau + w) : 1.0 / (tau - w);
  const double sign_t = t > 0.0 ? 1.0 : -1.0;
  const double n = 1.0 / sqrt(t * t + 1.0);
  const double sj = -sign_t * (y / fabs(y)) * fabs(t) * n;
  c = tiny ? 1.0 : n;
  s = tiny ? 0.0 : sj;
}

// PartialPivLU determinant of a dynamic 2x2 (only its sign is consumed).
__device__ __forceinline__ double det2_lu(const double* A) {
  double a00 = A[0], a10 = A[1], a01 = A[2], a11 = A[3];
  double sign = 1.0;
  const double b0 = fabs(a00), b1 = fabs(a10);
  const bool piv = b1 > b0;
  const double biggest = piv ? b1 : b0;
  if (biggest != 0.0) {
    if (piv) {
      double t = a00; a00 = a10; a10 = t;
      t = a01; a01 = a11; a11 = t;
      sign = -1.0;
    }
    a10 = a10 / a00;
  }
  a11 = a11 - a10 * a01;
  return (a00 * a11) * sign;
}

// JacobiSVD<MatrixXd>(A, ComputeFullU | ComputeFullV) for 2x2 A (column-major).
// Returns false when A is not finite (Eigen: InvalidInput).
__device__ inline bool jacobi_svd2(const double* A, double* U, double* sv, double* V) {
  const double precision = 2.0 * DBL_EPSILON;
  const double considerAsZero = DBL_MIN;
  double scale = fabs(A[0]);
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    const double a = fabs(A[i]);
    if (a > scale || isnan(a)) scale = a;
  }
  if (!isfinite(scale)) return false;
  if (scale == 0.0) scale = 1.0;
  double W[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) W[i] = A[i] / scale;
  U[0] = 1.0; U[1] = 0.0; U[2] = 0.0; U[3] = 1.0;
  V[0] = 1.0; V[1] = 0.0; V[2] = 0.0; V[3] = 1.0;
  double maxDiag = fabs(W[0]);
  if (maxDiag < fabs(W[3])) maxDiag = fabs(W[3]);
  // Each sweep of a 2x2 is one (p=1, q=0) rotation; the loop ends when the
  // off-diagonal is below threshold (at most a few sweeps; bounded for safety).
  for (int sweep = 0; sweep < 64; ++sweep) {
    double threshold = precision * maxDiag;
    if (threshold < considerAsZero) threshold = considerAsZero;
    if (!(fabs(W[1]) > threshold || fabs(W[2]) > threshold)) break;
    // real_2x2_jacobi_svd(W, 1, 0): m = [W11 W10; W01 W00]
    double m[4];
    m[0] = W[3];
    m[2] = W[1];
    m[1] = W[2];
    m[3] = W[0];
    const double t = m[0] + m[3];
    const double d = m[1] - m[2];
    const bool dz = fabs(d) < DBL_MIN;
    const double u = t / d;
    const double tmp = sqrt(1.0 + u * u);
    const double s1 = dz ? 0.0 : 1.0 / tmp;
    const double c1 = dz ? 1.0 : u / tmp;
    rot_rows(m, 0, 1, c1, s1);
    double cr, sr;
    make_jacobi(m[0], m[2], m[3], cr, sr);
    const double ocs = -sr;
    const double cl = c1 * cr - s1 * ocs;
    const double sl = c1 * ocs + s1 * cr;
    rot_rows(W, 1, 0, cl, sl);
    rot_cols(U, 1, 0, cl, sl);
    rot_cols(W, 1, 0, cr, -sr);
    rot_cols(V, 1, 0, cr, -sr);
    double md = fabs(W[3]);
    if (md < fabs(W[0])) md = fabs(W[0]);
    if (maxDiag < md) maxDiag = md;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double a = W[i * 3];
    sv[i] = fabs(a);
    if (a < 0.0) {
      U[2 * i] = -U[2 * i];
      U[2 * i + 1] = -U[2 * i + 1];
    }
  }
  sv[0] *= scale;
  sv[1] *= scale;
  const bool pos = sv[1] > sv[0];
  const double mx = pos ? sv[1] : sv[0];
  if (mx != 0.0 && pos) {
    double t = sv[0]; sv[0] = sv[1]; sv[1] = t;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      t = U[k]; U[k] = U[2 + k]; U[2 + k] = t;
      t = V[k]; V[k] = V[2 + k]; V[2 + k] = t;
    }
  }
  return true;
}

// Finishes Eigen::umeyama (3.3.x rank rule) from the means and the
// accumulated cross-covariance. R row-major 2x2, t[2]; *gap the decision gap
// of the determinant-sign and rank tests (common.h align_gap; 0 when the
// input is not finite).
__device__ inline bool umeyama_finish(const double* S, const double* sm, const double* dm,
                                      double* R, double* t, double* gap) {
  double U[4], V[4], sv[2];
  if (!jacobi_svd2(S, U, sv, V)) {
    const double nan = __builtin_nan("");
    R[0] = R[1] = R[2] = R[3] = nan;
    t[0] = t[1] = nan;
    *gap = 0.0;
    return false;
  }
  const double det = det2_lu(S);
  *gap = align_gap(S, det, sv);
  double s1 = (det < 0.0) ? -1.0 : 1.0;
  int rank = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
    if (!(fabs(sv[i]) <= fabs(sv[0]) * 1e-12)) ++rank;
  if (rank == 1) s1 = (det2_lu(U) * det2_lu(V) > 0.0) ? 1.0 : -1.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      R[2 * i + j] = (U[i] * 1.0) * V[j] + (U[i + 2] * s1) * V[j + 2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    double ti = dm[i];
    ti = ti + R[2 * i + 0] * (-sm[0]);
    ti = ti + R[2 * i + 1] * (-sm[1]);
    t[i] = ti;
  }
  return true;
}

// One vehicle that holds its own assignment (acl_solve_args_t::P_rows): its
// row (formation point -> vehicle) is checked to be a permutation with the
// vehicle at its point i, its closed CBAA neighbourhood in vehicle space is
// {row[j] : j = i or adj(i, j)} (bidIterComplete, auctioneer.cpp:419-437,
// with the vehicle's own P_ / Pt_), and Auctioneer::alignFormation (:347-415)
// runs on the members j of formation row i's closed neighbourhood ascending,
// src p_j.xy, dst the q of vehicle row[j] (qxy(u, x, y)). The arithmetic is
// align_chunk's / align_wide_kernel's: sums from -0.0 in ascending order, the
// lazy (k + 4 < 20) or GEMM product form. adjrow: formation row i's words
// (NW of them, masked past n); NWM: the mask arrays' size. Returns false when
// the row is not such a permutation (the swarm is BAD_INPUT).
template <int NWM, class RowAt, class QXY>
__device__ inline bool align_own_row(int n, int NW, int v, int i, const unsigned long long* adjrow,
                                     const double* p, RowAt row, QXY qxy,
                                     unsigned long long (&nb)[NWM], double* o6, double& gap) {
  unsigned long long mem[NWM], seen[NWM];
#pragma unroll
  for (int w = 0; w < NWM; ++w) {
    mem[w] = w < NW ? adjrow[w] : 0ull;
    if (w == (i >> 6)) mem[w] |= 1ull << (i & 63);
    seen[w] = 0ull;
    nb[w] = 0ull;
  }
  bool ok = row(i) == v;
  int k = 0;
  double s0 = -0.0, s1 = -0.0, s2 = -0.0, s3 = -0.0;
  for (int j = 0; j < n; ++j) {
    const int u = row(j);
    const unsigned long long bu = 1ull << (u & 63);
    bool dup = false;
#pragma unroll
    for (int w = 0; w < NWM; ++w)
      if (w == (u >> 6)) {
        dup = (seen[w] & bu) != 0ull;
        seen[w] |= bu;
      }
    ok = ok && u < n && !dup;
    bool m = false;
#pragma unroll
    for (int w = 0; w < NWM; ++w)
      if (w == (j >> 6)) m = ((mem[w] >> (j & 63)) & 1ull) != 0ull;
    if (m && u < n) {
#pragma unroll
      for (int w = 0; w < NWM; ++w)
        if (w == (u >> 6)) nb[w] |= bu;
      double qx, qy;
      qxy(u, qx, qy);
      s0 = s0 + p[3 * j];
      s1 = s1 + p[3 * j + 1];
      s2 = s2 + qx;
      s3 = s3 + qy;
      ++k;
    }
  }
  if (!ok) return false;
  const double oon = 1.0 / (double)k;
  const double sm[2] = {s0 * oon, s1 * oon};
  const double dm[2] = {s2 * oon, s3 * oon};
  const bool lazy = (k + 4) < 20;
  const double z0 = lazy ? -0.0 : 0.0;
  double c0 = z0, c1 = z0, c2 = z0, c3 = z0;
  for (int j = 0; j < n; ++j) {
    bool m = false;
#pragma unroll
    for (int w = 0; w < NWM; ++w)
      if (w == (j >> 6)) m = ((mem[w] >> (j & 63)) & 1ull) != 0ull;
    if (!m) continue;
    double qx, qy;
    qxy(row(j), qx, qy);
    const double e0 = p[3 * j] - sm[0], e1 = p[3 * j + 1] - sm[1];
    double d0 = qx - dm[0], d1 = qy - dm[1];
    if (lazy) {
      d0 = oon * d0;
      d1 = oon * d1;
    }
    c0 = c0 + d0 * e0;
    c1 = c1 + d0 * e1;
    c2 = c2 + d1 * e0;
    c3 = c3 + d1 * e1;
  }
  if (!lazy) {
    c0 = c0 * oon; c1 = c1 * oon; c2 = c2 * oon; c3 = c3 * oon;
  }
  const double S[4] = {c0, c2, c1, c3};
  double R[4], t[2], g;
  umeyama_finish(S, sm, dm, R, t, &g);
  gap = g < gap ? g : gap;
  o6[0] = R[0]; o6[1] = R[1]; o6[2] = R[2]; o6[3] = R[3]; o6[4] = t[0]; o6[5] = t[1];
  return true;
}

}  // namespace acl_amd
