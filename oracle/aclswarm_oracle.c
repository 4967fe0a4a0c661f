/*
 * aclswarm_oracle.c -- CPU restatement of aclswarm's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see aclswarm_oracle.h). Built with
 * -O2 -ffp-contract=off so that every double operation is one IEEE-754
 * rounding, as in the reference's x86-64 (SSE2, no FMA) build.
 *
 * Every function cites the reference lines it restates. "Eigen x.y" comments
 * restate the published algorithm of the unpinned Eigen3 dependency (see
 * DESIGN.md §3 for the version choice and its consequences).
 */
#include "aclswarm_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------------ */
/* Eigen JacobiRotation / JacobiSVD (2x2), Eigen 3.3.4                       */
/* ------------------------------------------------------------------------ */

/* MatrixBase::applyOnTheLeft(p,q,j) on a column-major 2x2: x=row p, y=row q,
 * apply_rotation_in_the_plane: x' = c x + s y, y' = -s x + c y
 * (Eigen/src/Jacobi/Jacobi.h; early return when c==1 && s==0). */
static void rot_rows(double* W, int p, int q, double c, double s) {
  if (c == 1.0 && s == 0.0) return;
  for (int k = 0; k < 2; ++k) {
    const double xi = W[p + 2 * k], yi = W[q + 2 * k];
    W[p + 2 * k] = c * xi + s * yi;
    W[q + 2 * k] = -s * xi + c * yi;
  }
}

/* apply_rotation_in_the_plane on columns p (x) and q (y) with rotation (c,s). */
static void rot_cols(double* M, int p, int q, double c, double s) {
  if (c == 1.0 && s == 0.0) return;
  for (int k = 0; k < 2; ++k) {
    const double xi = M[k + 2 * p], yi = M[k + 2 * q];
    M[k + 2 * p] = c * xi + s * yi;
    M[k + 2 * q] = -s * xi + c * yi;
  }
}

/* JacobiRotation::makeJacobi(x, y, z) for reals. */
static void make_jacobi(double x, double y, double z, double* c, double* s) {
  const double deno = 2.0 * fabs(y);
  if (deno < DBL_MIN) {
    *c = 1.0;
    *s = 0.0;
    return;
  }
  const double tau = (x - z) / deno;
  const double w = sqrt(tau * tau + 1.0);
  double t;
  if (tau > 0.0)
    t = 1.0 / (tau + w);
  else
    t = 1.0 / (tau - w);
  const double sign_t = t > 0.0 ? 1.0 : -1.0;
  const double n = 1.0 / sqrt(t * t + 1.0);
  *s = -sign_t * (y / fabs(y)) * fabs(t) * n;
  *c = n;
}

/* internal::real_2x2_jacobi_svd(W, p=1, q=0, &j_left, &j_right)
 * (Eigen/src/misc/RealSvd2x2.h). */
static void real_2x2_jacobi_svd(const double* W, double* cl, double* sl,
                                double* cr, double* sr) {
  /* m << W(p,p), W(p,q), W(q,p), W(q,q) with p=1, q=0 (row-major fill) */
  double m[4]; /* column-major 2x2 */
  m[0] = W[3];  /* m(0,0) = W(1,1) */
  m[2] = W[1];  /* m(0,1) = W(1,0) */
  m[1] = W[2];  /* m(1,0) = W(0,1) */
  m[3] = W[0];  /* m(1,1) = W(0,0) */
  double c1, s1;
  const double t = m[0] + m[3];
  const double d = m[1] - m[2];
  if (fabs(d) < DBL_MIN) {
    s1 = 0.0;
    c1 = 1.0;
  } else {
    const double u = t / d;
    const double tmp = sqrt(1.0 + u * u);
    s1 = 1.0 / tmp;
    c1 = u / tmp;
  }
  rot_rows(m, 0, 1, c1, s1);
  make_jacobi(m[0], m[2], m[3], cr, sr);
  /* j_left = rot1 * j_right.transpose(); j_right^T = (cr, -sr) */
  const double ocs = -*sr;
  *cl = c1 * (*cr) - s1 * ocs;
  *sl = c1 * ocs + s1 * (*cr);
}

/* LU-based determinant of a dynamic 2x2 (PartialPivLU::determinant). */
static double det2_lu(const double* A /* column-major */) {
  double a00 = A[0], a10 = A[1], a01 = A[2], a11 = A[3];
  double sign = 1.0;
  /* maxCoeff(&row) of |col 0|: first index of the maximum */
  const double b0 = fabs(a00), b1 = fabs(a10);
  const int piv = (b1 > b0) ? 1 : 0;
  const double biggest = piv ? b1 : b0;
  if (biggest != 0.0) {
    if (piv) {
      double t;
      t = a00; a00 = a10; a10 = t;
      t = a01; a01 = a11; a11 = t;
      sign = -1.0;
    }
    a10 = a10 / a00;
  }
  a11 = a11 - a10 * a01;
  return (a00 * a11) * sign;
}

int orc_jacobi_svd2(const double A[4], double U[4], double sv[2],
                    double V[4]) {
  /* JacobiSVD::compute, Eigen 3.3.4 */
  const double precision = 2.0 * DBL_EPSILON;
  const double considerAsZero = DBL_MIN;
  double scale = fabs(A[0]);
  for (int i = 1; i < 4; ++i) {
    const double a = fabs(A[i]);
    if (a > scale || isnan(a)) scale = a;
  }
  if (!isfinite(scale)) return -1;
  if (scale == 0.0) scale = 1.0;
  double W[4];
  for (int i = 0; i < 4; ++i) W[i] = A[i] / scale;
  U[0] = 1.0; U[1] = 0.0; U[2] = 0.0; U[3] = 1.0;
  V[0] = 1.0; V[1] = 0.0; V[2] = 0.0; V[3] = 1.0;
  double maxDiag = fabs(W[0]);
  if (maxDiag < fabs(W[3])) maxDiag = fabs(W[3]);
  int finished = 0;
  while (!finished) {
    finished = 1;
    /* the only (p,q) pair of a 2x2: p=1, q=0 */
    double threshold = precision * maxDiag;
    if (threshold < considerAsZero) threshold = considerAsZero;
    if (fabs(W[1]) > threshold || fabs(W[2]) > threshold) {
      finished = 0;
      double cl, sl, cr, sr;
      real_2x2_jacobi_svd(W, &cl, &sl, &cr, &sr);
      rot_rows(W, 1, 0, cl, sl);    /* W.applyOnTheLeft(1,0,j_left) */
      rot_cols(U, 1, 0, cl, sl);    /* U.applyOnTheRight(1,0,j_left^T) */
      rot_cols(W, 1, 0, cr, -sr);   /* W.applyOnTheRight(1,0,j_right) */
      rot_cols(V, 1, 0, cr, -sr);   /* V.applyOnTheRight(1,0,j_right) */
      double md = fabs(W[3]);
      if (md < fabs(W[0])) md = fabs(W[0]);
      if (maxDiag < md) maxDiag = md;
    }
  }
  for (int i = 0; i < 2; ++i) {
    const double a = W[i * 3]; /* W(i,i) */
    sv[i] = fabs(a);
    if (a < 0.0) {
      U[2 * i] = -U[2 * i];
      U[2 * i + 1] = -U[2 * i + 1];
    }
  }
  sv[0] *= scale;
  sv[1] *= scale;
  /* sort descending (step 4) */
  {
    const int pos = (sv[1] > sv[0]) ? 1 : 0;
    const double mx = pos ? sv[1] : sv[0];
    if (mx != 0.0 && pos) {
      double t = sv[0]; sv[0] = sv[1]; sv[1] = t;
      for (int k = 0; k < 2; ++k) {
        t = U[k]; U[k] = U[2 + k]; U[2 + k] = t;
        t = V[k]; V[k] = V[2 + k]; V[2 + k] = t;
      }
    }
  }
  return 0;
}

/* Decision gaps of the alignment's two sign/rank tests (the margin of
 * include/aclswarm_amd.h): |det S| / (|S00 S11| + |S01 S10|) for the
 * determinant sign, |s1 - 1e-12 s0| / max(s1, 1e-12 s0) for the rank. */
static double align_gap(const double S[4], double det, const double sv[2]) {
  const double den = fabs(S[0] * S[3]) + fabs(S[2] * S[1]);
  double g = (den > 0.0) ? fabs(det) / den : 0.0;
  if (!(g <= 1.0)) g = (g > 1.0) ? 1.0 : 0.0;
  const double th = fabs(sv[0]) * 1e-12, a = fabs(sv[1]);
  const double mx = (a > th) ? a : th;
  const double gr = (mx > 0.0) ? fabs(a - th) / mx : 0.0;
  return (gr < g) ? gr : g;
}

int orc_umeyama2(int k, const double* src, const double* dst, double R[4],
                 double t[2], int variant) {
  return orc_umeyama2_gap(k, src, dst, R, t, variant, NULL);
}

int orc_umeyama2_gap(int k, const double* src, const double* dst, double R[4],
                     double t[2], int variant, double* gap) {
  /* Eigen::umeyama(src, dst, false), Eigen/src/Geometry/Umeyama.h (3.3.4),
   * Dimension = Dynamic since pp.topRows(d) has a runtime row count. */
  const double one_over_n = 1.0 / (double)k;
  double sm[2], dm[2];
  for (int r = 0; r < 2; ++r) {
    double a = src[r], b = dst[r];
    for (int i = 1; i < k; ++i) {
      a = a + src[2 * i + r];
      b = b + dst[2 * i + r];
    }
    sm[r] = a * one_over_n;
    dm[r] = b * one_over_n;
  }
  /* sigma = one_over_n * dst_demean * src_demean^T (2x2). Eigen evaluates it
   * lazily (scaled lhs, coefficient-wise) when k + 4 < 20, otherwise by GEMM
   * (alpha applied to the accumulated sum). */
  double S[4]; /* column-major */
  for (int i = 0; i < 2; ++i) {
    for (int j = 0; j < 2; ++j) {
      double acc = 0.0;
      if (k + 4 < 20) {
        for (int kk = 0; kk < k; ++kk) {
          const double a = one_over_n * (dst[2 * kk + i] - dm[i]);
          const double b = src[2 * kk + j] - sm[j];
          acc = (kk == 0) ? a * b : acc + a * b;
        }
        S[i + 2 * j] = acc;
      } else {
        for (int kk = 0; kk < k; ++kk) {
          const double a = dst[2 * kk + i] - dm[i];
          const double b = src[2 * kk + j] - sm[j];
          acc = acc + a * b;
        }
        S[i + 2 * j] = acc * one_over_n;
      }
    }
  }
  double U[4], V[4], sv[2];
  if (gap) *gap = 0.0;
  if (orc_jacobi_svd2(S, U, sv, V) != 0) {
    R[0] = R[1] = R[2] = R[3] = NAN;
    t[0] = t[1] = NAN;
    return -1;
  }
  double s1 = 1.0;
  if (variant == 1) {
    /* Eigen 3.4: S(m-1) = -1 iff det(U) det(V) < 0 (orthogonal factors,
     * determinants +-1: no near-tie to track, the gap is 1) */
    if (gap) *gap = 1.0;
    if (det2_lu(U) * det2_lu(V) < 0.0) s1 = -1.0;
  } else {
    /* Eigen 3.3.x: S from det(sigma); rank-deficient branch */
    const double det = det2_lu(S);
    if (gap) *gap = align_gap(S, det, sv);
    if (det < 0.0) s1 = -1.0;
    int rank = 0;
    for (int i = 0; i < 2; ++i)
      if (!(fabs(sv[i]) <= fabs(sv[0]) * 1e-12)) ++rank;
    if (rank == 1) s1 = (det2_lu(U) * det2_lu(V) > 0.0) ? 1.0 : -1.0;
  }
  /* R = U * diag(1, s1) * V^T, coefficient-wise (a0*b0) + (a1*b1) */
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      R[2 * i + j] = (U[i] * 1.0) * V[j] + (U[i + 2] * s1) * V[j + 2];
  /* t = dst_mean; t -= R * src_mean (column-major GEMV, alpha = -1) */
  for (int i = 0; i < 2; ++i) {
    double ti = dm[i];
    ti = ti + R[2 * i + 0] * (-sm[0]);
    ti = ti + R[2 * i + 1] * (-sm[1]);
    t[i] = ti;
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Auctioneer                                                                */
/* ------------------------------------------------------------------------ */

static void invert_perm(int n, const uint16_t* P, uint16_t* Pt) {
  for (int i = 0; i < n; ++i) Pt[P[i]] = (uint16_t)i;
}

static int is_perm(int n, const uint16_t* P) {
  unsigned char* seen = (unsigned char*)calloc((size_t)n, 1);
  int ok = 1;
  for (int i = 0; i < n && ok; ++i) {
    if (P[i] >= n || seen[P[i]]) ok = 0;
    else seen[P[i]] = 1;
  }
  free(seen);
  return ok;
}

void orc_align(int n, int v, const double* q, const double* p,
               const uint8_t* adj, const uint16_t* P, double R[4],
               double t[2]) {
  orc_align_gap(n, v, q, p, adj, P, R, t, NULL);
}

/* The Eigen version whose umeyama rule the vehicle alignments follow (SURVEY
 * App. B; the reference pins none): 0 = 3.3.x (the default, the GPU's rule),
 * 1 = 3.4. A process-wide switch for the version-risk measurement
 * (scripts/eigen_variant_risk.py); set it before any solve runs. */
static int g_umeyama_variant = 0;
void orc_set_umeyama_variant(int variant) { g_umeyama_variant = variant ? 1 : 0; }
int orc_get_umeyama_variant(void) { return g_umeyama_variant; }

void orc_align_gap(int n, int v, const double* q, const double* p,
                   const uint8_t* adj, const uint16_t* P, double R[4],
                   double t[2], double* gap) {
  /* auctioneer.cpp:347-415. Formation space: i = P[v]; neighbourhood
   * {j : adj(i,j) || i == j} ascending; p rows j, q rows Pt[j]. */
  uint16_t* Pt = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)n);
  invert_perm(n, P, Pt);
  const int i = P[v];
  double* src = (double*)malloc(sizeof(double) * 2 * (size_t)n);
  double* dst = (double*)malloc(sizeof(double) * 2 * (size_t)n);
  int k = 0;
  for (int j = 0; j < n; ++j) {
    if (adj[(size_t)i * n + j] || i == j) {
      src[2 * k] = p[3 * j];
      src[2 * k + 1] = p[3 * j + 1];
      dst[2 * k] = q[3 * Pt[j]];
      dst[2 * k + 1] = q[3 * Pt[j] + 1];
      ++k;
    }
  }
  orc_umeyama2_gap(k, src, dst, R, t, g_umeyama_variant, gap);
  free(src);
  free(dst);
  free(Pt);
}

void orc_prices(int n, const double* q, const double* p, const uint8_t* adj,
                const uint16_t* P, float* C, double* Rt) {
  orc_prices_gap(n, q, p, adj, P, C, Rt, NULL);
}

void orc_prices_gap(int n, const double* q, const double* p, const uint8_t* adj,
                    const uint16_t* P, float* C, double* Rt, double* gap_min) {
  orc_prices_rows(n, q, p, adj, P, NULL, C, Rt, gap_min);
}

void orc_prices_rows(int n, const double* q, const double* p, const uint8_t* adj,
                     const uint16_t* P, const uint16_t* Prows, float* C, double* Rt,
                     double* gap_min) {
  /* Prows (optional [n][n]): vehicle v aligns with its own assignment, the
   * inverse of its row (auctioneer.cpp:357,369: P_, Pt_ are the vehicle's) */
  uint16_t* Pv = Prows ? (uint16_t*)malloc(sizeof(uint16_t) * (size_t)n) : NULL;
  if (gap_min) *gap_min = 1.0;
  for (int v = 0; v < n; ++v) {
    double R[4], t[2], g = 1.0;
    if (Pv) invert_perm(n, Prows + (size_t)v * n, Pv);
    orc_align_gap(n, v, q, p, adj, Pv ? Pv : P, R, t, &g);
    if (gap_min && g < *gap_min) *gap_min = g;
    if (Rt) {
      Rt[6 * v + 0] = R[0]; Rt[6 * v + 1] = R[1];
      Rt[6 * v + 2] = R[2]; Rt[6 * v + 3] = R[3];
      Rt[6 * v + 4] = t[0]; Rt[6 * v + 5] = t[1];
    }
    const double qx = q[3 * v], qy = q[3 * v + 1], qz = q[3 * v + 2];
    for (int j = 0; j < n; ++j) {
      const double px = p[3 * j], py = p[3 * j + 1], pz = p[3 * j + 2];
      /* aligned = ((R*p^T).colwise() + t)^T with R = [R2 0; 0 0 1] */
      const double ax = ((R[0] * px + R[1] * py) + 0.0 * pz) + t[0];
      const double ay = ((R[2] * px + R[3] * py) + 0.0 * pz) + t[1];
      const double az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0;
      /* getPrice (auctioneer.cpp:546-549): 1/(||p1-p2|| + 1e-8) -> float */
      const double dx = qx - ax, dy = qy - ay, dz = qz - az;
      const double nrm = sqrt((dx * dx + dy * dy) + dz * dz);
      C[(size_t)v * n + j] = (float)(1.0 / (nrm + 1e-8));
    }
  }
  free(Pv);
}

/* Decision-margin tracker (include/aclswarm_amd.h): the compared pair
 * (hi, lo), hi >= lo >= 0, with the largest ratio lo / hi, ranked exactly
 * (products of two floats are exact in double). A tie (lo == hi) is the
 * largest ratio, 1. */
void orc_margin_track(float* m, float hi, float lo) {
  if (!(lo < hi)) {
    if (lo == hi) { m[0] = 1.0f; m[1] = 1.0f; }
    return; /* NaN: the swarm is NONFINITE, margin 0 */
  }
  if ((double)lo * (double)m[0] > (double)m[1] * (double)hi) {
    m[0] = hi;
    m[1] = lo;
  }
}

/* Gap of the tracked pair: (hi - lo) / hi in double, 1 when lo < 2^-28 hi
 * (where hi - lo is exact in double the gap is monotone in the ratio). */
double orc_margin_gap(const float* m) {
  const double hi = m[0], lo = m[1];
  if (lo * 268435456.0 < hi) return 1.0;
  return (hi - lo) / hi;
}

/* selectTaskAssignment (auctioneer.cpp:517-542), plus the margin of its
 * decisive comparisons (include/aclswarm_amd.h) when m != NULL */
static void cbaa_select(int n, int v, const float* C, int32_t* who,
                        float* price, float* m) {
  float max = 0.0f;
  int task = 0, assigned = 0;
  for (int j = 0; j < n; ++j) {
    const float c = C[(size_t)v * n + j];
    if (c > max && c > price[j]) {
      max = c;
      task = j;
      assigned = 1;
    }
  }
  if (m) {
    const int js = assigned ? task : -1;
    for (int k = 0; k < n; ++k) {
      if (who[k] == v) continue; /* compared with itself */
      const float c = C[(size_t)v * n + k];
      if (k == js) {
        orc_margin_track(m, c, price[k]);
      } else if (c > price[k] && c > 0.0f) {
        orc_margin_track(m, max, c); /* an eligible task that lost */
      } else if (c > 0.0f && (js < 0 || c > max || (c == max && k < js))) {
        orc_margin_track(m, price[k], c); /* would win if it became eligible */
      }
    }
  }
  if (assigned) {
    price[task] = max;
    who[task] = v;
  }
}

int orc_cbaa(int n, const float* C, const uint8_t* adj, const uint16_t* P,
             int early_exit, int32_t* who_out, float* price_out) {
  return orc_cbaa_m(n, C, adj, P, early_exit, who_out, price_out, NULL);
}

int orc_cbaa_m(int n, const float* C, const uint8_t* adj, const uint16_t* P,
               int early_exit, int32_t* who_out, float* price_out, float* m) {
  return orc_cbaa_rows(n, C, adj, P, NULL, early_exit, who_out, price_out, m);
}

int orc_cbaa_rows(int n, const float* C, const uint8_t* adj, const uint16_t* P,
                  const uint16_t* Prows, int early_exit, int32_t* who_out,
                  float* price_out, float* m) {
  const size_t nn = (size_t)n * n;
  int32_t* who = (int32_t*)malloc(sizeof(int32_t) * nn);
  int32_t* who2 = (int32_t*)malloc(sizeof(int32_t) * nn);
  float* pr = (float*)malloc(sizeof(float) * nn);
  float* pr2 = (float*)malloc(sizeof(float) * nn);
  int* nb = (int*)malloc(sizeof(int) * nn);
  int* deg = (int*)malloc(sizeof(int) * (size_t)n);
  if (m) { m[0] = 1.0f; m[1] = 0.0f; }
  /* Closed neighbourhood in vehicle space, ascending vehid = std::map order
   * of bids_curr_ (auctioneer.cpp:419-437, 480): u is a neighbour of v iff
   * adj(P[v], P[u]) (u = Pt[j] <=> j = P[u]), plus v itself. */
  /* Prows (optional): v's neighbours come from its own assignment, the
   * inverse of its row (bidIterComplete uses the vehicle's P_ and Pt_) */
  uint16_t* Pv = Prows ? (uint16_t*)malloc(sizeof(uint16_t) * (size_t)n) : NULL;
  for (int v = 0; v < n; ++v) {
    const uint16_t* Pw = P;
    if (Pv) {
      invert_perm(n, Prows + (size_t)v * n, Pv);
      Pw = Pv;
    }
    int d = 0;
    for (int u = 0; u < n; ++u)
      if (u == v || adj[(size_t)Pw[v] * n + Pw[u]]) nb[(size_t)v * n + d++] = u;
    deg[v] = d;
  }
  free(Pv);
  /* reset (auctioneer.cpp:448-465) and the START bid (round 0) */
  for (size_t k = 0; k < nn; ++k) {
    who[k] = ORC_NONE;
    pr[k] = 0.0f;
  }
  for (int v = 0; v < n; ++v)
    cbaa_select(n, v, C, who + (size_t)v * n, pr + (size_t)v * n, m);
  const int max_iter = n * 2; /* cbaa_max_iter_ = n * diameter (:50-51) */
  int eff = 0;
  for (int r = 1; r <= max_iter; ++r) {
    for (int v = 0; v < n; ++v) {
      /* updateTaskAssignment (auctioneer.cpp:469-513) */
      const int* nbv = nb + (size_t)v * n;
      int outbid = 0;
      for (int j = 0; j < n; ++j) {
        int maxit = nbv[0];
        for (int a = 0; a < deg[v]; ++a) {
          const int u = nbv[a];
          if (pr[(size_t)u * n + j] > pr[(size_t)maxit * n + j]) maxit = u;
        }
        const int32_t wnew = who[(size_t)maxit * n + j];
        if (m) {
          /* margin: the winning price vs the best price of another `who` */
          const float p1 = pr[(size_t)maxit * n + j];
          int have = 0;
          float p2 = 0.0f;
          for (int a = 0; a < deg[v]; ++a) {
            const int u = nbv[a];
            if (who[(size_t)u * n + j] == wnew) continue;
            const float px = pr[(size_t)u * n + j];
            if (!have || px > p2) p2 = px;
            have = 1;
          }
          if (have) orc_margin_track(m, p1, p2);
        }
        if (who[(size_t)v * n + j] == v && wnew != v) outbid = 1;
        who2[(size_t)v * n + j] = wnew;
        pr2[(size_t)v * n + j] = pr[(size_t)maxit * n + j];
      }
      if (outbid)
        cbaa_select(n, v, C, who2 + (size_t)v * n, pr2 + (size_t)v * n, m);
    }
    const int changed = memcmp(who, who2, sizeof(int32_t) * nn) != 0 ||
                        memcmp(pr, pr2, sizeof(float) * nn) != 0;
    memcpy(who, who2, sizeof(int32_t) * nn);
    memcpy(pr, pr2, sizeof(float) * nn);
    if (changed)
      eff = r;
    else if (early_exit)
      break; /* fixed point: rounds r+1..2N are identical */
  }
  if (who_out) memcpy(who_out, who, sizeof(int32_t) * nn);
  if (price_out) memcpy(price_out, pr, sizeof(float) * nn);
  free(who); free(who2); free(pr); free(pr2); free(nb); free(deg);
  return eff;
}

/* ------------------------------------------------------------------------ */
/* DistCntrl                                                                 */
/* ------------------------------------------------------------------------ */

void orc_pdist(int n, const double* p, double* dxy, double* dz) {
  /* utils::pdistmat (utils.h:137-147): D = N 1^T + 1 N^T - 2 M M^T, sqrt */
  for (int i = 0; i < n; ++i) {
    const double xi = p[3 * i], yi = p[3 * i + 1], zi = p[3 * i + 2];
    const double Ni = xi * xi + yi * yi, Nzi = zi * zi;
    for (int j = 0; j < n; ++j) {
      const double xj = p[3 * j], yj = p[3 * j + 1], zj = p[3 * j + 2];
      const double Nj = xj * xj + yj * yj, Nzj = zj * zj;
      const double dot = xi * xj + yi * yj;
      dxy[(size_t)i * n + j] = sqrt((Ni + Nj) - 2.0 * dot);
      dz[(size_t)i * n + j] = sqrt((Nzi + Nzj) - 2.0 * (zi * zj));
    }
  }
}

void orc_control(int n, int v, const double* q, const double* vel_v,
                 const uint16_t* Pt, const uint8_t* adj, const double* gains,
                 const double* dxy, const double* dz,
                 const acl_cntrl_gains_t* g, double u[3]) {
  orc_control_g(n, v, q, vel_v, Pt, adj, gains, dxy, dz, g, u, NULL);
}

void orc_control_g(int n, int v, const double* q, const double* vel_v,
                   const uint16_t* Pt, const uint8_t* adj, const double* gains,
                   const double* dxy, const double* dz,
                   const acl_cntrl_gains_t* g, double u[3], double* gate_min) {
  /* DistCntrl::compute (distcntrl.cpp:46-102); gate_min (optional) takes the
   * minimum of | |e| - thr | / thr over the two gates of every edge */
  int i = 0;
  while (Pt[i] != v) ++i; /* i = P[v] */
  const size_t ld = (size_t)3 * n;
  u[0] = u[1] = u[2] = 0.0;
  const double* qi = q + 3 * Pt[i];
  for (int j = 0; j < n; ++j) {
    if (!adj[(size_t)i * n + j]) continue;
    const double* qj = q + 3 * Pt[j];
    const double qij[3] = {qj[0] - qi[0], qj[1] - qi[1], qj[2] - qi[2]};
    const double e_xy =
        sqrt(qij[0] * qij[0] + qij[1] * qij[1]) - dxy[(size_t)i * n + j];
    const double e_z = sqrt(qij[2] * qij[2]) - dz[(size_t)i * n + j];
    double F[3] = {0.0, 0.0, 0.0};
    if (gate_min) {
      const double gx = fabs(fabs(e_xy) - g->e_xy_thr) / g->e_xy_thr;
      const double gz = fabs(fabs(e_z) - g->e_z_thr) / g->e_z_thr;
      if (gx < *gate_min) *gate_min = gx;
      if (gz < *gate_min) *gate_min = gz;
    }
    if (fabs(e_xy) > g->e_xy_thr) F[0] = F[1] = g->K1_xy * atan(g->K2_xy * e_xy);
    if (fabs(e_z) > g->e_z_thr) F[2] = g->K1_z * atan(g->K2_z * e_z);
    for (int r = 0; r < 3; ++r) {
      const double* A = gains + (3 * (size_t)i + r) * ld + 3 * (size_t)j;
      const double prod = (A[0] * qij[0] + A[1] * qij[1]) + A[2] * qij[2];
      const double up = prod + F[r] * qij[r];
      const double ud = -vel_v[r];
      u[r] = u[r] + (g->kp * up + g->kd * ud);
    }
  }
}

/* ------------------------------------------------------------------------ */
/* Safety                                                                    */
/* ------------------------------------------------------------------------ */

void orc_saturate(const acl_safety_params_t* s, double g[3]) {
  /* Safety::cmdinCb (safety.cpp:185-196) */
  const double velxy = sqrt(g[0] * g[0] + g[1] * g[1]);
  if (velxy > s->max_vel_xy) {
    g[0] = g[0] / velxy * s->max_vel_xy;
    g[1] = g[1] / velxy * s->max_vel_xy;
  }
  const double velz = fabs(g[2]);
  if (velz > s->max_vel_z) g[2] = g[2] / velz * s->max_vel_z;
}

static double wrap_to_pi(double a) { /* utils::wrapToPi (utils.h:275-280) */
  if (a > M_PI) return a - 2 * M_PI;
  if (a < -M_PI) return a + 2 * M_PI;
  return a;
}

typedef struct {
  double a;
  int s;
} orc_edge_t;

static int edge_cmp(const void* x, const void* y) { /* std::pair operator< */
  const orc_edge_t* e = (const orc_edge_t*)x;
  const orc_edge_t* f = (const orc_edge_t*)y;
  if (e->a < f->a) return -1;
  if (f->a < e->a) return 1;
  return (e->s > f->s) - (e->s < f->s);
}

static int dbl_cmp(const void* x, const void* y) {
  const double a = *(const double*)x, b = *(const double*)y;
  return (a > b) - (a < b);
}

int orc_collision_avoidance(int n, int v, const double* q,
                            const acl_safety_params_t* s, double g[3]) {
  /* Safety::collisionAvoidance (safety.cpp:412-541) */
  int didWrap = 0, modified = 0;
  orc_edge_t* edges = (orc_edge_t*)malloc(sizeof(orc_edge_t) * 4 * (size_t)n + 4);
  int ne = 0;
  for (int j = 0; j < n; ++j) {
    if (v == j) continue;
    const double qx = q[3 * j] - q[3 * v], qy = q[3 * j + 1] - q[3 * v + 1];
    const double d = sqrt(qx * qx + qy * qy);
    if (d > s->d_avoid_thresh) continue;
    const double theta = atan2(qy, qx);
    const double x = s->r_keep_out / d;
    const double ratio = (x < 1.0) ? x : 1.0; /* std::min(1.0, x) */
    const double alpha = fabs(asin(ratio));
    const double beg = wrap_to_pi(theta - alpha);
    const double end = wrap_to_pi(theta + alpha);
    edges[ne].a = beg; edges[ne++].s = +1;
    edges[ne].a = end; edges[ne++].s = -1;
    if (beg > end) {
      didWrap = 1;
      edges[ne].a = -M_PI; edges[ne++].s = +1;
      edges[ne].a = M_PI; edges[ne++].s = -1;
    }
  }
  if (ne == 0) {
    free(edges);
    return 0;
  }
  qsort(edges, (size_t)ne, sizeof(orc_edge_t), edge_cmp);
  double* zs = (double*)malloc(sizeof(double) * 2 * (size_t)ne);
  int nz = 0, count = 0;
  double start = 0.0;
  for (int k = 0; k < ne; ++k) {
    if (count == 0) start = edges[k].a;
    count += edges[k].s;
    if (count == 0) {
      zs[2 * nz] = start;
      zs[2 * nz + 1] = edges[k].a;
      ++nz;
    }
  }
  const double psi = atan2(g[1], g[0]);
  int safe = 1;
  for (int k = 0; k < nz; ++k)
    if (psi > zs[2 * k] && psi < zs[2 * k + 1]) {
      safe = 0;
      break;
    }
  if (!safe) {
    modified = 1;
    double* ze = (double*)malloc(sizeof(double) * 2 * (size_t)nz + 1);
    int m = 0;
    for (int k = 0; k < nz; ++k) {
      if (!didWrap || fabs(zs[2 * k]) != (double)M_PI) ze[m++] = zs[2 * k];
      if (!didWrap || fabs(zs[2 * k + 1]) != (double)M_PI) ze[m++] = zs[2 * k + 1];
    }
    if (m == 0) {
      g[0] = g[1] = 0.0;
      g[2] = 0.0;
    } else {
      qsort(ze, (size_t)m, sizeof(double), dbl_cmp);
      /* utils::closest (utils.h:308-325) via std::lower_bound */
      int it = 0;
      while (it < m && ze[it] < psi) ++it;
      int idx;
      if (it == 0)
        idx = 0;
      else if (it == m || fabs(ze[it - 1] - psi) < fabs(ze[it] - psi))
        idx = it - 1;
      else
        idx = it;
      const double edge = ze[idx];
      if (fabs(wrap_to_pi(edge - psi)) <= M_PI / 2) {
        const double umag = sqrt(g[0] * g[0] + g[1] * g[1]);
        g[0] = umag * cos(edge);
        g[1] = umag * sin(edge);
      } else {
        g[0] = g[1] = 0.0;
        g[2] = 0.0;
      }
    }
    free(ze);
  }
  free(zs);
  free(edges);
  return modified;
}

/* ------------------------------------------------------------------------ */
/* One solve                                                                 */
/* ------------------------------------------------------------------------ */

void orc_solve(int n, const double* q, const double* vel, const double* p,
               const uint8_t* adj, const double* gains, const uint16_t* P_in,
               const acl_cntrl_gains_t* g, const acl_safety_params_t* s,
               int early_exit, uint16_t* P_out, acl_swarm_status_t* st,
               double* u, double* u_safe, uint8_t* ca, uint16_t* who_out) {
  orc_solve_g(n, q, vel, p, adj, gains, P_in, g, s, early_exit, P_out, st, u, u_safe, ca,
              who_out, NULL);
}

/* 1: orc_solve skips the decision-margin bookkeeping (the CPU baseline
 * times the reference's work only; the margin is then reported as 1). */
static __thread int orc_no_margin = 0;

void orc_solve_g(int n, const double* q, const double* vel, const double* p,
                 const uint8_t* adj, const double* gains, const uint16_t* P_in,
                 const acl_cntrl_gains_t* g, const acl_safety_params_t* s,
                 int early_exit, uint16_t* P_out, acl_swarm_status_t* st,
                 double* u, double* u_safe, uint8_t* ca, uint16_t* who_out,
                 double* gate_margin) {
  orc_solve_rows(n, q, vel, p, adj, gains, P_in, NULL, g, s, early_exit, P_out, st, u,
                 u_safe, ca, who_out, gate_margin);
}

/* every row of Prows a permutation that puts its vehicle at its P_in point */
static int rows_ok(int n, const uint16_t* P_in, const uint16_t* Prows) {
  for (int v = 0; v < n; ++v) {
    const uint16_t* r = Prows + (size_t)v * n;
    if (!is_perm(n, r) || r[P_in[v]] != v) return 0;
  }
  return 1;
}

void orc_solve_rows(int n, const double* q, const double* vel, const double* p,
                    const uint8_t* adj, const double* gains, const uint16_t* P_in,
                    const uint16_t* Prows, const acl_cntrl_gains_t* g,
                    const acl_safety_params_t* s, int early_exit, uint16_t* P_out,
                    acl_swarm_status_t* st, double* u, double* u_safe, uint8_t* ca,
                    uint16_t* who_out, double* gate_margin) {
  const size_t nn = (size_t)n * n;
  if (gate_margin) *gate_margin = INFINITY;
  memset(st, 0, sizeof(*st));
  st->rounds = (uint16_t)(2 * n);
  if (!is_perm(n, P_in) || (Prows && !rows_ok(n, P_in, Prows))) {
    st->flags = ACL_SWARM_BAD_INPUT;
    st->margin = 1.0f; /* nothing compared */
    for (int v = 0; v < n; ++v) {
      P_out[v] = P_in[v];
      for (int r = 0; r < 3; ++r) {
        if (u) u[3 * v + r] = 0.0;
        if (u_safe) u_safe[3 * v + r] = 0.0;
      }
      if (ca) ca[v] = 0;
    }
    if (who_out)
      for (size_t k = 0; k < nn; ++k) who_out[k] = 0xFFFF;
    return;
  }
  float* C = (float*)malloc(sizeof(float) * nn);
  int32_t* who = (int32_t*)malloc(sizeof(int32_t) * nn);
  uint16_t* Pt_in = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)n);
  uint16_t* Pt_v = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)n);
  double* dxy = (double*)malloc(sizeof(double) * nn);
  double* dz = (double*)malloc(sizeof(double) * nn);
  invert_perm(n, P_in, Pt_in);
  double gmin = 1.0;
  orc_prices_rows(n, q, p, adj, P_in, Prows, C, NULL, &gmin);
  uint32_t flags = 0;
  for (size_t k = 0; k < nn; ++k)
    if (isnan(C[k])) flags |= ACL_SWARM_NONFINITE;
  float mpair[2] = {1.0f, 0.0f};
  st->eff_rounds = (uint16_t)orc_cbaa_rows(n, C, adj, P_in, Prows, early_exit, who, NULL,
                                           orc_no_margin ? NULL : mpair);
  {
    const double gc = orc_margin_gap(mpair);
    if (gc < gmin) gmin = gc;
    if (flags & ACL_SWARM_NONFINITE) gmin = 0.0;
    st->margin = (float)gmin;
    if (gmin < ACL_FRAGILE_MARGIN) flags |= ACL_SWARM_FRAGILE;
  }
  if (who_out)
    for (size_t k = 0; k < nn; ++k) who_out[k] = (uint16_t)who[k];
  int n_invalid = 0, agree = 1, changed = 0, n_ca = 0;
  for (int v = 1; v < n && agree; ++v)
    if (memcmp(who, who + (size_t)v * n, sizeof(int32_t) * (size_t)n)) agree = 0;
  orc_pdist(n, p, dxy, dz);
  for (int v = 0; v < n; ++v) {
    /* isValidAssignment on the uint8 cast of `who` (auctioneer.cpp:255,325) */
    const int32_t* w = who + (size_t)v * n;
    int valid = 1;
    for (int j = 0; j < n && valid; ++j)
      if (w[j] < 0 || w[j] >= n) valid = 0;
    if (valid) {
      for (int j = 0; j < n; ++j) Pt_v[j] = (uint16_t)w[j];
      valid = is_perm(n, Pt_v);
    }
    if (!valid) {  /* the vehicle keeps its own assignment */
      ++n_invalid;
      memcpy(Pt_v, Prows ? Prows + (size_t)v * n : Pt_in, sizeof(uint16_t) * (size_t)n);
    }
    int i = 0;
    while (Pt_v[i] != v) ++i;
    P_out[v] = (uint16_t)i;
    if (P_out[v] != P_in[v]) changed = 1;
    double cmd[3];
    orc_control_g(n, v, q, vel + 3 * v, Pt_v, adj, gains, dxy, dz, g, cmd, gate_margin);
    if (u) {
      u[3 * v] = cmd[0];
      u[3 * v + 1] = cmd[1];
      u[3 * v + 2] = cmd[2];
    }
    orc_saturate(s, cmd);
    const int mod = orc_collision_avoidance(n, v, q, s, cmd);
    n_ca += mod;
    if (ca) ca[v] = (uint8_t)mod;
    if (u_safe) {
      u_safe[3 * v] = cmd[0];
      u_safe[3 * v + 1] = cmd[1];
      u_safe[3 * v + 2] = cmd[2];
    }
  }
  if (n_invalid == 0) flags |= ACL_SWARM_VALID;
  if (agree) flags |= ACL_SWARM_AGREE;
  if (changed) flags |= ACL_SWARM_CHANGED;
  if (n_ca) flags |= ACL_SWARM_CA_ACTIVE;
  st->flags = flags;
  st->n_invalid = (uint16_t)n_invalid;
  st->n_ca = (uint16_t)n_ca;
  free(C); free(who); free(Pt_in); free(Pt_v); free(dxy); free(dz);
}

/* ------------------------------------------------------------------------ */
/* Thread-pool batch (the CPU baseline)                                      */
/* ------------------------------------------------------------------------ */

typedef struct {
  int B, n, early_exit, with_margin;
  const int32_t* fidx;
  const double *q, *vel, *p, *gains;
  const uint8_t* adj;
  const uint16_t* P_in;
  const acl_cntrl_gains_t* g;
  const acl_safety_params_t* s;
  uint16_t* P_out;
  acl_swarm_status_t* st;
  double *u, *u_safe;
  uint8_t* ca;
  int next;
  pthread_mutex_t mu;
} orc_job_t;

static void* orc_worker(void* arg) {
  orc_job_t* J = (orc_job_t*)arg;
  const size_t n = (size_t)J->n;
  orc_no_margin = !J->with_margin;
  for (;;) {
    pthread_mutex_lock(&J->mu);
    const int b = J->next++;
    pthread_mutex_unlock(&J->mu);
    if (b >= J->B) break;
    const size_t f = (size_t)J->fidx[b];
    orc_solve(J->n, J->q + 3 * n * b, J->vel + 3 * n * b, J->p + 3 * n * f,
              J->adj + n * n * f, J->gains + 9 * n * n * f, J->P_in + n * b,
              J->g, J->s, J->early_exit, J->P_out + n * b, J->st + b,
              J->u ? J->u + 3 * n * b : NULL,
              J->u_safe ? J->u_safe + 3 * n * b : NULL,
              J->ca ? J->ca + n * b : NULL, NULL);
  }
  return NULL;
}

double orc_solve_batch(int B, int n, int nthreads, const int32_t* fidx,
                       const double* q, const double* vel, const double* p,
                       const uint8_t* adj, const double* gains,
                       const uint16_t* P_in, const acl_cntrl_gains_t* g,
                       const acl_safety_params_t* s, int early_exit,
                       uint16_t* P_out, acl_swarm_status_t* st, double* u,
                       double* u_safe, uint8_t* ca, int with_margin) {
  orc_job_t J;
  J.B = B; J.n = n; J.early_exit = early_exit; J.with_margin = with_margin; J.fidx = fidx;
  J.q = q; J.vel = vel; J.p = p; J.gains = gains; J.adj = adj; J.P_in = P_in;
  J.g = g; J.s = s; J.P_out = P_out; J.st = st; J.u = u; J.u_safe = u_safe;
  J.ca = ca; J.next = 0;
  pthread_mutex_init(&J.mu, NULL);
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int k = 0; k < nthreads; ++k) pthread_create(&th[k], NULL, orc_worker, &J);
  for (int k = 0; k < nthreads; ++k) pthread_join(th[k], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  pthread_mutex_destroy(&J.mu);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
