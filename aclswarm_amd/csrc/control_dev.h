// control_dev.h -- device code of the control stage shared by control.hip
// (the gain kernels) and auction.hip (the fused auction + control kernel):
// Safety::cmdinCb saturation and the first collision test, the gate decision
// of DistCntrl::compute (distcntrl.cpp:46-102) and the pair evaluation of one
// swarm's control law (pair_gain_swarm).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/aclswarm_amd.h"
#include "common.h"
#include "control_params.h"

namespace acl_amd {

constexpr int kCtlBlock = 256;
#ifndef ACL_GAIN_WAVES
#define ACL_GAIN_WAVES 6  // waves per SIMD the record-layout gain kernel is built for
#endif
#ifndef ACL_GAIN_FASTMATH
#define ACL_GAIN_FASTMATH 1  // binade-indexed atan and one-step sqrt (about 1e-14 relative)
#endif
#if ACL_GAIN_FASTMATH
#define ACL_GAIN_SQRT sqrt_nr1
#define ACL_GAIN_ATAN acl_atan_b
#define ACL_ATAB_N 170  // kAtanBTab's 34 rows of 5
#define ACL_ATAB_AT(k) kAtanBTab[(k) / 5][(k) % 5]
#else
#define ACL_GAIN_SQRT sqrt_nr
#define ACL_GAIN_ATAN acl_atan_tab
#define ACL_ATAB_N 30
#define ACL_ATAB_AT(k) kAtanTab[(k) / 6][(k) % 6]
#endif
constexpr int kCtlWaves = kCtlBlock / 64;

__host__ __device__ inline int cal16(int x) { return (x + 15) & ~15; }

// Lane segments of the gain kernel: a wave processes G vehicles at once, each
// on S consecutive lanes, in `it` passes (j = s + S t), so that n columns fill
// the 64 lanes well (n = 100: S = 20, G = 3, 5 passes, 94% of the lanes busy,

// Safety::cmdinCb saturation (safety.cpp:185-196)
__device__ __forceinline__ void saturate(const acl_safety_params_t& sp, double& c0, double& c1,
                                         double& c2) {
  const double velxy = sqrt(c0 * c0 + c1 * c1);
  if (velxy > sp.max_vel_xy) {
    c0 = c0 / velxy * sp.max_vel_xy;
    c1 = c1 / velxy * sp.max_vel_xy;
  }
  const double velz = fabs(c2);
  if (velz > sp.max_vel_z) c2 = c2 / velz * sp.max_vel_z;
}

// per vehicle (lanes over vehicles): Safety::cmdinCb saturation and the
// first test of collisionAvoidance -- any other vehicle with
// !(|dq_xy| > d_avoid_thresh)? |dq_xy|^2 above (thr (1 + 2^-40))^2 is far
// for certain, so the sqrt is taken only near the threshold. q: the swarm's
// positions in vehicle order (LDS), uo: DistCntrl's u per vehicle (LDS).
// The close vehicles go to the swarm's mask words (a wave's 64 lanes are the
// vehicles of one word: nthreads is a multiple of 64), and the swarm once to
// the collision list: caw is an LDS word the caller zeroed before a barrier
// that precedes this call (the first wave with a close vehicle appends).
__device__ __forceinline__ void gain_epilogue(const CtlParams& P, int b, int n, const double* q,
                                              const double* uo, unsigned* caw, int tid,
                                              int nthreads = kCtlBlock) {
  const int NW = (n + 63) >> 6;
  const acl_safety_params_t sp = P.s;
  const double thr_hi = sp.d_avoid_thresh * (1.0 + 0x1p-40);
  const double thr2hi = thr_hi * thr_hi;
  for (int v = tid; v < n; v += nthreads) {
    double cmd0 = uo[3 * v], cmd1 = uo[3 * v + 1], cmd2 = uo[3 * v + 2];
    double* gu = P.u + ((size_t)b * n + v) * 3;
    gu[0] = cmd0; gu[1] = cmd1; gu[2] = cmd2;
    saturate(sp, cmd0, cmd1, cmd2);
    const double qv0 = q[3 * v], qv1 = q[3 * v + 1];
    bool near = false;  // any j != v with !(s2 > thr2hi) (NaN included)
    for (int j = 0; j < n; ++j) {
      const double dx = q[3 * j] - qv0, dy = q[3 * j + 1] - qv1;
      near |= (j != v) && !(dx * dx + dy * dy > thr2hi);
    }
    bool close = false;
    if (near) {
      for (int j = 0; j < n; ++j) {
        const double dx = q[3 * j] - qv0, dy = q[3 * j + 1] - qv1;
        const double s2 = dx * dx + dy * dy;
        if (j != v && !(s2 > thr2hi)) close |= !(sqrt(s2) > sp.d_avoid_thresh);
      }
    }
    if (P.u_safe) {
      double* o = P.u_safe + ((size_t)b * n + v) * 3;
      o[0] = cmd0; o[1] = cmd1; o[2] = cmd2;
    }
    if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 0;
    // the rest of collisionAvoidance runs in ca_kernel
    const unsigned long long cm = __ballot(close);
    if ((tid & 63) == 0) {
      P.ca_mask[(size_t)b * NW + (v >> 6)] = cm;
      if (cm && atomicOr(caw, 1u) == 0u) P.ca_list[atomicAdd(P.ca_count, 1u)] = (unsigned)b;
    }
  }
}

// The discrete gates |e| > thr of distcntrl.cpp:75,80 decide whether an
// atan term is added at all, so they are decided on the oracle's arithmetic:
// the fast e (fused multiply-adds, one-step sqrt; error far below 1e-9 at the
// configs' distances) is recomputed with correctly rounded square roots and
// no contraction whenever it lies within 1e-9 of a threshold. Returns the
// two gate decisions; mxy / mz take min | |e| - thr | of each gate (the gate
// margin min(| |e| - thr | / thr) is formed once per swarm by gate_margin_of:
// division by a positive constant is monotone under rounding, so
// fl(min x / thr) = min fl(x / thr) -- two divisions per swarm, not per edge).
#define ACL_GATE_WINDOW 1e-9
template <bool GM>
__device__ __forceinline__ void gate_decide_t(double txy, double tz, double win, double e_xy,
                                              double e_z, double q0, double q1, double q2,
                                              double Ni, double Nj, double Nzi, double Nzj,
                                              double pix, double piy, double piz, double pjx,
                                              double pjy, double pjz, bool& gxy, bool& gz,
                                              double& mxy, double& mz) {
  double axy = fabs(e_xy), az = fabs(e_z);
  const double dxy = fabs(axy - txy), dz = fabs(az - tz);
  if (dxy < win || dz < win) {
#pragma clang fp contract(off)
    const double xy = sqrt(q0 * q0 + q1 * q1) - sqrt((Ni + Nj) - 2.0 * (pix * pjx + piy * pjy));
    const double zz = sqrt(q2 * q2) - sqrt((Nzi + Nzj) - 2.0 * (piz * pjz));
    axy = fabs(xy);
    az = fabs(zz);
  }
  gxy = axy > txy;
  gz = az > tz;
  if (GM) {
    mxy = fmin(mxy, fabs(axy - txy));
    mz = fmin(mz, fabs(az - tz));
  }
}

template <bool GM>
__device__ __forceinline__ void gate_decide(const acl_cntrl_gains_t& g, double e_xy, double e_z,
                                            double q0, double q1, double q2, double Ni, double Nj,
                                            double Nzi, double Nzj, double pix, double piy,
                                            double piz, double pjx, double pjy, double pjz,
                                            bool& gxy, bool& gz, double& mxy, double& mz) {
  double axy = fabs(e_xy), az = fabs(e_z);
  const double dxy = fabs(axy - g.e_xy_thr), dz = fabs(az - g.e_z_thr);
  if (dxy < ACL_GATE_WINDOW || dz < ACL_GATE_WINDOW) {
#pragma clang fp contract(off)
    const double xy = sqrt(q0 * q0 + q1 * q1) - sqrt((Ni + Nj) - 2.0 * (pix * pjx + piy * pjy));
    const double zz = sqrt(q2 * q2) - sqrt((Nzi + Nzj) - 2.0 * (piz * pjz));
    axy = fabs(xy);
    az = fabs(zz);
  }
  gxy = axy > g.e_xy_thr;
  gz = az > g.e_z_thr;
  if (GM) {
    mxy = fmin(mxy, fabs(axy - g.e_xy_thr));
    mz = fmin(mz, fabs(az - g.e_z_thr));
  }
}

// The scale terms' errors of a pair (distcntrl.cpp:67-72): e_xy = |q.xy| -
// dstar_xy, e_z = |q.z| - dstar_z, pdistmat's Gram-formula distances from
// the formation points (utils.h:137-147). The contractions are written out
// (explicit fma), so every kernel that evaluates pairs gets the same bits
// (gate margins are compared exactly between them); s2 = |q.xy|^2.
__device__ __forceinline__ void pair_e(double q0, double q1, double q2, double Ni, double Nj,
                                       double Nzi, double Nzj, double pix, double piy, double piz,
                                       double pjx, double pjy, double pjz, double s2,
                                       double& e_xy, double& e_z) {
  const double dxy = ACL_GAIN_SQRT(__builtin_fma(-2.0, __builtin_fma(pix, pjx, piy * pjy), Ni + Nj));
  const double dz = ACL_GAIN_SQRT(__builtin_fma(-2.0, piz * pjz, Nzi + Nzj));
  e_xy = ACL_GAIN_SQRT(s2) - dxy;
  e_z = fabs(q2) - dz;
}

__device__ __forceinline__ double pair_s2(double q0, double q1) {
  return __builtin_fma(q0, q0, q1 * q1);
}

__device__ __forceinline__ double gate_margin_of(const acl_cntrl_gains_t& g, double mxy, double mz) {
  return fmin(mxy / g.e_xy_thr, mz / g.e_z_thr);
}

// per-swarm gate margin: wave minimum, then the block's minimum through LDS
// (non-negative doubles order like their bits); all lanes active
__device__ __forceinline__ void gate_margin_reduce(unsigned long long* word, double gm) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(gm);
  const unsigned long long m = ~wave_max_u64(~bits);
  if ((threadIdx.x & 63) == 0) atomicMin(word, m);
}

// NP = 9: general 3x3 gain blocks; NP = 5: the ADMM block structure, the four
// structural zeros supplied as constants (acl_formations_t::gain_planes)

// ---- tiled gain records (acl_formations_t::gains_tiled, acl_tile_gains) ----
// Tile t = (I, J), J >= I, row block by row block, is what one wave of
// gain_pair_kernel evaluates: lane = 8r + c takes the pair (8I + r, 8J + c).
// Its records are two runs in lane order: first edge (i, j) of every lane
// (run 1, mask tmask[2t]), then edge (j, i) of every lane (run 2, mask
// tmask[2t + 1]); on a diagonal tile run 1 holds the lanes r <= c and run 2
// the lanes r < c. A lane's record index is then its run's first record
// plus the mask bits below the lane (v_mbcnt).
__host__ __device__ inline int pair_tiles(int n) {
  const int nb = (n + 7) >> 3;
  return nb * (nb + 1) / 2;
}

__device__ __forceinline__ void tile_ij(int t, int nb, int& I, int& J) {
  int rem = t, ii = 0;
  while (rem >= nb - ii) {
    rem -= nb - ii;
    ++ii;
  }
  I = ii;
  J = ii + rem;
}

// block (I, J) of the adjacency, bit 8r + c = adjmat(8I + r, 8J + c); adjF
// rows are masked past n
__device__ __forceinline__ unsigned long long block_mask(const unsigned long long* adjF, int NW,
                                                         int n, int I, int J) {
  unsigned long long m = 0ull;
  const int cw = (8 * J) >> 6, cb = (8 * J) & 63;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int i = 8 * I + r;
    if (i < n) m |= ((adjF[i * NW + cw] >> cb) & 0xFFull) << (8 * r);
  }
  return m;
}

// 8 x 8 bit-matrix transpose (bit 8r + c -> bit 8c + r)
__device__ __forceinline__ unsigned long long transpose8(unsigned long long x) {
  unsigned long long t;
  t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;  x ^= t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull; x ^= t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull; x ^= t ^ (t << 28);
  return x;
}

constexpr unsigned long long kUpperIncl = 0x80C0E0F0F8FCFEFFull;  // bits 8r + c, r <= c

// one wave: tile masks and run offsets (exclusive scan in tile order)
__device__ __forceinline__ void build_tiles(const unsigned long long* adjF, int NW, int n, int lane,
                            unsigned long long* tm, int* ts) {
  const int nb = (n + 7) >> 3, NT = pair_tiles(n);
  int base = 0;
  for (int t0 = 0; t0 < NT; t0 += 64) {
    const int t = t0 + lane;
    int cnt = 0, ca = 0;
    if (t < NT) {
      int I, J;
      tile_ij(t, nb, I, J);
      const unsigned long long b = block_mask(adjF, NW, n, I, J);
      const unsigned long long a = I == J ? (b & kUpperIncl) : b;
      const unsigned long long m2 = I == J ? (transpose8(b) & kUpperIncl & ~0x8040201008040201ull)
                                           : transpose8(block_mask(adjF, NW, n, J, I));
      tm[2 * t] = a;
      tm[2 * t + 1] = m2;
      ca = __popcll(a);
      cnt = ca + __popcll(m2);
    }
    int x = cnt;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (t < NT) {
      ts[2 * t] = base + x - cnt;
      ts[2 * t + 1] = base + x - cnt + ca;
    }
    base += __shfl(x, 63, 64);
  }
}

// DPP move of a double for patterns whose every lane has a source lane
// (quad_perm, row_half_mirror, row_ror): no `old` operand to initialise.
template <int CTRL>
__device__ __forceinline__ double dpp_f64_all(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)u, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// x + (x of lane ^ W), W = 16 or 32, with gfx950's v_permlane{16,32}_swap:
// swapping a copy of x with itself leaves {x[l], x[l ^ W]} in the two
// registers of lane l; their sum is the xor-butterfly step exactly (IEEE
// addition commutes).
template <int W>
__device__ __forceinline__ double swap_sum(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  unsigned a0, a1, b0, b1;
  if constexpr (W == 16) {
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a0 = l[0]; b0 = l[1]; a1 = h[0]; b1 = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a0 = l[0]; b0 = l[1]; a1 = h[0]; b1 = h[1];
  }
  const double a = __longlong_as_double((long long)(((unsigned long long)a1 << 32) | a0));
  const double b = __longlong_as_double((long long)(((unsigned long long)b1 << 32) | b0));
  return a + b;
}

struct PairLayout {
  int q, qf, p, pn, adjF, rowpre, etab, Pt, acc, out, atab, tmask, tstart, gmw, caw, total;
};

__host__ __device__ inline PairLayout make_pair_layout(int n, int kW = kCtlWaves, bool tiled = true) {
  const int NW = (n + 63) >> 6;
  PairLayout L;
  int o = 0;
  L.q = o;      o = cal16(o + n * 3 * 8);            // vehicle order
  L.qf = o;     o = cal16(o + n * 3 * 8);            // formation order: qf[i] = q[Pt[i]]
  L.p = o;      o = cal16(o + n * 3 * 8);
  L.pn = o;     o = cal16(o + n * 2 * 8);
  L.adjF = o;   o = cal16(o + n * NW * 8);
  L.rowpre = o; o = cal16(o + (n * NW + 1) * 4);
  L.etab = o;   // [i][J] record base << 8 | column bits (n <= 128; else edge_idx from adjF)
  o = cal16(o + (n <= kMaxN ? n * ((n + 7) >> 3) * 4 : 0));
  L.Pt = o;     o = cal16(o + n * 2);
  L.acc = o;    o = cal16(o + kW * n * 3 * 8);       // per-wave u partial sums (row order)
  L.out = o;    o = cal16(o + n * 3 * 8);            // u per vehicle
  L.atab = o;   o = cal16(o + ACL_ATAB_N * 8);
  const int NT = (tiled && n <= kMaxN) ? pair_tiles(n) : 0;  // tiled records: n <= 128 only
  L.tmask = o;  o = cal16(o + 2 * NT * 8);
  L.tstart = o; o = cal16(o + 2 * NT * 4);
  L.gmw = o;    o = o + 8;                         // gate margin word
  L.caw = o;    o = cal16(o + 4);                  // the swarm is on the collision list
  L.total = o;
  return L;
}

// ---- pair evaluation of one swarm ---------------------------------------------
//
// The scale terms of distcntrl.cpp:67-83 are symmetric: q_ji = q_i - q_j is
// -q_ij exactly (IEEE subtraction), so |q_ij.xy|, |q_ij.z|, pdistmat's
// Gram-formula distances (sums and products commute) and hence e_xy, e_z and
// the gated atan terms of edge (j, i) equal those of (i, j) bit for bit. The
// pair evaluation computes them once per pair {i, j} and applies both blocks:
// A_ij q_ij + F q_ij to u_i and A_ji q_ji + F q_ji to u_j -- about 60% of the
// fp64 work of the directed walk. For swarms whose vehicles all adopted the
// same assignment (wsMode 0: formation row i is vehicle Pt[i]).
//
// kW waves (threads tid < 64 kW; the caller's other threads, if any, only
// join the barriers) take 8 x 8 tiles (rows I-block x columns J-block,
// J >= I; lane = 8 r + c, pair (8I + r, 8J + c); in diagonal tiles r < c,
// and r == c for a diagonal edge), tile t = wave + kW k. Row sums (over c)
// and column sums (over r) are butterfly shuffles; each wave accumulates into
// its own u array in LDS in a fixed tile order, and the kW arrays are added in
// wave order: deterministic for a given kW (tolerance-based parity, 1e-5
// relative). kPrefetch: 1 -- the next tile's two 40-byte records are loaded
// into registers before the current tile's math (20 VGPRs; the stand-alone
// kernel); 2 -- loaded once the current tile's scale terms are done (the fused
// kernel, which must stay within 80 VGPRs: the records then are not live
// across the atan evaluations); 0 -- each tile's loads are waited for.
//
// LDS: make_pair_layout(n, kW, kTiled) at `smem`. The caller has written
// Pt (formation point -> vehicle) into L.Pt, or passes the global row Ptg.
// Ends with the epilogue (saturation, the collision test, u / u_safe /
// ca_flag / gate_margin writes) over nthreads threads.
template <int kW, bool kTiled, bool GM, int kPrefetch>
__device__ __forceinline__ void pair_gain_swarm(const CtlParams& P, int b, int f,
                                                unsigned char* smem, int tid, int nthreads,
                                                const uint16_t* Ptg) {
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const PairLayout L = make_pair_layout(n, kW, kTiled);
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool inw = wave < kW;  // a pair-evaluating wave

  double* q = reinterpret_cast<double*>(smem + L.q);
  double* qf = reinterpret_cast<double*>(smem + L.qf);
  double* p = reinterpret_cast<double*>(smem + L.p);
  double* pn = reinterpret_cast<double*>(smem + L.pn);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adjF);
  int* rowpre = reinterpret_cast<int*>(smem + L.rowpre);
  uint16_t* Pt = reinterpret_cast<uint16_t*>(smem + L.Pt);
  double* acc = reinterpret_cast<double*>(smem + L.acc);
  double* uo = reinterpret_cast<double*>(smem + L.out);
  double* atab = reinterpret_cast<double*>(smem + L.atab);
#if ACL_GAIN_FASTMATH
  for (int k = tid; k < ACL_ATAB_N; k += nthreads) atab[k] = ACL_ATAB_AT(k);
#else
  for (int k = tid; k < ACL_ATAB_N; k += nthreads) atab[k] = kAtanTab[k / 6][k % 6];
#endif
  // gate margin word (in the dynamic layout: the fused kernel may use all
  // 160 KiB): set before the barriers below
  unsigned long long& gmw = *reinterpret_cast<unsigned long long*>(smem + L.gmw);
  if (GM && tid == 0) gmw = (unsigned long long)__double_as_longlong(__builtin_inf());
  unsigned* caw = reinterpret_cast<unsigned*>(smem + L.caw);
  if (tid == 0) *caw = 0u;
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  {
    const double* gq = P.q + (size_t)b * n * 3;
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += nthreads) {
      q[k] = gq[k];
      p[k] = gp[k];
    }
    for (int j = tid; j < n; j += nthreads) {
      const double x = gp[3 * j], y = gp[3 * j + 1], z = gp[3 * j + 2];
      pn[2 * j] = x * x + y * y;
      pn[2 * j + 1] = z * z;
      if (Ptg) Pt[j] = Ptg[j];
    }
    const uint64_t* ga = P.adj + (size_t)f * n * NW;
    for (int k = tid; k < n * NW; k += nthreads) {
      unsigned long long x = ga[k];
      if (k % NW == NW - 1) x &= lastmask;
      adjF[k] = x;
    }
    for (int k = tid; k < kW * n * 3; k += nthreads) acc[k] = 0.0;
  }
  __syncthreads();
  for (int k = tid; k < 3 * n; k += nthreads) {
    const int i = k / 3, c = k - 3 * i;
    qf[k] = q[3 * Pt[i] + c];
  }
  if (wave == 0) {  // edge index of the first bit of every row word (row-major edges)
    int base = 0;
    for (int w = 0; w < NW * n; w += 64) {
      const int k = w + lane;
      const int cnt = (k < n * NW) ? __popcll(adjF[k]) : 0;
      int x = cnt;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (k < n * NW) rowpre[k] = base + x - cnt;
      base += __shfl(x, 63, 64);
    }
    if (lane == 0) rowpre[n * NW] = base;
  }
  unsigned long long* tmask = reinterpret_cast<unsigned long long*>(smem + L.tmask);
  int* tstart = reinterpret_cast<int*>(smem + L.tstart);
  if (kTiled && wave == (kW > 1 ? 1 : 0)) build_tiles(adjF, NW, n, lane, tmask, tstart);
  __syncthreads();
  // record table of the 8-column blocks: etab[i][J] = (index of row i's first
  // edge at a column >= 8J) << 8 | adjmat(i, 8J .. 8J + 7) bits; a lane's
  // record is then one LDS read and a byte popcount (row-major records)
  const int nbk = (n + 7) >> 3;
  unsigned* etab = reinterpret_cast<unsigned*>(smem + L.etab);
  const bool use_etab = n <= kMaxN;
  if (!kTiled && use_etab) {
    for (int k = tid; k < n * nbk; k += nthreads) {
      const int i = k / nbk, J = k - i * nbk;
      const int w = (8 * J) >> 6, sh = (8 * J) & 63;
      const unsigned long long word = adjF[i * NW + w];
      const unsigned below = (unsigned)__popcll(sh ? (word & ((1ull << sh) - 1ull)) : 0ull);
      etab[k] = ((unsigned)(rowpre[i * NW + w] + (int)below) << 8) |
                (unsigned)((word >> sh) & 0xFFull);
    }
    __syncthreads();
  }

  double gmxy = __builtin_inf(), gmz = __builtin_inf();
  if (inw) {
    const int E = __builtin_amdgcn_readfirstlane(rowpre[n * NW]);
    const double* G = (kTiled ? P.gains_tiled : P.gains) + 5 * P.gain_off[f];
    const __amdgpu_buffer_rsrc_t grs =
        __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, 5 * E * 8, 0x00020000);
    const acl_cntrl_gains_t g = P.g;
    const int r = lane >> 3, c = lane & 7;
    const int nb = nbk;
    const int NT = nb * (nb + 1) / 2;
    double* myacc = acc + wave * n * 3;
    // this wave's tiles: a contiguous range of the row-block-major order, so
    // consecutive tiles mostly share their row block I and the row sums can
    // stay per lane in registers until the block changes
    const int t0 = (wave * NT) / kW, t1 = ((wave + 1) * NT) / kW;

    // record of (i, j) in column block J (cc = j - 8J), -1 if no edge
    auto rec_of = [&](int i, int J, int cc) -> int {
      if (!use_etab) {  // n > 128: the row's bit words and prefixes
        const int j = 8 * J + cc, jw = j >> 6, jb = j & 63;
        const unsigned long long word = adjF[i * NW + jw];
        if (!((word >> jb) & 1ull)) return -1;
        return rowpre[i * NW + jw] + __popcll(word & ((1ull << jb) - 1ull));
      }
      const unsigned x = etab[i * nb + J];
      if (!((x >> cc) & 1u)) return -1;
      // (1 << cc) - 1 made where it is used (v_bfm_b32; volatile: a hoisted
      // per-lane mask would hold a VGPR across the loop)
      unsigned below;
      asm volatile("v_bfm_b32 %0, %1, 0" : "=v"(below) : "v"(cc));
      return (int)(x >> 8) + __popc(x & below);
    };
    auto load_rec = [&](int e, double (&Lg)[5]) {
      const int voff = e >= 0 ? e * 40 : 0x40000000;  // past num_records -> 0
      const auto r0 = __builtin_amdgcn_raw_buffer_load_b128(grs, voff, 0, 0);
      const auto r1 = __builtin_amdgcn_raw_buffer_load_b128(grs, voff, 16, 0);
      const auto r2 = __builtin_amdgcn_raw_buffer_load_b64(grs, voff, 32, 0);
      __builtin_memcpy(&Lg[0], &r0, 16);
      __builtin_memcpy(&Lg[2], &r1, 16);
      __builtin_memcpy(&Lg[4], &r2, 8);
    };
    // tile t (wave-uniform: scalar code) -> (I, J), J >= I, row block by row block
    auto tile_of = [&](int t, int& I, int& J) {
      int rem = t, ii = 0;
      while (rem >= nb - ii) {
        rem -= nb - ii;
        ++ii;
      }
      I = ii;
      J = ii + rem;
    };
    auto lane_pair = [&](int t, int I, int J, int& i, int& j, int& eij, int& eji) {
      eij = eji = -1;
      i = j = 0;
      if (t >= t1) return;
      i = 8 * I + r;
      j = 8 * J + c;
      if (i >= n || j >= n || (I == J && r > c)) {
        i = j = 0;
        return;
      }
      if (kTiled) {  // record index within the tile's contiguous run
        const unsigned long long a = uni_u64(tmask[2 * t]), m2 = uni_u64(tmask[2 * t + 1]);
        const int s1 = __builtin_amdgcn_readfirstlane(tstart[2 * t]);
        const int s2 = __builtin_amdgcn_readfirstlane(tstart[2 * t + 1]);
        if ((a >> lane) & 1ull)
          eij = s1 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(a >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)a, 0u));
        if ((m2 >> lane) & 1ull)
          eji = s2 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m2 >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)m2, 0u));
        return;
      }
      eij = rec_of(i, J, c);
      if (i != j) eji = rec_of(j, I, r);
    };

    int I = 0, J = 0;
    if (t0 < t1) tile_of(t0, I, J);
    // a tile's lanes with a record in each direction, as lane masks (SGPRs:
    // the pair indices are 8I + r, 8J + c, nothing else stays in VGPRs)
    unsigned long long m_ij = 0ull, m_ji = 0ull;
    double Aij[5], Aji[5];
    if (kPrefetch != 0) {
      int i0, j0, e0, e1;
      lane_pair(t0, I, J, i0, j0, e0, e1);
      m_ij = __ballot(e0 >= 0);
      m_ji = __ballot(e1 >= 0);
      load_rec(e0, Aij);
      load_rec(e1, Aji);
    }
    // row sums of the current row block, per lane (row 8I + r, this lane's c)
    double ra0 = 0.0, ra1 = 0.0, ra2 = 0.0;
#pragma unroll 1
    for (int t = t0; t < t1; ++t) {
      int In = I, Jn = J;  // the next tile
      if (++Jn == nb) {
        ++In;
        Jn = In;
      }
      unsigned long long mn_ij = 0ull, mn_ji = 0ull;
      double Bij[5], Bji[5];
      auto prefetch_next = [&]() {
        int i1, j1, e0, e1;
        lane_pair(t + 1, In, Jn, i1, j1, e0, e1);
        mn_ij = __ballot(e0 >= 0);
        mn_ji = __ballot(e1 >= 0);
        load_rec(e0, Bij);
        load_rec(e1, Bji);
      };
      if (kPrefetch == 1) {
        prefetch_next();
      } else if (kPrefetch == 0) {
        int i0, j0, e0, e1;
        lane_pair(t, I, J, i0, j0, e0, e1);
        m_ij = __ballot(e0 >= 0);
        m_ji = __ballot(e1 >= 0);
        load_rec(e0, Aij);
        load_rec(e1, Aji);
      }
      const bool has_ij = lanebit_u64(m_ij), has_ji = lanebit_u64(m_ji);
      double rs0 = 0.0, rs1 = 0.0, rs2 = 0.0, cs0 = 0.0, cs1 = 0.0, cs2 = 0.0;
#ifdef ACL_EXP_GAIN_STREAM_ONLY
      // diagnostic builds: the record stream without the edge math
      rs0 = Aij[0] + Aji[1]; rs1 = Aij[2] + Aji[3]; rs2 = Aij[4] + Aji[4];
      const bool anyedge = false;
#else
      const bool anyedge = has_ij || has_ji;
#endif
      double q0 = 0.0, q1 = 0.0, q2 = 0.0, Fxy = 0.0, Fz = 0.0;
      if (anyedge) {
#pragma clang fp contract(fast)
        const int i = 8 * I + r, j = 8 * J + c;
        q0 = qf[3 * j] - qf[3 * i];
        q1 = qf[3 * j + 1] - qf[3 * i + 1];
        q2 = qf[3 * j + 2] - qf[3 * i + 2];
        const double pix = p[3 * i], piy = p[3 * i + 1], piz = p[3 * i + 2];
        const double pjx = p[3 * j], pjy = p[3 * j + 1], pjz = p[3 * j + 2];
        double e_xy, e_z;
        pair_e(q0, q1, q2, pn[2 * i], pn[2 * j], pn[2 * i + 1], pn[2 * j + 1], pix, piy, piz, pjx,
               pjy, pjz, pair_s2(q0, q1), e_xy, e_z);
        bool gxy, gz;
        gate_decide<GM>(g, e_xy, e_z, q0, q1, q2, pn[2 * i], pn[2 * j], pn[2 * i + 1],
                        pn[2 * j + 1], pix, piy, piz, pjx, pjy, pjz, gxy, gz, gmxy, gmz);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bool on = kk ? gz : gxy;
          if (on) {
            const double fa = kk ? g.K1_z * ACL_GAIN_ATAN(g.K2_z * e_z, atab)
                                 : g.K1_xy * ACL_GAIN_ATAN(g.K2_xy * e_xy, atab);
            if (kk) Fz = fa; else Fxy = fa;
          }
        }
      }
      if (kPrefetch == 2) {
        // the next tile's records, issued once the scale terms are done (the
        // registers they need are free from here on): their latency is
        // covered by this tile's block products, sums and LDS updates
        prefetch_next();
      }
      if (anyedge) {
#pragma clang fp contract(fast)
        // (0,0) (0,1) (1,0) (1,1) (2,2) stored; the structural zeros still
        // multiply q (solver.cpp:49-77, NaN propagation as the 3x3 product)
        if (has_ij) {
          const double up0 = ((Aij[0] * q0 + Aij[1] * q1) + 0.0 * q2) + Fxy * q0;
          const double up1 = ((Aij[2] * q0 + Aij[3] * q1) + 0.0 * q2) + Fxy * q1;
          const double up2 = ((0.0 * q0 + 0.0 * q1) + Aij[4] * q2) + Fz * q2;
          rs0 = g.kp * up0; rs1 = g.kp * up1; rs2 = g.kp * up2;
        }
        if (has_ji) {
          const double m0 = -q0, m1 = -q1, m2 = -q2;  // q_ji
          const double up0 = ((Aji[0] * m0 + Aji[1] * m1) + 0.0 * m2) + Fxy * m0;
          const double up1 = ((Aji[2] * m0 + Aji[3] * m1) + 0.0 * m2) + Fxy * m1;
          const double up2 = ((0.0 * m0 + 0.0 * m1) + Aji[4] * m2) + Fz * m2;
          cs0 = g.kp * up0; cs1 = g.kp * up1; cs2 = g.kp * up2;
        }
      }
      ra0 += rs0; ra1 += rs1; ra2 += rs2;
      // column sums over r (stride 8): DPP row_ror:8 = xor 8, then gfx950's
      // v_permlane{16,32}_swap for xor 16 and xor 32 (the same additions in
      // the same order as the xor butterfly)
      cs0 += dpp_f64_all<0x128>(cs0); cs1 += dpp_f64_all<0x128>(cs1); cs2 += dpp_f64_all<0x128>(cs2);
      cs0 = swap_sum<16>(cs0); cs1 = swap_sum<16>(cs1); cs2 = swap_sum<16>(cs2);
      cs0 = swap_sum<32>(cs0); cs1 = swap_sum<32>(cs1); cs2 = swap_sum<32>(cs2);
      {
        const int cj = 8 * J + c;
        if (r == 0 && cj < n) {
          myacc[3 * cj] += cs0; myacc[3 * cj + 1] += cs1; myacc[3 * cj + 2] += cs2;
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
      if (t + 1 == t1 || In != I) {
        // the row block ends: row sums over c (lanes 8r .. 8r + 7; DPP
        // quad_perm xor 1, xor 2, then row_half_mirror -- after the quad sums
        // lane 8r + c reads the other quad's sum)
        ra0 += dpp_f64_all<0xB1>(ra0); ra1 += dpp_f64_all<0xB1>(ra1); ra2 += dpp_f64_all<0xB1>(ra2);
        ra0 += dpp_f64_all<0x4E>(ra0); ra1 += dpp_f64_all<0x4E>(ra1); ra2 += dpp_f64_all<0x4E>(ra2);
        ra0 += dpp_f64_all<0x141>(ra0); ra1 += dpp_f64_all<0x141>(ra1); ra2 += dpp_f64_all<0x141>(ra2);
        const int ri = 8 * I + r;
        if (c == 0 && ri < n) {
          myacc[3 * ri] += ra0; myacc[3 * ri + 1] += ra1; myacc[3 * ri + 2] += ra2;
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        ra0 = ra1 = ra2 = 0.0;
      }
      I = In;
      J = Jn;
      if (kPrefetch != 0) {
        m_ij = mn_ij;
        m_ji = mn_ji;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          Aij[k] = Bij[k];
          Aji[k] = Bji[k];
        }
      }
    }
    if (GM) gate_margin_reduce(&gmw, gate_margin_of(g, gmxy, gmz));
  }
  __syncthreads();
  if (GM && tid == 0) P.gate_margin[b] = __longlong_as_double((long long)gmw);
  // u of the vehicle at row i: the kW waves' sums in wave order, plus
  // kd (-vel) once per edge of row i (distcntrl.cpp:85-95)
  {
    const acl_cntrl_gains_t g = P.g;
    for (int i = tid; i < n; i += nthreads) {
      const int v = Pt[i];
      int deg = 0;
      for (int w = 0; w < NW; ++w) deg += __popcll(adjF[i * NW + w]);
      double u0 = 0.0, u1 = 0.0, u2 = 0.0;
      for (int w = 0; w < kW; ++w) {
        const double* a = acc + w * n * 3 + 3 * i;
        u0 += a[0]; u1 += a[1]; u2 += a[2];
      }
      if (deg) {
        const double* gv = P.vel + ((size_t)b * n + v) * 3;
        const double cn = (double)deg;
        u0 += cn * (g.kd * (-gv[0]));
        u1 += cn * (g.kd * (-gv[1]));
        u2 += cn * (g.kd * (-gv[2]));
      }
      uo[3 * v] = u0; uo[3 * v + 1] = u1; uo[3 * v + 2] = u2;
    }
  }
  __syncthreads();
  gain_epilogue(P, b, n, q, uo, caw, tid, nthreads);
}

}  // namespace acl_amd
