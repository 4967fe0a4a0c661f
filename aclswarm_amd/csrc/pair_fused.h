// pair_fused.h -- the control phase of the fused auction + control kernel
// (auction.hip, FUSE): DistCntrl::compute (distcntrl.cpp:46-102) once per
// undirected formation edge, Safety::cmdinCb saturation (safety.cpp:185-196)
// and the first collision test of collisionAvoidance (safety.cpp:412-430),
// for one swarm (n <= 128) whose vehicles all adopted one assignment, on the
// row-major 5-entry gain records (acl_formations_t, gain_planes = 5).
//
// The same pair evaluation as pair_gain_swarm (control_dev.h): the scale
// terms of edge (j, i) equal those of (i, j) bit for bit, so one lane per
// pair {i, j} applies both gain blocks (kW waves take 8 x 8 tiles, row block
// by row block, a contiguous tile range per wave). What differs is the
// instruction budget -- the fused kernel is bound by the vector ALU
// (DESIGN.md §4):
//   * per-point data packed in one LDS row {q, p, |p.xy|^2, p.z^2}, rows
//     padded to a multiple of 8 with zeros, so no lane needs a bounds test;
//   * a lane's record index from one LDS word per direction (etab) and a
//     masked popcount; the diagonal tiles' lane masks are scalar constants;
//   * the records of tile t + 1 load into the other set of a two-set
//     register ring (the tile loop is unrolled by two: no register copies);
//   * the gain products without the four structural zeros when every q of
//     the swarm is finite (0 * q is then a signed zero, which can change only
//     the sign of an exactly-zero sum; a non-finite q keeps the 3x3 product's
//     terms: 0 * inf = NaN), and kp applied once per vehicle instead of once
//     per edge (the commands' parity is 1e-5 relative);
//   * the column sums of the three components reduced together: one
//     v_permlane32_swap of two components halves both at once, one
//     v_permlane16_swap packs the third beside them, one DPP step finishes
//     (14 vector instructions per tile instead of 36), then one ds_add_f64
//     per (column, component) lane into the wave's own accumulator (one
//     writer per address and instruction, in program order: deterministic);
//   * the first collision test's candidate search from the pair loop's own q
//     differences: a conservative test (the squared xy distance, contracted,
//     against (thr (1 + 2^-40))^2) flags the formation rows that need the
//     exact test, which every thread of the workgroup then runs on a share
//     of the rows (gain_epilogue's test); a vehicle not flagged has no other
//     vehicle within the threshold, so the outcome is the same, without an
//     n^2 loop per swarm.
// Gates, gate margin and collision flags are decided by the same expressions
// as in pair_gain_swarm (bit-identical); u / u_safe are tolerance parity.
#pragma once

#include "control_dev.h"

// diagnostic bounds (wrong results, A/B builds only): the pair loop without
// its scale terms / without its record reads / without its tiles
#ifndef ACL_DIAG_NOPAIR
#define ACL_DIAG_NOPAIR 0
#endif
#ifndef ACL_DIAG_NOLOADS
#define ACL_DIAG_NOLOADS 0
#endif
#ifndef ACL_DIAG_NOLOOP
#define ACL_DIAG_NOLOOP 0
#endif

namespace acl_amd {

struct FusedLayout {
  int pt, adj, etab, rowb, Pt, Pinv, acc, atab, cst, nearb, clf, vel, flags, gmw, caw, total;
};

// the pair loop's constants (FusedLayout::cst), read from LDS where they are
// used: held in scalar registers across the loop they made the register
// allocator spill and reload them through VGPR lanes (v_readlane: vector
// instructions) several times per tile
enum { FC_K1XY, FC_K2XY, FC_K1Z, FC_K2Z, FC_TXY, FC_TZ, FC_WIN, FC_THR2, FC_N };

// rows padded to R = 8 ceil(n / 8); kW waves evaluate pairs
__host__ __device__ inline FusedLayout make_fused_layout(int n, int kW) {
  const int nb = (n + 7) >> 3, R = 8 * nb;
  FusedLayout L;
  int o = 0;
  L.pt = o;    o = cal16(o + R * 64);          // [R] {q.x, q.y, q.z, p.x, p.y, p.z, pn_xy, pn_z}
  L.adj = o;   o = cal16(o + R * 2 * 8);       // [R][2] formation rows (masked past n)
  L.etab = o;  o = cal16(o + R * nb * 4);      // [R][nb] record base << 8 | 8 column bits
  L.rowb = o;  o = cal16(o + (R + 1) * 4);     // [R + 1] record base of every row
  L.Pt = o;    o = cal16(o + n * 2);           // formation point -> vehicle (the caller's)
  L.Pinv = o;  o = cal16(o + n * 2);           // vehicle -> formation point
  L.acc = o;   o = cal16(o + kW * R * 3 * 8);  // [kW][R][3] per-wave sums (formation rows)
  L.atab = o;  o = cal16(o + ACL_ATAB_N * 8);
  L.cst = o;   o = cal16(o + FC_N * 8);        // the pair loop's constants (FC_*)
  L.nearb = o; o = cal16(o + 4 * 4);           // [4] u32: rows flagged for the exact test
  L.clf = o;   o = cal16(o + R * 4);           // [R] u32: vehicle close (the exact test's result)
  L.vel = o;   o = cal16(o + n * 24);          // [n][3] f64 vel per vehicle (loaded with q)
  L.flags = o; o = cal16(o + 4);               // bit 0: a q coordinate is not finite
  L.gmw = o;   o = o + 8;                      // gate margin word
  L.caw = o;   o = cal16(o + 4);               // the swarm is on the collision list
  L.total = o;
  return L;
}

// one direction's 5-entry record: two 16-byte and one 8-byte buffer loads
// (an offset past num_records reads zeros)
struct Rec5 {
  double a[5];
};

__device__ __forceinline__ void load_rec5(__amdgpu_buffer_rsrc_t grs, int voff, Rec5& R) {
  const auto r0 = __builtin_amdgcn_raw_buffer_load_b128(grs, voff, 0, 0);
  const auto r1 = __builtin_amdgcn_raw_buffer_load_b128(grs, voff, 16, 0);
  const auto r2 = __builtin_amdgcn_raw_buffer_load_b64(grs, voff, 32, 0);
  __builtin_memcpy(&R.a[0], &r0, 16);
  __builtin_memcpy(&R.a[2], &r1, 16);
  __builtin_memcpy(&R.a[4], &r2, 8);
}

// tile lane bits 8r + c with r <= c (inclusive) / r < c (strict)
constexpr unsigned long long kTileUpIncl = 0x80C0E0F0F8FCFEFFull;
constexpr unsigned long long kTileUpStrict = kTileUpIncl & ~0x8040201008040201ull;
// lanes holding the packed column sums: 0-7 (x), 16-23 (z), 32-39 (y)
constexpr unsigned long long kColLanes = 0x000000FF00FF00FFull;

__device__ __forceinline__ double f64_of(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Column sums over r (lane = 8r + c) of three per-lane values, negated:
// lanes 0-7 get -sum(a), 16-23 -sum(c3), 32-39 -sum(b) of column c = lane & 7.
__device__ __forceinline__ double col3_neg(double a, double b, double c3) {
  // xor 32, a and b together: lanes 0-31 a_lo + a_hi, 32-63 b_lo + b_hi
  const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
  const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
  const auto s0 = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
  const auto s1 = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32),
                                                   false, false);
  const double p = f64_of(s0[0], s1[0]) + f64_of(s0[1], s1[1]);
  const double cc = swap_sum<32>(c3);  // xor 32 of the third, both halves
  // xor 16, p beside cc: rows of 16 lanes {p0 + p1, c0 + c1, p2 + p3, c2 + c3}
  const unsigned long long up = (unsigned long long)__double_as_longlong(p);
  const unsigned long long uc = (unsigned long long)__double_as_longlong(cc);
  const auto t0 = __builtin_amdgcn_permlane16_swap((unsigned)up, (unsigned)uc, false, false);
  const auto t1 = __builtin_amdgcn_permlane16_swap((unsigned)(up >> 32), (unsigned)(uc >> 32),
                                                   false, false);
  const double qn = -(f64_of(t0[0], t1[0]) + f64_of(t0[1], t1[1]));
  // xor 8 (DPP row_ror:8) on the negated sums
  return qn + dpp_f64_all<0x128>(qn);
}

// a constant of the pair loop, read at its use (volatile: not hoisted; the
// LDS address space spelled out, or a volatile access becomes a flat load)
__device__ __forceinline__ double fcst(const double* cst, int k) {
  return *((const volatile __attribute__((address_space(3))) double*)(cst) + k);
}

// The control parameters in the kernel-argument segment (address space 4:
// scalar loads). The fused kernel passes a pointer laundered through an
// empty asm so the loads happen where the phase uses them: a by-value kernel
// argument is loaded at the kernel's entry, and its fields would then stay
// live in scalar registers through the whole auction.
typedef const __attribute__((address_space(4))) CtlParams KCtlParams;

__device__ __forceinline__ acl_cntrl_gains_t kgains(KCtlParams& P) {
  acl_cntrl_gains_t g;
  g.K1_xy = P.g.K1_xy; g.K2_xy = P.g.K2_xy; g.K1_z = P.g.K1_z; g.K2_z = P.g.K2_z;
  g.e_xy_thr = P.g.e_xy_thr; g.e_z_thr = P.g.e_z_thr; g.kp = P.g.kp; g.kd = P.g.kd;
  return g;
}

__device__ __forceinline__ acl_safety_params_t ksafety(KCtlParams& P) {
  acl_safety_params_t s;
  s.max_vel_xy = P.s.max_vel_xy; s.max_vel_z = P.s.max_vel_z;
  s.d_avoid_thresh = P.s.d_avoid_thresh; s.r_keep_out = P.s.r_keep_out;
  return s;
}

// The control phase's global reads, issued by the caller right after its
// CBAA rounds (before adoption and the hand-off, whose work then hides their
// latency): thread tid < n holds vehicle tid's q and vel and formation row
// tid's point and adjacency words. None of it depends on the assignment.
struct FusedPre {
  double q0, q1, q2, v0, v1, v2, px, py, pz;
  unsigned long long a0, a1;
};

__device__ __forceinline__ void fused_prefetch(KCtlParams& P, int b, int f, int tid,
                                               FusedPre& X) {
  const int n = P.n;
  X.q0 = X.q1 = X.q2 = X.v0 = X.v1 = X.v2 = X.px = X.py = X.pz = 0.0;
  X.a0 = X.a1 = 0ull;
  if (tid < n) {
    const int NWg = (n + 63) >> 6;
    const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
    const double* gq = P.q + ((size_t)b * n + tid) * 3;
    const double* gv = P.vel + ((size_t)b * n + tid) * 3;
    const double* gp = P.p + ((size_t)f * n + tid) * 3;
    const uint64_t* ga = P.adj + ((size_t)f * n + tid) * NWg;
    X.q0 = gq[0]; X.q1 = gq[1]; X.q2 = gq[2];
    X.v0 = gv[0]; X.v1 = gv[1]; X.v2 = gv[2];
    X.px = gp[0]; X.py = gp[1]; X.pz = gp[2];
    X.a0 = ga[0];
    if (NWg > 1) X.a1 = ga[1] & lastmask;
    else X.a0 &= lastmask;
  }
}

template <int kW, bool GM>
__device__ __forceinline__ void pair_gain_fused(KCtlParams* Pp, int b, int f,
                                                unsigned char* smem, int tid, int nthreads,
                                                const FusedPre& X) {
  KCtlParams& P = *Pp;
  const int n = P.n;  // n <= 128 <= nthreads
  const int nb = (n + 7) >> 3, R = 8 * nb;
  const FusedLayout L = make_fused_layout(n, kW);
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  double* pt = reinterpret_cast<double*>(smem + L.pt);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adj);
  unsigned* etab = reinterpret_cast<unsigned*>(smem + L.etab);
  int* rowb = reinterpret_cast<int*>(smem + L.rowb);
  const uint16_t* Pt = reinterpret_cast<const uint16_t*>(smem + L.Pt);
  uint16_t* Pinv = reinterpret_cast<uint16_t*>(smem + L.Pinv);
  double* acc = reinterpret_cast<double*>(smem + L.acc);
  double* atab = reinterpret_cast<double*>(smem + L.atab);
  double* cst = reinterpret_cast<double*>(smem + L.cst);
  unsigned* nearb = reinterpret_cast<unsigned*>(smem + L.nearb);
  unsigned* clf = reinterpret_cast<unsigned*>(smem + L.clf);
  double* velv = reinterpret_cast<double*>(smem + L.vel);
  unsigned* flags = reinterpret_cast<unsigned*>(smem + L.flags);
  unsigned long long& gmw = *reinterpret_cast<unsigned long long*>(smem + L.gmw);
  unsigned* caw = reinterpret_cast<unsigned*>(smem + L.caw);
  // [n][3] q by vehicle: the prefetched values' way to their formation rows
  // (in the per-wave sums' region, zeroed only after the rows are built)
  double* qs = acc;

  // ---- setup: the caller has written Pt[tid] (thread tid reads it back
  // here, so no barrier is needed first); every other table is built here
  for (int k = tid; k < ACL_ATAB_N; k += nthreads) atab[k] = ACL_ATAB_AT(k);
  if (GM && tid == 0) gmw = (unsigned long long)__double_as_longlong(__builtin_inf());
  if (tid == 0) {
    *caw = 0u;
    *flags = 0u;
  }
  if (tid < 4) nearb[tid] = 0u;
  for (int k = tid; k < R; k += nthreads) clf[k] = 0u;
  if (tid < FC_N) {
    const double thr_hi = P.s.d_avoid_thresh * (1.0 + 0x1p-40);
    const double v[FC_N] = {P.g.K1_xy, P.g.K2_xy, P.g.K1_z, P.g.K2_z,
                            P.g.e_xy_thr, P.g.e_z_thr, ACL_GATE_WINDOW, thr_hi * thr_hi};
    double x = v[0];
#pragma unroll
    for (int k = 1; k < FC_N; ++k) x = tid == k ? v[k] : x;
    cst[tid] = x;
  }
  {
    bool qbad = false;
    if (tid < n) {
      // vehicle tid: q into the scratch, vel (the epilogue's damping term)
      const int v = tid;
      qs[3 * v] = X.q0;
      qs[3 * v + 1] = X.q1;
      qs[3 * v + 2] = X.q2;
      velv[3 * v] = X.v0;
      velv[3 * v + 1] = X.v1;
      velv[3 * v + 2] = X.v2;
      qbad = !(__builtin_isfinite(X.q0) && __builtin_isfinite(X.q1) && __builtin_isfinite(X.q2));
    }
    if (tid < R) {
      // formation row tid: its point and adjacency (zeros past n)
      const int i = tid;
      double row[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      if (i < n) {
        Pinv[Pt[i]] = (uint16_t)i;
        const double x = X.px, y = X.py, z = X.pz;
        row[0] = x;
        row[1] = y;
        row[2] = z;
        row[3] = x * x + y * y;
        row[4] = z * z;
      }
      pt[8 * i + 3] = row[0];
      reinterpret_cast<double4*>(pt + 8 * i)[1] = make_double4(row[1], row[2], row[3], row[4]);
      adjF[2 * i] = X.a0;
      adjF[2 * i + 1] = X.a1;
    }
    if (__any(qbad) && lane == 0) atomicOr(flags, 1u);
  }
  __syncthreads();
  if (tid < R) {  // row i's q: vehicle Pt[i]'s (zeros past n)
    const int i = tid;
    double q0 = 0.0, q1 = 0.0, q2 = 0.0;
    if (i < n) {
      const int v = Pt[i];
      q0 = qs[3 * v];
      q1 = qs[3 * v + 1];
      q2 = qs[3 * v + 2];
    }
    pt[8 * i] = q0;
    pt[8 * i + 1] = q1;
    pt[8 * i + 2] = q2;
  }
  if (wave == 0) {  // record base of every row: a scan of the row popcounts
    int base = 0;
    for (int i0 = 0; i0 < R; i0 += 64) {
      const int i = i0 + lane;
      const int cnt = (i < R) ? __popcll(adjF[2 * i]) + __popcll(adjF[2 * i + 1]) : 0;
      // inclusive prefix on DPP (row_shr 1, 2, 4, 8, then row_bcast 15 / 31):
      // no ds_bpermute round trips while the other waves wait at the barrier
      int x = cnt;
      x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);
      x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);
      x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);
      x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);
      x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
      x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
      if (i < R) rowb[i] = base + x - cnt;
      base += __builtin_amdgcn_readlane(x, 63);
    }
    if (lane == 0) rowb[R] = base;
  }
  __syncthreads();
  // k / nb as a multiply-shift: exact for k < R nb <= 2048 and nb <= 16 (the
  // error k (m - 2^16 / nb) / 2^16 < 1/32 stays below the 1/nb gap to the
  // next integer); a 32-bit division is ~30 vector instructions per entry
  const unsigned nbm = (65536u + (unsigned)nb - 1u) / (unsigned)nb;
  for (int k = tid; k < R * nb; k += nthreads) {
    const int i = (int)(((unsigned)k * nbm) >> 16), J = k - i * nb;
    const int w = J >> 3, sh = (8 * J) & 63;
    const unsigned long long word = adjF[2 * i + w];
    const unsigned below = (unsigned)__popcll(sh ? (word & ((1ull << sh) - 1ull)) : 0ull) +
                           (w ? (unsigned)__popcll(adjF[2 * i]) : 0u);
    etab[k] = ((unsigned)rowb[i] + below) << 8 | (unsigned)((word >> sh) & 0xFFull);
  }
  for (int k = tid; k < kW * R * 3; k += nthreads) acc[k] = 0.0;  // (the q scratch is dead)
  const bool qfin = (*flags & 1u) == 0u;  // workgroup-uniform (set before the barriers)
  __syncthreads();

  // ---- the pair loop
  double gmxy = __builtin_inf(), gmz = __builtin_inf();
  if (wave < kW) {
    const int E = __builtin_amdgcn_readfirstlane(rowb[R]);
    const double* G = P.gains + 5 * P.gain_off[f];
    const __amdgpu_buffer_rsrc_t grs =
        __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, 5 * E * 8, 0x00020000);
    const int r = lane >> 3, c = lane & 7;
    // the lane's (column, component) slot of the packed column sums
    const int colk = 3 * c + ((lane >> 4) == 0 ? 0 : ((lane >> 4) == 1 ? 2 : 1));
    const int NT = nb * (nb + 1) / 2;
    const int t0 = (wave * NT) / kW, t1 = ACL_DIAG_NOLOOP ? t0 : ((wave + 1) * NT) / kW;
    double* myacc = acc + wave * R * 3;

    // tile t -> (I, J), J >= I, row block by row block
    int I = 0, J = 0;
    if (t0 < t1) {
      int rem = t0;
      while (rem >= nb - I) {
        rem -= nb - I;
        ++I;
      }
      J = I + rem;
    }
    // A direction's records of tile (I, J): the lane's etab word x (bit `s`
    // of it: an edge; `below` bits under it: the record rank in its block),
    // its lane mask (diagonal tiles: `up` lanes only) and the loads (an
    // offset past num_records reads zeros). The record registers of a tile
    // are dead before the next tile's loads are issued into them.
    auto rec_mask = [&](unsigned x, int s, bool diag, unsigned long long up) {
      return __ballot((x >> s) & 1u) & (diag ? up : ~0ull);
    };
    auto rec_load = [&](unsigned x, int s, unsigned long long m, Rec5& R) {
      const unsigned e = (x >> 8) + (unsigned)__popc(x & ((1u << s) - 1u));
#if ACL_DIAG_NOLOADS  // diagnostic bound (wrong results): records without HBM reads
      const double d = (double)(lanebit_u64(m) ? (e & 7u) : 0u) * 0.125;
      R.a[0] = d; R.a[1] = -d; R.a[2] = d; R.a[3] = d; R.a[4] = -d;
#else
      load_rec5(grs, lanebit_u64(m) ? (int)__umul24(e, 40u) : 0x40000000, R);
#endif
    };
    Rec5 X, Y;
    unsigned long long mx = 0ull, my = 0ull;
    if (t0 < t1) {
      const unsigned xij = etab[__umul24(8 * I + r, nb) + J], xji = etab[__umul24(8 * J + c, nb) + I];
      mx = rec_mask(xij, c, I == J, kTileUpIncl);
      my = rec_mask(xji, r, I == J, kTileUpStrict);
      rec_load(xij, c, mx, X);
      rec_load(xji, r, my, Y);
    }
    double ra0 = 0.0, ra1 = 0.0, ra2 = 0.0;  // row sums of the current row block
#pragma unroll 1
    for (int t = t0; t < t1; ++t) {
#pragma clang fp contract(fast)
      int In = I, Jn = J;  // the next tile
      if (++Jn == nb) {
        ++In;
        Jn = In;
      }
      const bool more = t + 1 < t1;  // wave-uniform
      // the next tile's etab words, read early (their latency hides here)
      unsigned xijn = 0u, xjin = 0u;
      if (more) {
        xijn = etab[__umul24(8 * In + r, nb) + Jn];
        xjin = etab[__umul24(8 * Jn + c, nb) + In];
      }
      const int i = 8 * I + r, j = 8 * J + c;
      const double4* pi = reinterpret_cast<const double4*>(pt + 8 * i);
      const double4* pj = reinterpret_cast<const double4*>(pt + 8 * j);
      const double4 ai = pi[0], aj = pj[0];  // {q.x, q.y, q.z, p.x}
      const double q0 = aj.x - ai.x, q1 = aj.y - ai.y, q2 = aj.z - ai.z;
      const double s2 = pair_s2(q0, q1);
      {
        // collision candidates: every pair i < j of the swarm (edge or not)
        const int nr = n - 8 * I, nc = n - 8 * J;
        const unsigned long long rows = nr >= 8 ? ~0ull : ((1ull << (8 * nr)) - 1ull);
        const unsigned long long cols =
            (nc >= 8 ? 0xFFull : ((1ull << nc) - 1ull)) * 0x0101010101010101ull;
        const unsigned long long vm = rows & cols & (I == J ? kTileUpStrict : ~0ull);
        const unsigned long long nm = __ballot(!(s2 > fcst(cst, FC_THR2))) & vm;
        if (nm) {  // rare: flag both rows for the epilogue's exact test
          if (lanebit_u64(nm)) {
            atomicOr(&nearb[i >> 5], 1u << (i & 31));
            atomicOr(&nearb[j >> 5], 1u << (j & 31));
          }
        }
      }
      const unsigned long long many = mx | my;
      double Fxy = 0.0, Fz = 0.0;
      if (!ACL_DIAG_NOPAIR && lanebit_u64(many)) {
        const double4 bi = pi[1], bj = pj[1];  // {p.y, p.z, pn_xy, pn_z}
        const double pix = ai.w, piy = bi.x, piz = bi.y, pjx = aj.w, pjy = bj.x, pjz = bj.y;
        double e_xy, e_z;
        pair_e(q0, q1, q2, bi.z, bj.z, bi.w, bj.w, pix, piy, piz, pjx, pjy, pjz, s2, e_xy, e_z);
        bool gxy, gz;
        gate_decide_t<GM>(fcst(cst, FC_TXY), fcst(cst, FC_TZ), fcst(cst, FC_WIN), e_xy, e_z, q0,
                          q1, q2, bi.z, bj.z, bi.w, bj.w, pix, piy, piz, pjx, pjy, pjz, gxy, gz,
                          gmxy, gmz);
#if ACL_DIAG_NOATAN  // diagnostic bound (wrong results): linear scale terms
        if (gxy) Fxy = fcst(cst, FC_K1XY) * (fcst(cst, FC_K2XY) * e_xy);
        if (gz) Fz = fcst(cst, FC_K1Z) * (fcst(cst, FC_K2Z) * e_z);
#else
        if (gxy) Fxy = fcst(cst, FC_K1XY) * ACL_GAIN_ATAN(fcst(cst, FC_K2XY) * e_xy, atab);
        if (gz) Fz = fcst(cst, FC_K1Z) * ACL_GAIN_ATAN(fcst(cst, FC_K2Z) * e_z, atab);
#endif
      }
      const double f0 = Fxy * q0, f1 = Fxy * q1, f2 = Fz * q2;
      // row i: up_ij = A_ij q + F q (kp is applied per vehicle)
      if (lanebit_u64(mx)) {
        if (qfin) {
          ra0 += X.a[1] * q1 + (X.a[0] * q0 + f0);
          ra1 += X.a[3] * q1 + (X.a[2] * q0 + f1);
          ra2 += X.a[4] * q2 + f2;
        } else {  // the 3x3 product's structural zeros kept (NaN propagation)
          ra0 += ((X.a[0] * q0 + X.a[1] * q1) + 0.0 * q2) + f0;
          ra1 += ((X.a[2] * q0 + X.a[3] * q1) + 0.0 * q2) + f1;
          ra2 += ((0.0 * q0 + 0.0 * q1) + X.a[4] * q2) + f2;
        }
      }
      unsigned long long mxn = 0ull, myn = 0ull;
      if (more) {  // the next tile's (i, j) records into X
        mxn = rec_mask(xijn, c, In == Jn, kTileUpIncl);
        rec_load(xijn, c, mxn, X);
      }
      // row j: up_ji = A_ji (-q) + F (-q), summed as -(A_ji q + F q)
      double ct0 = 0.0, ct1 = 0.0, ct2 = 0.0;
      if (lanebit_u64(my)) {
        if (qfin) {
          ct0 = Y.a[1] * q1 + (Y.a[0] * q0 + f0);
          ct1 = Y.a[3] * q1 + (Y.a[2] * q0 + f1);
          ct2 = Y.a[4] * q2 + f2;
        } else {
          ct0 = ((Y.a[0] * q0 + Y.a[1] * q1) + 0.0 * q2) + f0;
          ct1 = ((Y.a[2] * q0 + Y.a[3] * q1) + 0.0 * q2) + f1;
          ct2 = ((0.0 * q0 + 0.0 * q1) + Y.a[4] * q2) + f2;
        }
      }
      if (more) {  // the next tile's (j, i) records into Y
        myn = rec_mask(xjin, r, In == Jn, kTileUpStrict);
        rec_load(xjin, r, myn, Y);
      }
      {
        const double cs = col3_neg(ct0, ct1, ct2);
        if (lanebit_u64(kColLanes)) unsafeAtomicAdd(myacc + 24 * J + colk, cs);
      }
      if (!more || In != I) {
        // the row block ends: row sums over c (DPP quad_perm xor 1, xor 2,
        // then row_half_mirror), lanes c == 0 add them
        ra0 += dpp_f64_all<0xB1>(ra0); ra1 += dpp_f64_all<0xB1>(ra1); ra2 += dpp_f64_all<0xB1>(ra2);
        ra0 += dpp_f64_all<0x4E>(ra0); ra1 += dpp_f64_all<0x4E>(ra1); ra2 += dpp_f64_all<0x4E>(ra2);
        ra0 += dpp_f64_all<0x141>(ra0); ra1 += dpp_f64_all<0x141>(ra1); ra2 += dpp_f64_all<0x141>(ra2);
        if (c == 0) {
          double* a = myacc + 3 * i;
          unsafeAtomicAdd(a, ra0);
          unsafeAtomicAdd(a + 1, ra1);
          unsafeAtomicAdd(a + 2, ra2);
        }
        ra0 = ra1 = ra2 = 0.0;
      }
      I = In;
      J = Jn;
      mx = mxn;
      my = myn;
    }
    if (GM) {
      const acl_cntrl_gains_t g = kgains(P);
      gate_margin_reduce(&gmw, gate_margin_of(g, gmxy, gmz));
    }
  }
  __syncthreads();
  if (GM && tid == 0) P.gate_margin[b] = __longlong_as_double((long long)gmw);
  // the first collision test's exact pass over the rows the pair loop
  // flagged, on every thread: vehicle v = tid mod n against the rows
  // tid / n, + per, ... (gain_epilogue's test; OR over the rows, any order)
  // -- a crowded swarm's n x n tests on all of the workgroup's waves, not
  // on the per-vehicle loop's first ones. A swarm without a flagged row (the
  // usual case) skips the pass and its barrier (workgroup-uniform: nearb is
  // complete after the pair loop's barrier).
  if (nearb[0] | nearb[1] | nearb[2] | nearb[3]) {
    const double thr = P.s.d_avoid_thresh;
    const double thr_hi = thr * (1.0 + 0x1p-40);
    const double thr2hi = thr_hi * thr_hi;
    const int per = nthreads / n;  // >= 1: n <= nthreads
    const int v = tid % n, j0 = tid / n;
    if (j0 < per) {
      const int i = Pinv[v];
      if ((nearb[i >> 5] >> (i & 31)) & 1u) {
        const double qv0 = pt[8 * i], qv1 = pt[8 * i + 1];
        bool c = false;
        for (int k = j0; k < n; k += per) {
          const double dx = pt[8 * k] - qv0, dy = pt[8 * k + 1] - qv1;
          const double d2 = dx * dx + dy * dy;
          if (k != i && !(d2 > thr2hi)) c |= !(sqrt(d2) > thr);
        }
        if (c) clf[v] = 1u;
      }
    }
    __syncthreads();
  }

  // ---- per vehicle: u = kp (the kW waves' sums, in wave order) + kd (-vel)
  // once per edge of its row (distcntrl.cpp:85-95); saturation and the
  // first collision test (gain_epilogue's semantics)
  {
    const acl_cntrl_gains_t g = kgains(P);
    const acl_safety_params_t sp = ksafety(P);
    const int NW = (n + 63) >> 6;
    for (int v = tid; v < n; v += nthreads) {
      const int i = Pinv[v];
      const int deg = __popcll(adjF[2 * i]) + __popcll(adjF[2 * i + 1]);
      double s0 = 0.0, s1 = 0.0, s2 = 0.0;
      for (int w = 0; w < kW; ++w) {
        const double* a = acc + (w * R + i) * 3;
        s0 += a[0];
        s1 += a[1];
        s2 += a[2];
      }
      double cmd0 = g.kp * s0, cmd1 = g.kp * s1, cmd2 = g.kp * s2;
      if (deg) {
        const double* gv = velv + 3 * v;
        const double cn = (double)deg;
        cmd0 += cn * (g.kd * (-gv[0]));
        cmd1 += cn * (g.kd * (-gv[1]));
        cmd2 += cn * (g.kd * (-gv[2]));
      }
      double* gu = P.u + ((size_t)b * n + v) * 3;
      gu[0] = cmd0;
      gu[1] = cmd1;
      gu[2] = cmd2;
      saturate(sp, cmd0, cmd1, cmd2);
      const bool close = clf[v] != 0u;  // (the exact pass above)
      if (P.u_safe) {
        double* o = P.u_safe + ((size_t)b * n + v) * 3;
        o[0] = cmd0;
        o[1] = cmd1;
        o[2] = cmd2;
      }
      if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 0;
      const unsigned long long cm = __ballot(close);
      if ((tid & 63) == 0) {
        P.ca_mask[(size_t)b * NW + (v >> 6)] = cm;
        if (cm && atomicOr(caw, 1u) == 0u) P.ca_list[atomicAdd(P.ca_count, 1u)] = (unsigned)b;
      }
    }
  }
}

}  // namespace acl_amd
