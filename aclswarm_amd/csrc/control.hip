// control.hip -- batched DistCntrl::compute + Safety for gfx950.
//
// Runs after the auction kernel (solve.hip / solve_wide.hip) on the same
// swarms. Two kernels:
//
//   gain_kernel    DistCntrl::compute (aclswarm/src/distcntrl.cpp:46-102):
//                  the HBM stream (72 B of gain block per directed edge, 40 B
//                  in the 5-entry record layout of ADMM-structured blocks).
//                  One wave per vehicle v, lanes = formation neighbours j of
//                  v's adopted point i (chunks of 64), the 3x3 block A_ij read
//                  from the 9 coalesced planes, pdistmat's Gram-formula
//                  distances (utils.h:137-147), atan scale terms gated on
//                  |e| > thr, per-neighbour damping; a wave sum gives u (tree
//                  order: parity within 1e-5 relative). Lean on registers and
//                  LDS (~12 KB per swarm at n = 100) so several swarms are
//                  resident per CU and enough gain bytes are in flight. Its
//                  epilogue is Safety::cmdinCb saturation (safety.cpp:185-196)
//                  and the first test of Safety::collisionAvoidance
//                  (safety.cpp:412-541): a vehicle with no other vehicle
//                  inside d_avoid_thresh keeps its saturated command; the
//                  others are appended to a list.
//   ca_kernel      the rest of collisionAvoidance for the listed vehicles:
//                  lanes build the sector edges of the close vehicles, lane 0
//                  sorts them (std::sort on (angle, sign)), unions them and
//                  picks the closest safe edge exactly as the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/aclswarm_amd.h"
#include "common.h"
#include "control_params.h"

namespace acl_amd {

constexpr int kCtlBlock = 256;
#ifndef ACL_GAIN_WAVES
#define ACL_GAIN_WAVES 6  // waves per SIMD the record-layout gain kernel is built for
#endif
#ifndef ACL_GAIN_FASTMATH
#define ACL_GAIN_FASTMATH 1  // 17-point atan reduction and one-step sqrt (1e-14 relative)
#endif
#if ACL_GAIN_FASTMATH
#define ACL_GAIN_SQRT sqrt_nr1
#define ACL_GAIN_ATAN acl_atan_k32
#define ACL_ATAB_N 85
#else
#define ACL_GAIN_SQRT sqrt_nr
#define ACL_GAIN_ATAN acl_atan_tab
#define ACL_ATAB_N 30
#endif
constexpr int kCtlWaves = kCtlBlock / 64;

__host__ __device__ inline int cal16(int x) { return (x + 15) & ~15; }

// Lane segments of the gain kernel: a wave processes G vehicles at once, each
// on S consecutive lanes, in `it` passes (j = s + S t), so that n columns fill
// the 64 lanes well (n = 100: S = 20, G = 3, 5 passes, 94% of the lanes busy,
// against 78% for one vehicle per wave).
struct GainSeg {
  int S, G, it;
};

__host__ __device__ inline GainSeg gain_segments(int n) {
  GainSeg best = {64, 1, (n + 63) / 64};
  double bu = -1.0;
  for (int it = 1; it <= 16; ++it) {
    const int S = (n + it - 1) / it;
    if (S > 64) continue;
    const int G = 64 / S;
    const double u = (double)n * G / (64.0 * it);
    if (u > bu + 1e-9) {
      bu = u;
      best = {S, G, it};
    }
  }
  return best;
}

struct GainLayout {
  int q, p, pn, adjF, rowpre, Pt, myi, out, red, atab, total;
};

__host__ __device__ inline GainLayout make_gain_layout(int n) {
  const int NW = (n + 63) >> 6;
  GainLayout L;
  int o = 0;
  L.q = o;      o = cal16(o + n * 3 * 8);
  L.p = o;      o = cal16(o + n * 3 * 8);
  L.pn = o;     o = cal16(o + n * 2 * 8);       // |p_xy|^2, p_z^2 per point
  L.adjF = o;   o = cal16(o + n * NW * 8);
  L.rowpre = o; o = cal16(o + (n * NW + 1) * 4);  // edge index of each row word's first bit
  L.Pt = o;     o = cal16(o + n * 2);
  L.myi = o;    o = cal16(o + n * 2);
  L.out = o;    o = cal16(o + n * 3 * 8);       // u (DistCntrl)
  L.red = o;    o = cal16(o + kCtlWaves * 64 * 3 * 8);  // per-lane partial sums
  L.atab = o;   o = cal16(o + ACL_ATAB_N * 8);  // atan range-reduction table
  L.total = o;
  return L;
}

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
__device__ void gain_epilogue(const CtlParams& P, int b, int n, const double* q, const double* uo,
                              int tid) {
  const acl_safety_params_t sp = P.s;
  const double thr_hi = sp.d_avoid_thresh * (1.0 + 0x1p-40);
  const double thr2hi = thr_hi * thr_hi;
  for (int v = tid; v < n; v += kCtlBlock) {
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
    if (close) {  // the rest of collisionAvoidance runs in ca_kernel
      const unsigned slot = atomicAdd(P.ca_count, 1u);
      P.ca_list[slot] = (unsigned)(b * n + v);
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
// GM: the caller asked for the gate margin (acl_solve_args_t::gate_margin)
template <int NP, bool GM>
__global__ void __launch_bounds__(kCtlBlock, NP == 5 ? ACL_GAIN_WAVES : 4) gain_kernel(const CtlParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const GainLayout L = make_gain_layout(n);
  const int b = P.b0 + blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  if (P.status[b].flags & ACL_SWARM_BAD_INPUT) return;  // auction kernel zeroed outputs
  if (P.only_nonuniform && P.wsMode[b] == 0) return;    // gain_pair_kernel's swarms

  double* q = reinterpret_cast<double*>(smem + L.q);
  double* p = reinterpret_cast<double*>(smem + L.p);
  double* pn = reinterpret_cast<double*>(smem + L.pn);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adjF);
  int* rowpre = reinterpret_cast<int*>(smem + L.rowpre);
  uint16_t* Pt = reinterpret_cast<uint16_t*>(smem + L.Pt);
  uint16_t* myi = reinterpret_cast<uint16_t*>(smem + L.myi);
  double* uo = reinterpret_cast<double*>(smem + L.out);
  double* red = reinterpret_cast<double*>(smem + L.red) + wave * 64 * 3;
  double* atab = reinterpret_cast<double*>(smem + L.atab);
#if ACL_GAIN_FASTMATH
  if (tid < ACL_ATAB_N) atab[tid] = kAtan32Tab[tid / 5][tid % 5];
#else
  if (tid < ACL_ATAB_N) atab[tid] = kAtanTab[tid / 6][tid % 6];
#endif

  // the gate-margin word: set before the barriers below, so that every
  // wave's atomicMin after the edge loop follows it
  __shared__ unsigned long long gmw;
  if (GM && tid == 0) gmw = (unsigned long long)__double_as_longlong(__builtin_inf());
  const int f = P.fidx[b];
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  const bool uniform = P.wsMode[b] == 0;
  const uint16_t* rows = P.wsRows + (size_t)b * n * n;
  {
    const double* gq = P.q + (size_t)b * n * 3;
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += kCtlBlock) {
      q[k] = gq[k];
      p[k] = gp[k];
    }
    for (int j = tid; j < n; j += kCtlBlock) {
      const double x = gp[3 * j], y = gp[3 * j + 1], z = gp[3 * j + 2];
      pn[2 * j] = x * x + y * y;
      pn[2 * j + 1] = z * z;
    }
    const uint64_t* ga = P.adj + (size_t)f * n * NW;
    for (int k = tid; k < n * NW; k += kCtlBlock) {
      unsigned long long x = ga[k];
      if (k % NW == NW - 1) x &= lastmask;
      adjF[k] = x;
    }
    for (int v = tid; v < n; v += kCtlBlock) {
      myi[v] = P.P_out[(size_t)b * n + v];
      if (uniform) Pt[v] = P.wsPt[(size_t)b * n + v];
    }
  }
  __syncthreads();
  // edge index of the first bit of every row word: formation edges are
  // enumerated row-major (i, then j ascending), diagonal included
  if (wave == 0) {
    int base = 0;
    for (int w = 0; w < NW * n; w += 64) {
      const int k = w + lane;
      const int cnt = (k < n * NW) ? __popcll(adjF[k]) : 0;
      int x = cnt;  // inclusive wave scan
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (k < n * NW) rowpre[k] = base + x - cnt;
      base += __shfl(x, 63, 64);
    }
    if (lane == 0) rowpre[n * NW] = base;
  }
  __syncthreads();

  const int E = __builtin_amdgcn_readfirstlane(rowpre[n * NW]);
  double gmxy = __builtin_inf(), gmz = __builtin_inf();
  const double* G = P.gains + NP * P.gain_off[f];
  // the formation's gains through one buffer resource (9 planes: plane k at
  // SGPR offset 8kE, one VGPR offset per lane; 5: one 40-byte record per
  // edge); a lane with no edge reads past num_records, which returns 0
  const __amdgpu_buffer_rsrc_t grs =
      __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, NP * E * 8, 0x00020000);
  const acl_cntrl_gains_t g = P.g;
  const GainSeg sg = gain_segments(n);
  const int S = sg.S, GV = sg.G, IT = sg.it;
  const int seg = lane / S, s = lane - seg * S;
  const int ngroups = (n + GV - 1) / GV;
  // Groups walk formation rows in order when every vehicle holds the same
  // assignment (vehicle v = Pt[i] of row i): consecutive rows are consecutive
  // edge ranges, so the gain stream is read nearly sequentially.
  // Otherwise groups walk vehicles, each with its own adopted point.
  for (int grp = wave; grp < ngroups; grp += kCtlWaves) {
    const int r = grp * GV + seg;
    const bool act = seg < GV && r < n;
    const int rr = act ? r : 0;
    const int vv = uniform ? (int)Pt[rr] : rr;
    const int v = vv;
    const int i = uniform ? rr : (int)myi[vv];
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
    int nedge = 0;  // the damping term kd (-vel) is added once per edge, below
    // edge of pass t for this lane (-1: none); the gain loads of pass t + 1
    // are issued before pass t's math so that each wave keeps one pass of
    // the gain stream in flight while it computes
    auto edge_of = [&](int t) -> int {
      const int j = s + S * t;
      const int jw = j >> 6, jb = j & 63;
      const unsigned long long word = (act && j < n) ? adjF[i * NW + jw] : 0ull;
      if (!((word >> jb) & 1ull)) return -1;
      return rowpre[i * NW + jw] + __popcll(word & ((1ull << jb) - 1ull));
    };
    auto load_planes = [&](int e, double (&Lg)[NP]) {
      if constexpr (NP == 9) {
        const int voff = e >= 0 ? e * 8 : 0x40000000;  // past num_records -> 0
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const auto raw = __builtin_amdgcn_raw_buffer_load_b64(grs, voff, k * E * 8, 0);
          __builtin_memcpy(&Lg[k], &raw, 8);
        }
      } else {
        // one 40-byte record per edge: two 16-byte loads and one 8-byte load
        const int voff = e >= 0 ? e * 40 : 0x40000000;
        const auto r0 = __builtin_amdgcn_raw_buffer_load_b128(grs, voff, 0, 0);
        const auto r1 = __builtin_amdgcn_raw_buffer_load_b128(grs, voff, 16, 0);
        const auto r2 = __builtin_amdgcn_raw_buffer_load_b64(grs, voff, 32, 0);
        __builtin_memcpy(&Lg[0], &r0, 16);
        __builtin_memcpy(&Lg[2], &r1, 16);
        __builtin_memcpy(&Lg[4], &r2, 8);
      }
    };
    int e_cur = edge_of(0);
    double Lc[NP];
    load_planes(e_cur, Lc);
#pragma unroll 1
    for (int t = 0; t < IT; ++t) {
      // the vehicle's values are re-read from LDS every pass (short live
      // ranges: fewer VGPRs, more waves per SIMD)
      asm volatile("" ::: "memory");
      const double qv0 = q[3 * vv], qv1 = q[3 * vv + 1], qv2 = q[3 * vv + 2];
      const double pix = p[3 * i], piy = p[3 * i + 1], piz = p[3 * i + 2];
      const double Ni = pn[2 * i], Nzi = pn[2 * i + 1];
      int e_nxt = -1;
      double Ln[NP];
      if (t + 1 < IT) e_nxt = edge_of(t + 1);
      load_planes(e_nxt, Ln);
      if (e_cur >= 0) {
        // tolerance-based parity (1e-5 relative): fused multiply-adds and the
        // refined fast sqrt / quotient (common.h) are allowed here
#pragma clang fp contract(fast)
        const int j = s + S * t;
        double A[9];
        if constexpr (NP == 9) {
#pragma unroll
          for (int k = 0; k < 9; ++k) A[k] = Lc[k];
        } else {
          // (0,0) (0,1) (1,0) (1,1) (2,2) stored; +0.0 elsewhere (solver.cpp:49-77).
          // The zeros still multiply q below, as in the 9-plane layout.
          A[0] = Lc[0]; A[1] = Lc[1]; A[2] = 0.0;
          A[3] = Lc[2]; A[4] = Lc[3]; A[5] = 0.0;
          A[6] = 0.0;   A[7] = 0.0;   A[8] = Lc[4];
        }
        const int uu = uniform ? Pt[j] : rows[(size_t)v * n + j];
        const double q0 = q[3 * uu] - qv0, q1 = q[3 * uu + 1] - qv1, q2 = q[3 * uu + 2] - qv2;
        const double pjx = p[3 * j], pjy = p[3 * j + 1], pjz = p[3 * j + 2];
        const double dxy = ACL_GAIN_SQRT((Ni + pn[2 * j]) - 2.0 * (pix * pjx + piy * pjy));
        const double dz = ACL_GAIN_SQRT((Nzi + pn[2 * j + 1]) - 2.0 * (piz * pjz));
        const double e_xy = ACL_GAIN_SQRT(q0 * q0 + q1 * q1) - dxy;
        const double e_z = fabs(q2) - dz;  // |q_ij.z| = sqrt(q2^2) (no over/underflow)
        // the two gated atan terms, one after the other (register pressure)
        double Fxy = 0.0, Fz = 0.0;
        bool gxy, gz;
        gate_decide<GM>(g, e_xy, e_z, q0, q1, q2, Ni, pn[2 * j], Nzi, pn[2 * j + 1], pix, piy, piz,
                    pjx, pjy, pjz, gxy, gz, gmxy, gmz);
#pragma unroll 1
        for (int kk = 0; kk < 2; ++kk) {
          const bool on = kk ? gz : gxy;
          if (on) {
            const double fa = kk ? g.K1_z * ACL_GAIN_ATAN(g.K2_z * e_z, atab)
                                 : g.K1_xy * ACL_GAIN_ATAN(g.K2_xy * e_xy, atab);
            if (kk) Fz = fa; else Fxy = fa;
          }
        }
        const double up0 = ((A[0] * q0 + A[1] * q1) + A[2] * q2) + Fxy * q0;
        const double up1 = ((A[3] * q0 + A[4] * q1) + A[5] * q2) + Fxy * q1;
        const double up2 = ((A[6] * q0 + A[7] * q1) + A[8] * q2) + Fz * q2;
#ifdef ACL_EXP_GAIN_STREAM_ONLY
        acc0 += A[0] + A[1]; acc1 += A[3] + A[4]; acc2 += A[8];
        (void)up0; (void)up1; (void)up2;
#else
        acc0 += g.kp * up0;
        acc1 += g.kp * up1;
        acc2 += g.kp * up2;
        ++nedge;
#endif
      }
      e_cur = e_nxt;
#pragma unroll
      for (int k = 0; k < NP; ++k) Lc[k] = Ln[k];
    }
    // + kd (-vel) for each of the lane's edges (distcntrl.cpp:85-95 adds it
    // per neighbour)
    if (nedge) {
      const double* gv = P.vel + ((size_t)b * n + vv) * 3;
      const double cn = (double)nedge;
      acc0 += cn * (g.kd * (-gv[0]));
      acc1 += cn * (g.kd * (-gv[1]));
      acc2 += cn * (g.kd * (-gv[2]));
    }
    // segment sums: each vehicle's S lane partials, in lane order
    red[3 * lane] = acc0; red[3 * lane + 1] = acc1; red[3 * lane + 2] = acc2;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    if (lane < GV && grp * GV + lane < n) {
      const double* r = red + 3 * S * lane;
      double c0 = r[0], c1 = r[1], c2 = r[2];
      for (int k = 1; k < S; ++k) {
        c0 += r[3 * k]; c1 += r[3 * k + 1]; c2 += r[3 * k + 2];
      }
      const int w = uniform ? (int)Pt[grp * GV + lane] : grp * GV + lane;
      uo[3 * w] = c0; uo[3 * w + 1] = c1; uo[3 * w + 2] = c2;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  if (GM) gate_margin_reduce(&gmw, gate_margin_of(g, gmxy, gmz));
  __syncthreads();
  if (GM && tid == 0) P.gate_margin[b] = __longlong_as_double((long long)gmw);
  gain_epilogue(P, b, n, q, uo, tid);
}

// ---- gain_pair_kernel: DistCntrl::compute once per undirected edge ----------
//
// The scale terms of distcntrl.cpp:67-83 are symmetric: q_ji = q_i - q_j is
// -q_ij exactly (IEEE subtraction), so |q_ij.xy|, |q_ij.z|, pdistmat's
// Gram-formula distances (sums and products commute) and hence e_xy, e_z and
// the gated atan terms of edge (j, i) equal those of (i, j) bit for bit. This
// kernel evaluates them once per pair {i, j} and applies both blocks: A_ij
// q_ij + F q_ij to u_i and A_ji q_ji + F q_ji to u_j -- about 60% of the fp64
// work of the directed walk. For swarms whose vehicles all adopted the same
// assignment (wsMode 0: formation row i is vehicle Pt[i]); the others run in
// gain_kernel.
//
// A wave takes 8 x 8 tiles (rows I-block x columns J-block, J >= I; lane =
// 8 r + c, pair (8I + r, 8J + c); in diagonal tiles r < c, and r == c for a
// diagonal edge), loading the next tile's two 40-byte records per lane before
// the current tile's math. Row sums (over c) and column sums (over r) are
// butterfly shuffles; each wave accumulates into its own u array in LDS in a
// fixed tile order, and the four arrays are added in wave order: the result
// is deterministic (tolerance-based parity, 1e-5 relative).
#ifndef ACL_GAIN_PAIR_WAVES
#define ACL_GAIN_PAIR_WAVES 5
#endif

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
__device__ void build_tiles(const unsigned long long* adjF, int NW, int n, int lane,
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
  int q, qf, p, pn, adjF, rowpre, Pt, acc, out, atab, tmask, tstart, total;
};

__host__ __device__ inline PairLayout make_pair_layout(int n) {
  const int NW = (n + 63) >> 6;
  PairLayout L;
  int o = 0;
  L.q = o;      o = cal16(o + n * 3 * 8);            // vehicle order
  L.qf = o;     o = cal16(o + n * 3 * 8);            // formation order: qf[i] = q[Pt[i]]
  L.p = o;      o = cal16(o + n * 3 * 8);
  L.pn = o;     o = cal16(o + n * 2 * 8);
  L.adjF = o;   o = cal16(o + n * NW * 8);
  L.rowpre = o; o = cal16(o + (n * NW + 1) * 4);
  L.Pt = o;     o = cal16(o + n * 2);
  L.acc = o;    o = cal16(o + kCtlWaves * n * 3 * 8);  // per-wave u partial sums (row order)
  L.out = o;    o = cal16(o + n * 3 * 8);            // u per vehicle
  L.atab = o;   o = cal16(o + ACL_ATAB_N * 8);
  const int NT = n <= kMaxN ? pair_tiles(n) : 0;   // tiled records: n <= 128 only
  L.tmask = o;  o = cal16(o + 2 * NT * 8);
  L.tstart = o; o = cal16(o + 2 * NT * 4);
  L.total = o;
  return L;
}

template <bool kTiled, bool GM>
__global__ void __launch_bounds__(kCtlBlock, ACL_GAIN_PAIR_WAVES) gain_pair_kernel(const CtlParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const PairLayout L = make_pair_layout(n);
  const int b = P.b0 + blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  if (P.status[b].flags & ACL_SWARM_BAD_INPUT) return;
  if (P.wsMode[b] != 0) return;  // per-vehicle assignments: gain_kernel

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
  if (tid < ACL_ATAB_N) atab[tid] = kAtan32Tab[tid / 5][tid % 5];
#else
  if (tid < ACL_ATAB_N) atab[tid] = kAtanTab[tid / 6][tid % 6];
#endif
  __shared__ unsigned long long gmw;  // gate margin: set before the barriers below
  if (GM && tid == 0) gmw = (unsigned long long)__double_as_longlong(__builtin_inf());
  const int f = P.fidx[b];
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  {
    const double* gq = P.q + (size_t)b * n * 3;
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += kCtlBlock) {
      q[k] = gq[k];
      p[k] = gp[k];
    }
    for (int j = tid; j < n; j += kCtlBlock) {
      const double x = gp[3 * j], y = gp[3 * j + 1], z = gp[3 * j + 2];
      pn[2 * j] = x * x + y * y;
      pn[2 * j + 1] = z * z;
      Pt[j] = P.wsPt[(size_t)b * n + j];
    }
    const uint64_t* ga = P.adj + (size_t)f * n * NW;
    for (int k = tid; k < n * NW; k += kCtlBlock) {
      unsigned long long x = ga[k];
      if (k % NW == NW - 1) x &= lastmask;
      adjF[k] = x;
    }
    for (int k = tid; k < kCtlWaves * n * 3; k += kCtlBlock) acc[k] = 0.0;
  }
  __syncthreads();
  for (int k = tid; k < 3 * n; k += kCtlBlock) {
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
  constexpr bool tiled = kTiled;  // P.gains_tiled != NULL
  unsigned long long* tmask = reinterpret_cast<unsigned long long*>(smem + L.tmask);
  int* tstart = reinterpret_cast<int*>(smem + L.tstart);
  if (tiled && wave == 1) build_tiles(adjF, NW, n, lane, tmask, tstart);
  __syncthreads();

  const int E = __builtin_amdgcn_readfirstlane(rowpre[n * NW]);
  double gmxy = __builtin_inf(), gmz = __builtin_inf();
  const double* G = (tiled ? P.gains_tiled : P.gains) + 5 * P.gain_off[f];
  const __amdgpu_buffer_rsrc_t grs =
      __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, 5 * E * 8, 0x00020000);
  const acl_cntrl_gains_t g = P.g;
  const int r = lane >> 3, c = lane & 7;
  const int nb = (n + 7) >> 3;
  const int NT = nb * (nb + 1) / 2;
  double* myacc = acc + wave * n * 3;

  // edge index of (i, j), -1 if adjmat(i, j) == 0
  auto edge_idx = [&](int i, int j) -> int {
    const int jw = j >> 6, jb = j & 63;
    const unsigned long long word = adjF[i * NW + jw];
    if (!((word >> jb) & 1ull)) return -1;
    return rowpre[i * NW + jw] + __popcll(word & ((1ull << jb) - 1ull));
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
  // tile t -> (I, J), J >= I, enumerated row block by row block
  auto tile_of = [&](int t, int& I, int& J) {
    int rem = t, ii = 0;
    while (rem >= nb - ii) {
      rem -= nb - ii;
      ++ii;
    }
    I = ii;
    J = ii + rem;
  };
  auto lane_pair = [&](int t, int& i, int& j, int& eij, int& eji) {
    eij = eji = -1;
    i = j = 0;
    if (t >= NT) return;
    int I, J;
    tile_of(t, I, J);
    i = 8 * I + r;
    j = 8 * J + c;
    if (i >= n || j >= n || (I == J && r > c)) {
      i = j = 0;
      return;
    }
    if (tiled) {  // record index within the tile's contiguous run
      // t is wave-uniform: the masks and offsets live in SGPRs
      auto uni64 = [](unsigned long long x) -> unsigned long long {
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)x);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(x >> 32));
        return ((unsigned long long)hi << 32) | lo;
      };
      const unsigned long long a = uni64(tmask[2 * t]), m2 = uni64(tmask[2 * t + 1]);
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
    eij = edge_idx(i, j);
    if (i != j) eji = edge_idx(j, i);
  };

  int i_c, j_c, eij_c, eji_c;
  lane_pair(wave, i_c, j_c, eij_c, eji_c);
  double Aij[5], Aji[5];
  load_rec(eij_c, Aij);
  load_rec(eji_c, Aji);
#pragma unroll 1
  for (int t = wave; t < NT; t += kCtlWaves) {
    int i_n, j_n, eij_n, eji_n;
    lane_pair(t + kCtlWaves, i_n, j_n, eij_n, eji_n);
    double Bij[5], Bji[5];
    load_rec(eij_n, Bij);
    load_rec(eji_n, Bji);
    double rs0 = 0.0, rs1 = 0.0, rs2 = 0.0, cs0 = 0.0, cs1 = 0.0, cs2 = 0.0;
    if (eij_c >= 0 || eji_c >= 0) {
#pragma clang fp contract(fast)
      const int i = i_c, j = j_c;
      const double q0 = qf[3 * j] - qf[3 * i], q1 = qf[3 * j + 1] - qf[3 * i + 1],
                   q2 = qf[3 * j + 2] - qf[3 * i + 2];
      const double pix = p[3 * i], piy = p[3 * i + 1], piz = p[3 * i + 2];
      const double pjx = p[3 * j], pjy = p[3 * j + 1], pjz = p[3 * j + 2];
      const double dxy = ACL_GAIN_SQRT((pn[2 * i] + pn[2 * j]) - 2.0 * (pix * pjx + piy * pjy));
      const double dz = ACL_GAIN_SQRT((pn[2 * i + 1] + pn[2 * j + 1]) - 2.0 * (piz * pjz));
      const double e_xy = ACL_GAIN_SQRT(q0 * q0 + q1 * q1) - dxy;
      const double e_z = fabs(q2) - dz;
      double Fxy = 0.0, Fz = 0.0;
      bool gxy, gz;
      gate_decide<GM>(g, e_xy, e_z, q0, q1, q2, pn[2 * i], pn[2 * j], pn[2 * i + 1], pn[2 * j + 1],
                  pix, piy, piz, pjx, pjy, pjz, gxy, gz, gmxy, gmz);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bool on = kk ? gz : gxy;
        if (on) {
          const double fa = kk ? g.K1_z * ACL_GAIN_ATAN(g.K2_z * e_z, atab)
                               : g.K1_xy * ACL_GAIN_ATAN(g.K2_xy * e_xy, atab);
          if (kk) Fz = fa; else Fxy = fa;
        }
      }
      // (0,0) (0,1) (1,0) (1,1) (2,2) stored; the structural zeros still
      // multiply q (solver.cpp:49-77, NaN propagation as the 3x3 product)
      if (eij_c >= 0) {
        const double up0 = ((Aij[0] * q0 + Aij[1] * q1) + 0.0 * q2) + Fxy * q0;
        const double up1 = ((Aij[2] * q0 + Aij[3] * q1) + 0.0 * q2) + Fxy * q1;
        const double up2 = ((0.0 * q0 + 0.0 * q1) + Aij[4] * q2) + Fz * q2;
        rs0 = g.kp * up0; rs1 = g.kp * up1; rs2 = g.kp * up2;
      }
      if (eji_c >= 0) {
        const double m0 = -q0, m1 = -q1, m2 = -q2;  // q_ji
        const double up0 = ((Aji[0] * m0 + Aji[1] * m1) + 0.0 * m2) + Fxy * m0;
        const double up1 = ((Aji[2] * m0 + Aji[3] * m1) + 0.0 * m2) + Fxy * m1;
        const double up2 = ((0.0 * m0 + 0.0 * m1) + Aji[4] * m2) + Fz * m2;
        cs0 = g.kp * up0; cs1 = g.kp * up1; cs2 = g.kp * up2;
      }
    }
    // row sums over c (lanes 8r .. 8r + 7), column sums over r (stride 8)
    // (DPP for the steps inside a 16-lane row: quad_perm xor 1, xor 2, then
    // row_half_mirror -- after the quad sums lane 8r + c reads the other
    // quad's sum -- and row_ror:8 = xor 8; the same additions in the same
    // order as the xor butterfly)
    rs0 += dpp_f64_all<0xB1>(rs0); rs1 += dpp_f64_all<0xB1>(rs1); rs2 += dpp_f64_all<0xB1>(rs2);
    rs0 += dpp_f64_all<0x4E>(rs0); rs1 += dpp_f64_all<0x4E>(rs1); rs2 += dpp_f64_all<0x4E>(rs2);
    rs0 += dpp_f64_all<0x141>(rs0); rs1 += dpp_f64_all<0x141>(rs1); rs2 += dpp_f64_all<0x141>(rs2);
    cs0 += dpp_f64_all<0x128>(cs0); cs1 += dpp_f64_all<0x128>(cs1); cs2 += dpp_f64_all<0x128>(cs2);
    cs0 = swap_sum<16>(cs0); cs1 = swap_sum<16>(cs1); cs2 = swap_sum<16>(cs2);
    cs0 = swap_sum<32>(cs0); cs1 = swap_sum<32>(cs1); cs2 = swap_sum<32>(cs2);
    {
      int I, J;
      tile_of(t, I, J);
      const int ri = 8 * I + r, cj = 8 * J + c;
      if (c == 0 && ri < n) {
        myacc[3 * ri] += rs0; myacc[3 * ri + 1] += rs1; myacc[3 * ri + 2] += rs2;
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (r == 0 && cj < n) {
        myacc[3 * cj] += cs0; myacc[3 * cj + 1] += cs1; myacc[3 * cj + 2] += cs2;
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    i_c = i_n; j_c = j_n; eij_c = eij_n; eji_c = eji_n;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      Aij[k] = Bij[k];
      Aji[k] = Bji[k];
    }
  }
  if (GM) gate_margin_reduce(&gmw, gate_margin_of(g, gmxy, gmz));
  __syncthreads();
  if (GM && tid == 0) P.gate_margin[b] = __longlong_as_double((long long)gmw);
  // u of the vehicle at row i: the four waves' sums in wave order, plus
  // kd (-vel) once per edge of row i (distcntrl.cpp:85-95)
  for (int i = tid; i < n; i += kCtlBlock) {
    const int v = Pt[i];
    int deg = 0;
    for (int w = 0; w < NW; ++w) deg += __popcll(adjF[i * NW + w]);
    double u0 = 0.0, u1 = 0.0, u2 = 0.0;
    for (int w = 0; w < kCtlWaves; ++w) {
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
  __syncthreads();
  gain_epilogue(P, b, n, q, uo, tid);
}

// acl_tile_gains: one workgroup per formation copies every 40-byte record
// from its row-major position to its tile position (formation setup).
__global__ void __launch_bounds__(kCtlBlock) tile_gains_kernel(int n, const uint64_t* adj,
                                                               const double* gains,
                                                               const int64_t* gain_off,
                                                               double* out) {
  constexpr int kNW = (kMaxN + 63) / 64;
  constexpr int kNT = (kMaxN / 8) * (kMaxN / 8 + 1) / 2;
  __shared__ unsigned long long adjF[kMaxN * kNW];
  __shared__ int rowpre[kMaxN * kNW + 1];
  __shared__ unsigned long long tm[2 * kNT];
  __shared__ int ts[2 * kNT];
  __shared__ double stage[kCtlWaves][64 * 5];
  const int NW = (n + 63) >> 6, nb = (n + 7) >> 3;
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  for (int k = tid; k < n * NW; k += kCtlBlock) {
    unsigned long long x = adj[(size_t)f * n * NW + k];
    if (k % NW == NW - 1) x &= lastmask;
    adjF[k] = x;
  }
  __syncthreads();
  if (wave == 0) {
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
  } else if (wave == 1) {
    build_tiles(adjF, NW, n, lane, tm, ts);
  }
  __syncthreads();
  const double* src = gains + 5 * gain_off[f];
  double* dst = out + 5 * gain_off[f];
  // one wave per run (s = 2t + run), lane = 8r + c: each lane gathers its
  // record into the wave's LDS stage at its rank in the run, then the wave
  // writes the run -- one contiguous block of 40-byte records -- with
  // consecutive lanes on consecutive doubles (512 B per store instruction;
  // per-lane 40-byte-strided stores had written 3.4x the bytes)
  double* stg = stage[wave];
  const int r = lane >> 3, c = lane & 7;
  for (int s = wave; s < 2 * pair_tiles(n); s += kCtlWaves) {
    const unsigned long long m = tm[s];
    if (!m) continue;
    if ((m >> lane) & 1ull) {
      int I, J;
      tile_ij(s >> 1, nb, I, J);
      int i = 8 * I + r, j = 8 * J + c;
      if (s & 1) {  // run 2: edge (j, i)
        const int x = i;
        i = j;
        j = x;
      }
      const int jw = j >> 6, jb = j & 63;
      const unsigned long long word = adjF[i * NW + jw];
      const int e = rowpre[i * NW + jw] + __popcll(word & ((1ull << jb) - 1ull));
      const int rk = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
#pragma unroll
      for (int k = 0; k < 5; ++k) stg[5 * rk + k] = src[5 * (size_t)e + k];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    double* d = dst + 5 * (size_t)ts[s];
    const int cnt = 5 * __popcll(m);
    for (int k = lane; k < cnt; k += 64) d[k] = stg[k];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

hipError_t launch_tile_gains(int n, int F, const uint64_t* adj, const double* gains,
                             const int64_t* gain_off, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(tile_gains_kernel, dim3(F), dim3(kCtlBlock), 0, stream, n, adj, gains,
                     gain_off, out);
  return hipGetLastError();
}

// collisionAvoidance (safety.cpp:412-541) for the vehicles gain_kernel
// listed; one wave per listed vehicle, the swarm's q in the wave's LDS.
constexpr int kCaWaves = 4;

__host__ __device__ inline int ca_wave_bytes(int n) {
  return cal16(n * 3 * 8) + cal16(4 * n * 8) + cal16(4 * n);
}

// Wave-parallel tail of collisionAvoidance for one vehicle whose sector
// edges fit one wave (lane k < nslot holds slot k of caA / caS; sign 0 =
// unused). Same results as the serial lane-0 path below: the edges sorted as
// std::sort on (angle, sign) pairs (bitonic network on lanes; the order of a
// sequence of keys is unique), the parenthesis-count union as a prefix sum of
// the signs, a zone's start the edge after the previous zone's end, the
// closest zone edge by lower_bound over the sorted, flattened zone edges.
// Returns true when psi lies strictly inside a zone (cmd is then updated).
__device__ __forceinline__ bool ca_resolve_wave(int lane, int nslot, const double* caA,
                                                const signed char* caS, bool didWrap,
                                                double& cmd0, double& cmd1, double& cmd2) {
  double a = 0.0;
  int sg = 0;
  if (lane < nslot) {
    a = caA[lane];
    sg = caS[lane];
  }
  // sort key: the angle's total order (-0.0 as +0.0, so equal angles tie as
  // in the double comparison), unused slots last
  auto keyof = [](double x, int sgn) -> unsigned long long {
    if (sgn == 0) return ~0ull;
    const unsigned long long u = (unsigned long long)__double_as_longlong(x + 0.0);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
  };
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const double pa = __shfl_xor(a, j, 64);
      const int ps = __shfl_xor(sg, j, 64);
      const unsigned long long mk = keyof(a, sg), pk = keyof(pa, ps);
      const bool pless = pk < mk || (pk == mk && ps < sg);
      const bool mless = mk < pk || (mk == pk && sg < ps);
      const bool take_min = ((lane & k) == 0) == ((lane & j) == 0);
      if (take_min ? pless : mless) {
        a = pa;
        sg = ps;
      }
    }
  }
  // union: inclusive prefix count of the signs
  int incl = sg;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  const int excl = incl - sg;
  const bool isEnd = sg != 0 && incl == 0;
  const unsigned long long endMask = __ballot(isEnd);
  if (!endMask) return false;
  // zone of an end lane e: from the lane after the previous end (or lane 0)
  const unsigned long long below = endMask & ((1ull << lane) - 1ull);
  const int sLane = below ? 64 - __clzll(below) : 0;
  const double zs = __shfl(a, sLane, 64);
  const double psi = atan2(cmd1, cmd0);
  const bool inside = isEnd && psi > zs && psi < a;
  if (!__any(inside)) return false;
  // zone edges in order: every closed zone's start and end; +-pi dropped
  // when some sector wrapped
  const int lastEnd = 63 - __clzll(endMask);
  const bool isStart = sg != 0 && excl == 0 && lane < lastEnd;
  const bool keep = (isStart || isEnd) && !(didWrap && fabs(a) == kPi);
  const unsigned long long km = __ballot(keep);
  const int m = __popcll(km);
  if (m == 0) {
    cmd0 = cmd1 = 0.0;
    cmd2 = 0.0;
    return true;
  }
  const int it = __popcll(km & __ballot(keep && a < psi));  // std::lower_bound
  auto nth = [&](int r) -> int {  // lane of the r-th kept edge
    unsigned long long x = km;
    for (int t = 0; t < r; ++t) x &= x - 1ull;
    return __ffsll((long long)x) - 1;
  };
  int idx;
  if (it == 0) idx = 0;
  else if (it == m) idx = it - 1;
  else {
    const double lo = __shfl(a, nth(it - 1), 64), hi = __shfl(a, nth(it), 64);
    idx = fabs(lo - psi) < fabs(hi - psi) ? it - 1 : it;
  }
  const double edge = __shfl(a, nth(idx), 64);
  if (fabs(wrap_to_pi(edge - psi)) <= kPi / 2) {
    const double umag = sqrt(cmd0 * cmd0 + cmd1 * cmd1);
    cmd0 = umag * cos(edge);
    cmd1 = umag * sin(edge);
  } else {
    cmd0 = cmd1 = 0.0;
    cmd2 = 0.0;
  }
  return true;
}

__global__ void __launch_bounds__(64 * kCaWaves) ca_kernel(const CtlParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  unsigned char* base_ = smem + wave * ca_wave_bytes(n);
  double* q = reinterpret_cast<double*>(base_);
  double* caA = reinterpret_cast<double*>(base_ + cal16(n * 3 * 8));
  signed char* caS = reinterpret_cast<signed char*>(base_ + cal16(n * 3 * 8) + cal16(4 * n * 8));
  const acl_safety_params_t sp = P.s;
  const unsigned count = *P.ca_count;
  for (unsigned it = blockIdx.x * kCaWaves + wave; it < count; it += gridDim.x * kCaWaves) {
    const unsigned ent = P.ca_list[it];
    const int b = (int)(ent / (unsigned)n), v = (int)(ent % (unsigned)n);
    const double* gq = P.q + (size_t)b * n * 3;
    for (int k = lane; k < 3 * n; k += 64) q[k] = gq[k];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const double* gu = P.u + ((size_t)b * n + v) * 3;
    double cmd0 = gu[0], cmd1 = gu[1], cmd2 = gu[2];
    saturate(sp, cmd0, cmd1, cmd2);
    const double qv0 = q[3 * v], qv1 = q[3 * v + 1];
    // Safety::collisionAvoidance (safety.cpp:412-541)
    bool modified = false;
    {
      int base = 0;
      bool wrapped = false;
      for (int c = 0; c < NW; ++c) {
        const int j = lane + 64 * c;
        bool cand = false;
        double dx = 0.0, dy = 0.0, dd = 0.0;
        if (j < n && j != v) {
          dx = q[3 * j] - qv0;
          dy = q[3 * j + 1] - qv1;
          dd = sqrt(dx * dx + dy * dy);
          cand = !(dd > sp.d_avoid_thresh);
        }
        const unsigned long long m = __ballot(cand);
        if (cand) {
          const int slot = 4 * (base + __popcll(m & ((1ull << lane) - 1ull)));
          const double theta = atan2(dy, dx);
          const double x = sp.r_keep_out / dd;
          const double alpha = fabs(asin(x < 1.0 ? x : 1.0));
          const double beg = wrap_to_pi(theta - alpha);
          const double end = wrap_to_pi(theta + alpha);
          caA[slot] = beg;     caS[slot] = +1;
          caA[slot + 1] = end; caS[slot + 1] = -1;
          if (beg > end) {
            wrapped = true;
            caA[slot + 2] = -kPi; caS[slot + 2] = +1;
            caA[slot + 3] = kPi;  caS[slot + 3] = -1;
          } else {
            caS[slot + 2] = 0;
            caS[slot + 3] = 0;
          }
        }
        base += __popcll(m);
      }
      if (base > 0) {
        const bool didWrap = __any(wrapped);
        const int nslot = 4 * base;
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        // up to 16 close vehicles: the whole wave resolves the sectors; more
        // (or a NaN angle) take the serial path
        bool nanA = false;
        if (nslot <= 64 && lane < nslot) nanA = caS[lane] != 0 && caA[lane] != caA[lane];
        const bool par = nslot <= 64 && !__any(nanA);
        if (par) modified = ca_resolve_wave(lane, nslot, caA, caS, didWrap, cmd0, cmd1, cmd2);
        if (!par && lane == 0) {
          // compact + insertion sort by (angle, sign) = std::sort on pairs
          int ne = 0;
          for (int k = 0; k < nslot; ++k) {
            const signed char sg = caS[k];
            if (sg == 0) continue;
            const double a = caA[k];
            int pos = ne;
            while (pos > 0 && (a < caA[pos - 1] || (!(caA[pos - 1] < a) && sg < caS[pos - 1]))) {
              caA[pos] = caA[pos - 1];
              caS[pos] = caS[pos - 1];
              --pos;
            }
            caA[pos] = a;
            caS[pos] = sg;
            ++ne;
          }
          // parenthesis-count union into zones, stored in place (nz <= ne/2)
          int nz = 0, count = 0;
          double start = 0.0;
          for (int k = 0; k < ne; ++k) {
            const double a = caA[k];
            if (count == 0) start = a;
            count += caS[k];
            if (count == 0) {
              caA[2 * nz] = start;
              caA[2 * nz + 1] = a;
              ++nz;
            }
          }
          const double psi = atan2(cmd1, cmd0);
          bool safe = true;
          for (int k = 0; k < nz; ++k)
            if (psi > caA[2 * k] && psi < caA[2 * k + 1]) { safe = false; break; }
          if (!safe) {
            modified = true;
            // flatten zone edges (drop +-pi ones when wrapped), sort
            int m = 0;
            for (int k = 0; k < 2 * nz; ++k) {
              const double a = caA[k];
              if (!didWrap || fabs(a) != kPi) caA[m++] = a;
            }
            if (m == 0) {
              cmd0 = cmd1 = 0.0;
              cmd2 = 0.0;
            } else {
              for (int k = 1; k < m; ++k) {
                const double a = caA[k];
                int pos = k;
                while (pos > 0 && a < caA[pos - 1]) { caA[pos] = caA[pos - 1]; --pos; }
                caA[pos] = a;
              }
              int it = 0;  // std::lower_bound
              while (it < m && caA[it] < psi) ++it;
              int idx;
              if (it == 0) idx = 0;
              else if (it == m || fabs(caA[it - 1] - psi) < fabs(caA[it] - psi)) idx = it - 1;
              else idx = it;
              const double edge = caA[idx];
              if (fabs(wrap_to_pi(edge - psi)) <= kPi / 2) {
                const double umag = sqrt(cmd0 * cmd0 + cmd1 * cmd1);
                cmd0 = umag * cos(edge);
                cmd1 = umag * sin(edge);
              } else {
                cmd0 = cmd1 = 0.0;
                cmd2 = 0.0;
              }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
    }
    if (lane == 0) {
      if (P.u_safe) {
        double* o = P.u_safe + ((size_t)b * n + v) * 3;
        o[0] = cmd0; o[1] = cmd1; o[2] = cmd2;
      }
      if (modified) {
        if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 1;
        // n_ca is the high half of the status word at byte offset 8
        atomicAdd(reinterpret_cast<unsigned*>(&P.status[b]) + 2, 1u << 16);
        atomicOr(&P.status[b].flags, (uint32_t)ACL_SWARM_CA_ACTIVE);
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

// acl_control_batch's hand-off: P must be a permutation (else BAD_INPUT and
// zero commands, as for the auction's P_in); the inverse assignment is the
// shared row the gain kernel reads.
__global__ void __launch_bounds__(256) control_prep_kernel(const CtlParams P,
                                                           const uint16_t* Pg) {
  __shared__ unsigned long long seen[kMaxNWide / 64];
  __shared__ int bad;
  const int n = P.n, b = blockIdx.x, tid = threadIdx.x;
  if (tid < kMaxNWide / 64) seen[tid] = 0ull;
  if (tid == 0) bad = 0;
  __syncthreads();
  uint16_t* wsPt = const_cast<uint16_t*>(P.wsPt) + (size_t)b * n;
  const int f = P.fidx[b];
  if (tid == 0 && (f < 0 || f >= P.F)) bad = 1;  // formation index out of range
  for (int v = tid; v < n; v += 256) {
    const unsigned pv = Pg[(size_t)b * n + v];
    if (pv >= (unsigned)n) {
      bad = 1;
    } else {
      const unsigned long long bit = 1ull << (pv & 63);
      if (atomicOr(&seen[pv >> 6], bit) & bit) bad = 1;
      wsPt[pv] = (uint16_t)v;
    }
  }
  __syncthreads();
  if (tid == 0) {
    const_cast<uint8_t*>(P.wsMode)[b] = 0;
    acl_swarm_status_t st = {};
    st.flags = bad ? ACL_SWARM_BAD_INPUT : 0u;
    P.status[b] = st;
  }
  if (bad) {
    if (P.gate_margin && tid == 0) P.gate_margin[b] = __builtin_inf();
    for (int k = tid; k < 3 * n; k += 256) {
      P.u[(size_t)b * n * 3 + k] = 0.0;
      if (P.u_safe) P.u_safe[(size_t)b * n * 3 + k] = 0.0;
    }
    if (P.ca_flag)
      for (int v = tid; v < n; v += 256) P.ca_flag[(size_t)b * n + v] = 0;
  }
}

hipError_t launch_control_prep(const CtlParams& P, const uint16_t* Pgiven, int nb,
                               hipStream_t stream) {
  hipLaunchKernelGGL(control_prep_kernel, dim3(nb), dim3(256), 0, stream, P, Pgiven);
  return hipGetLastError();
}

// ACL_GAIN_PAIR=0 (diagnostic builds only) selects the directed walk
// (gain_kernel) for every swarm
#ifndef ACL_GAIN_PAIR
#define ACL_GAIN_PAIR 1
#endif

hipError_t launch_control(const CtlParams& P, int nb, int which, hipStream_t stream) {
  if (which == 0) {
    CtlParams Q = P;
    Q.only_nonuniform = 0;
    if (P.gain_planes == 5 && ACL_GAIN_PAIR) {
      // uniform swarms: one evaluation per undirected edge; then gain_kernel
      // for the swarms whose vehicles hold different assignments
      const PairLayout PL = make_pair_layout(P.n);
      const bool tiled = P.gains_tiled != nullptr && P.n <= kMaxN;
      const bool gm = P.gate_margin != nullptr;
#define ACL_PAIR(T_, G_)                                                                     \
  do {                                                                                       \
    if (PL.total > 64 * 1024)                                                                \
      (void)hipFuncSetAttribute((const void*)gain_pair_kernel<T_, G_>,                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, PL.total);       \
    hipLaunchKernelGGL((gain_pair_kernel<T_, G_>), dim3(nb), dim3(kCtlBlock), PL.total, stream, Q); \
  } while (0)
      if (tiled && gm) ACL_PAIR(true, true);
      else if (tiled) ACL_PAIR(true, false);
      else if (gm) ACL_PAIR(false, true);
      else ACL_PAIR(false, false);
#undef ACL_PAIR
      if (P.all_uniform) return hipGetLastError();
      Q.only_nonuniform = 1;
    }
    const GainLayout L = make_gain_layout(P.n);
    const bool gm = P.gate_margin != nullptr;
#define ACL_GAIN(NP_, G_)                                                                    \
  do {                                                                                       \
    if (L.total > 64 * 1024)                                                                 \
      (void)hipFuncSetAttribute((const void*)gain_kernel<NP_, G_>,                           \
                                hipFuncAttributeMaxDynamicSharedMemorySize, L.total);        \
    hipLaunchKernelGGL((gain_kernel<NP_, G_>), dim3(nb), dim3(kCtlBlock), L.total, stream, Q); \
  } while (0)
    if (P.gain_planes == 5 && gm) ACL_GAIN(5, true);
    else if (P.gain_planes == 5) ACL_GAIN(5, false);
    else if (gm) ACL_GAIN(9, true);
    else ACL_GAIN(9, false);
#undef ACL_GAIN
  } else {
    // a fixed grid striding over the device-side count of listed vehicles
    const int lds = kCaWaves * ca_wave_bytes(P.n);
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)ca_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(ca_kernel, dim3(nb < 1024 ? nb : 1024), dim3(64 * kCaWaves), lds, stream,
                       P);
  }
  return hipGetLastError();
}

}  // namespace acl_amd
