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
//                  others are marked in the swarm's mask words and the swarm
//                  is appended (once) to a list.
//   ca_kernel      the rest of collisionAvoidance for the listed swarms, one
//                  workgroup per swarm: a wave per close vehicle builds the
//                  sector edges (lanes over the other vehicles), sorts them
//                  (std::sort on (angle, sign): a bitonic network over lanes,
//                  or a rank sort for more than 16 close vehicles), unions
//                  them by a prefix count and picks the closest safe edge
//                  exactly as the reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/aclswarm_amd.h"
#include "common.h"
#include "control_params.h"
#include "control_dev.h"

namespace acl_amd {

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

__host__ __device__ inline GainLayout make_gain_layout(int n, int waves = kCtlWaves) {
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
  L.red = o;    o = cal16(o + waves * 64 * 3 * 8);  // per-lane partial sums
  L.atab = o;   o = cal16(o + ACL_ATAB_N * 8);  // atan range-reduction table
  L.total = o;
  return L;
}

// GM: the caller asked for the gate margin (acl_solve_args_t::gate_margin)
template <int NP, bool GM, int kB>
__device__ void gain_swarm(const CtlParams& P, int b) {
  constexpr int kW = kB / 64;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const GainLayout L = make_gain_layout(n, kW);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  if (P.status[b].flags & ACL_SWARM_BAD_INPUT) return;  // auction kernel zeroed outputs

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
  for (int k = tid; k < ACL_ATAB_N; k += kB) atab[k] = ACL_ATAB_AT(k);
#else
  for (int k = tid; k < ACL_ATAB_N; k += kB) atab[k] = kAtanTab[k / 6][k % 6];
#endif

  // the gate-margin word: set before the barriers below, so that every
  // wave's atomicMin after the edge loop follows it
  __shared__ unsigned long long gmw;
  if (GM && tid == 0) gmw = (unsigned long long)__double_as_longlong(__builtin_inf());
  __shared__ unsigned caw;  // the swarm is on the collision list (gain_epilogue)
  if (tid == 0) caw = 0u;
  const int f = P.fidx[b];
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  const bool uniform = P.wsMode[b] == 0;
  const uint16_t* rows = P.wsRows + (size_t)b * n * n;
  {
    const double* gq = P.q + (size_t)b * n * 3;
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += kB) {
      q[k] = gq[k];
      p[k] = gp[k];
    }
    for (int j = tid; j < n; j += kB) {
      const double x = gp[3 * j], y = gp[3 * j + 1], z = gp[3 * j + 2];
      pn[2 * j] = x * x + y * y;
      pn[2 * j + 1] = z * z;
    }
    const uint64_t* ga = P.adj + (size_t)f * n * NW;
    for (int k = tid; k < n * NW; k += kB) {
      unsigned long long x = ga[k];
      if (k % NW == NW - 1) x &= lastmask;
      adjF[k] = x;
    }
    for (int v = tid; v < n; v += kB) {
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
  for (int grp = wave; grp < ngroups; grp += kW) {
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
  gain_epilogue(P, b, n, q, uo, &caw, tid, kB);
}

// One workgroup per swarm. (A small grid striding over the swarms for the
// per-vehicle pass measured no faster -- 8.4 vs 8.1 us per empty launch of
// 4 096 swarms -- and a loop around the walk made the compiler hold the
// kernel arguments in registers across it: 40-60 VGPR spills.)
template <int NP, bool GM, int kB>
__global__ void __launch_bounds__(kB, kB == 256 ? (NP == 5 ? ACL_GAIN_WAVES : 4) : 1) gain_kernel(const CtlParams P) {
  const int b = P.b0 + blockIdx.x;
  if (P.only_nonuniform && P.wsMode[b] == 0) return;  // gain_pair_kernel's swarms
  gain_swarm<NP, GM, kB>(P, b);
}


// ---- gain_pair_kernel: DistCntrl::compute once per undirected edge ----------
// (pair_gain_swarm, control_dev.h) for the uniform swarms of acl_control_batch
// and of the unfused solve paths; one 256-thread workgroup per swarm.
#ifndef ACL_GAIN_PAIR_WAVES
#define ACL_GAIN_PAIR_WAVES 5
#endif

// kPB threads per swarm: 256, or one wave for n <= 32 (launch_control). The
// occupancy bound is the same for every size (a bound of 8 waves per SIMD
// for the small block capped it at 64 VGPRs: spills, slower)
template <bool kTiled, bool GM, int kPB>
__global__ void __launch_bounds__(kPB, ACL_GAIN_PAIR_WAVES)
    gain_pair_kernel(const CtlParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = P.b0 + blockIdx.x;
  if (P.status[b].flags & ACL_SWARM_BAD_INPUT) return;
  if (P.wsMode[b] != 0) {
    // per-vehicle assignments: the directed walk on the row-major records,
    // in this launch (no second launch over every swarm for the few)
    gain_swarm<5, GM, kPB>(P, b);
    return;
  }
  pair_gain_swarm<kPB / 64, kTiled, GM, 1>(P, b, P.fidx[b], smem, threadIdx.x, kPB,
                                           P.wsPt + (size_t)b * P.n);
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

// collisionAvoidance (safety.cpp:412-541) for the swarms gain_epilogue
// listed: one workgroup per listed swarm, the swarm's q loaded once into LDS,
// its kCaWaves waves taking the swarm's close vehicles (mask bits) in turn;
// each vehicle's sector edges in wave-private LDS.
constexpr int kCaWaves = 4;

// LDS of ca_kernel: q [n][3] f64 shared, then per wave the sector edges of
// one vehicle (caA/caS: up to 4 per other vehicle, sign 0 = unused slot) and
// the sorted copy of the general path (tA/tS), then the swarm's count of
// modified commands.
struct CaLayout {
  int a, t, s, ts, wbytes, wave, nca, total;
};
__host__ __device__ inline CaLayout ca_layout(int n) {
  CaLayout L;
  L.a = 0;
  L.t = cal16(4 * n * 8);
  L.s = 2 * L.t;
  L.ts = L.s + cal16(4 * n);
  L.wbytes = L.ts + cal16(4 * n);
  L.wave = cal16(n * 3 * 8);
  L.nca = L.wave + kCaWaves * L.wbytes;
  L.total = L.nca + 16;
  return L;
}

// sort key of a sector edge: the angle's total order (-0.0 as +0.0, so equal
// angles tie as in the double comparison), unused slots last
__device__ __forceinline__ unsigned long long ca_key(double x, int sgn) {
  if (sgn == 0) return ~0ull;
  const unsigned long long u = (unsigned long long)__double_as_longlong(x + 0.0);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// Wave-parallel tail of collisionAvoidance for one vehicle whose sector
// edges fit K <= 64 lanes (lane k < nslot holds slot k of caA / caS). Same
// results as the serial restatement (ca_resolve_serial): the edges sorted as
// std::sort on (angle, sign) pairs (bitonic network over K lanes; the order
// of a sequence of keys is unique), the parenthesis-count union as a prefix
// sum of the signs, a zone's start the edge after the previous zone's end,
// the closest zone edge by lower_bound over the sorted, flattened zone edges.
// Returns true when psi lies strictly inside a zone (cmd is then updated).
template <int K>
__device__ __forceinline__ bool ca_resolve_wave(int lane, int nslot, const double* caA,
                                                const signed char* caS, bool didWrap,
                                                double& cmd0, double& cmd1, double& cmd2) {
  double a = 0.0;
  int sg = 0;
  if (lane < nslot) {
    a = caA[lane];
    sg = caS[lane];
  }
  // lanes >= K hold unused slots only; their K-blocks sort among themselves
#pragma unroll
  for (int k = 2; k <= K; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const double pa = __shfl_xor(a, j, 64);
      const int ps = __shfl_xor(sg, j, 64);
      const unsigned long long mk = ca_key(a, sg), pk = ca_key(pa, ps);
      const bool pless = pk < mk || (pk == mk && ps < sg);
      const bool mless = mk < pk || (mk == pk && sg < ps);
      const bool take_min = ((lane & k) == 0) == ((lane & j) == 0);
      if (take_min ? pless : mless) {
        a = pa;
        sg = ps;
      }
    }
  }
  // union: inclusive prefix count of the signs (exact on lanes < K)
  int incl = sg;
#pragma unroll
  for (int o = 1; o < K; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  const int excl = incl - sg;
  const bool isEnd = lane < K && sg != 0 && incl == 0;
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
  const bool isStart = lane < K && sg != 0 && excl == 0 && lane < lastEnd;
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

// The same for any number of sector edges (more than 16 close vehicles):
// a rank sort of the used slots into tA / tS (rank = the number of edges
// before it in (angle, sign, slot) order -- stable, as the insertion sort of
// the serial restatement), then one pass over the sorted edges in chunks of
// 64 lanes carrying the sign count, the previous zone end and the counts of
// the flattened zone edges; the kept-edge masks per chunk (in caA, free once
// sorted) locate the lower_bound neighbours.
__device__ __forceinline__ bool ca_resolve_general(int lane, int nslot, double* caA,
                                                const signed char* caS, double* tA,
                                                signed char* tS, bool didWrap, double& cmd0,
                                                double& cmd1, double& cmd2) {
  int m = 0;
  for (int e0 = 0; e0 < nslot; e0 += 64)
    m += __popcll(__ballot(e0 + lane < nslot && caS[e0 + lane] != 0));
  for (int e = lane; e < nslot; e += 64) {
    const int s = caS[e];
    if (s == 0) continue;
    const double a = caA[e];
    const unsigned long long k = ca_key(a, s);
    int r = 0;
    for (int e2 = 0; e2 < nslot; ++e2) {
      const int s2 = caS[e2];
      const unsigned long long k2 = ca_key(caA[e2], s2);  // unused: ~0, never before
      r += (k2 < k) || (k2 == k && s2 != 0 && (s2 < s || (s2 == s && e2 < e)));
    }
    tA[r] = a;
    tS[r] = (signed char)s;
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  const double psi = atan2(cmd1, cmd0);
  unsigned long long* keepm = reinterpret_cast<unsigned long long*>(caA);
  const unsigned long long lt = (1ull << lane) - 1ull;
  int carry = 0, prevEnd = -1, m2 = 0, it = 0;
  bool inside = false;
  const int C = (m + 63) >> 6;
  for (int c = 0; c < C; ++c) {
    const int k = 64 * c + lane;
    const bool valid = k < m;
    const double a = valid ? tA[k] : 0.0;
    const int sg = valid ? (int)tS[k] : 0;
    int incl = sg;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    incl += carry;
    // every sector adds +1 and -1, so the count ends at 0 and no start
    // follows the last end (the serial path's unclosed zone cannot occur)
    const bool isEnd = sg != 0 && incl == 0;
    const bool isStart = sg != 0 && incl - sg == 0;
    const unsigned long long em = __ballot(isEnd);
    const unsigned long long below = em & lt;
    const int pe = below ? 64 * c + 63 - __clzll(below) : prevEnd;
    if (isEnd) inside |= psi > tA[pe + 1] && psi < a;
    const bool keep = (isStart || isEnd) && !(didWrap && fabs(a) == kPi);
    const unsigned long long km = __ballot(keep);
    if (lane == 0) keepm[c] = km;
    m2 += __popcll(km);
    it += __popcll(__ballot(keep && a < psi));
    carry = __shfl(incl, 63, 64);
    if (em) prevEnd = 64 * c + 63 - __clzll(em);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (!__any(inside)) return false;
  if (m2 == 0) {
    cmd0 = cmd1 = 0.0;
    cmd2 = 0.0;
    return true;
  }
  auto nth = [&](int r) -> int {  // sorted index of the r-th kept edge
    int c = 0;
    unsigned long long x = keepm[0];
    while (r >= __popcll(x)) {
      r -= __popcll(x);
      x = keepm[++c];
    }
    for (int t = 0; t < r; ++t) x &= x - 1ull;
    return 64 * c + __ffsll((long long)x) - 1;
  };
  int idx;
  if (it == 0) idx = 0;
  else if (it == m2) idx = it - 1;
  else idx = fabs(tA[nth(it - 1)] - psi) < fabs(tA[nth(it)] - psi) ? it - 1 : it;
  const double edge = tA[nth(idx)];
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

// Serial restatement (lane 0) for sector edges with a NaN angle, whose
// std::sort order the comparison networks above do not reproduce: insertion
// sort on (angle, sign), parenthesis-count union, closest zone edge.
__device__ __forceinline__ bool ca_resolve_serial(int nslot, double* caA, signed char* caS,
                                               bool didWrap, double& cmd0, double& cmd1,
                                               double& cmd2) {
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
  if (safe) return false;
  // flatten zone edges (drop +-pi ones when wrapped), sort
  int m = 0;
  for (int k = 0; k < 2 * nz; ++k) {
    const double a = caA[k];
    if (!didWrap || fabs(a) != kPi) caA[m++] = a;
  }
  if (m == 0) {
    cmd0 = cmd1 = 0.0;
    cmd2 = 0.0;
    return true;
  }
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
  return true;
}

#ifndef ACL_CA_GRID
#define ACL_CA_GRID 2048  // ca_kernel's workgroups at most (a grid-stride loop over the list)
#endif
// ca_pair_kernel's: more workgroups than the CU can hold, so the dispatcher
// evens out swarms of unequal work (crowded C3 15.60 -> 15.43 ms, the
// uncrowded launch unchanged; profiles/r5_ab_cagrid/)
#ifndef ACL_CA_PAIR_GRID
#define ACL_CA_PAIR_GRID 8192
#endif
// diagnostic build (-DACL_CA_PROF=1, scripts/phase_profile.py --crowd): wave
// cycles of the sector build, the resolution and the rest into
// P.stamps[b][kStampSec + 8..10], close vehicles into [kStampSec + 11]
#ifndef ACL_CA_PROF
#define ACL_CA_PROF 0
#endif
#if ACL_CA_PROF
#define CPROF_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define CPROF_ADD(acc, x) acc += (x)
#else
#define CPROF_T(v)
#define CPROF_ADD(acc, x)
#endif
// The collision list's counters (WsLayout::cacount, kCaCounterBytes) are zero
// between calls, so a persistent workspace needs no memset per solve
// (acl_solve_args_t::ws_persistent). The launch's first max(entries, 1)
// workgroups take part (each read the entry count at its start, before its
// increment below, so all read the same count; a workgroup past them reads
// either that count or 0 and takes no part either way -- an uncrowded launch
// costs one atomic): each adds one to its group's counter (workgroup b in
// group b mod kCaGroups), the group's last zeroes that counter and adds one to
// [1], and the last group zeroes [1] and the entry count. (One counter for
// every workgroup had made the C3 launch 6 -> 97 us: 8 192 returning atomics
// on one address.) The count is clamped to the batch: a list is never longer
// than B.
__device__ __forceinline__ unsigned ca_list_count(const CtlParams& P) {
  const unsigned c = *P.ca_count;
  return c < (unsigned)P.B ? c : (unsigned)P.B;
}

__device__ __forceinline__ void ca_list_release(const CtlParams& P, unsigned count) {
  const unsigned g = gridDim.x, parts = count == 0u ? 1u : (count < g ? count : g);
  if (blockIdx.x >= parts) return;  // workgroup-uniform
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned grp = blockIdx.x % kCaGroups;
    const unsigned gsize = (parts - 1u - grp) / kCaGroups + 1u;  // members grp, grp + 64, ... < parts
    unsigned* gc = P.ca_count + kCaGroupStride * (1 + grp);
    if (atomicAdd(gc, 1u) == gsize - 1u) {
      atomicExch(gc, 0u);
      const unsigned ng = parts < (unsigned)kCaGroups ? parts : (unsigned)kCaGroups;
      if (atomicAdd(P.ca_count + 1, 1u) == ng - 1u) {
        atomicExch(P.ca_count, 0u);
        atomicExch(P.ca_count + 1, 0u);
      }
    }
  }
}

__global__ void __launch_bounds__(64 * kCaWaves) ca_kernel(const CtlParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const CaLayout L = ca_layout(n);
  double* q = reinterpret_cast<double*>(smem);
  unsigned char* wb = smem + L.wave + wave * L.wbytes;
  double* caA = reinterpret_cast<double*>(wb + L.a);
  double* tA = reinterpret_cast<double*>(wb + L.t);
  signed char* caS = reinterpret_cast<signed char*>(wb + L.s);
  signed char* tS = reinterpret_cast<signed char*>(wb + L.ts);
  unsigned* nca = reinterpret_cast<unsigned*>(smem + L.nca);
  const acl_safety_params_t sp = P.s;
  const unsigned count = ca_list_count(P);
  for (unsigned it = blockIdx.x; it < count; it += gridDim.x) {
    const int b = (int)P.ca_list[it];
    const double* gq = P.q + (size_t)b * n * 3;
    for (int k = tid; k < 3 * n; k += 64 * kCaWaves) q[k] = gq[k];
    if (tid == 0) *nca = 0u;
    __syncthreads();
#if ACL_CA_PROF
    unsigned long long cp_build = 0, cp_res = 0, cp_all = 0, cp_cnt = 0;
    CPROF_T(cw0);
#endif
    unsigned mine = 0;  // commands this wave modified (lane 0)
    int r = 0;          // rank of the close vehicle in the swarm: wave r % kCaWaves
    const uint64_t* cmask = P.ca_mask + (size_t)b * NW;
    for (int w = 0; w < NW; ++w) {
      unsigned long long mw = cmask[w];
      while (mw) {
        const int v = 64 * w + __ffsll((long long)mw) - 1;
        mw &= mw - 1ull;
        if ((r++ % kCaWaves) != wave) continue;
        CPROF_T(cb0);
        CPROF_ADD(cp_cnt, 1ull);
        const double* gu = P.u + ((size_t)b * n + v) * 3;
        double cmd0 = gu[0], cmd1 = gu[1], cmd2 = gu[2];
        saturate(sp, cmd0, cmd1, cmd2);
        const double qv0 = q[3 * v], qv1 = q[3 * v + 1];
        // Safety::collisionAvoidance (safety.cpp:412-541): the sector of
        // every vehicle within d_avoid_thresh, 4 slots per vehicle (the
        // wrapped part [-pi, pi] when the sector crosses +-pi)
        bool modified = false;
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
        CPROF_T(cb1);
        CPROF_ADD(cp_build, cb1 - cb0);
        if (base > 0) {
          const bool didWrap = __any(wrapped);
          const int nslot = 4 * base;
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
          bool nanA = false;
          for (int e = lane; e < nslot; e += 64) nanA |= caS[e] != 0 && caA[e] != caA[e];
          if (__any(nanA)) {
            if (lane == 0) modified = ca_resolve_serial(nslot, caA, caS, didWrap, cmd0, cmd1, cmd2);
          } else if (nslot <= 8) {
            modified = ca_resolve_wave<8>(lane, nslot, caA, caS, didWrap, cmd0, cmd1, cmd2);
          } else if (nslot <= 16) {
            modified = ca_resolve_wave<16>(lane, nslot, caA, caS, didWrap, cmd0, cmd1, cmd2);
          } else if (nslot <= 32) {
            modified = ca_resolve_wave<32>(lane, nslot, caA, caS, didWrap, cmd0, cmd1, cmd2);
          } else if (nslot <= 64) {
            modified = ca_resolve_wave<64>(lane, nslot, caA, caS, didWrap, cmd0, cmd1, cmd2);
          } else {
            modified = ca_resolve_general(lane, nslot, caA, caS, tA, tS, didWrap, cmd0, cmd1,
                                          cmd2);
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
        }
        CPROF_T(cb2);
        CPROF_ADD(cp_res, cb2 - cb1);
        if (lane == 0) {
          if (P.u_safe) {
            double* o = P.u_safe + ((size_t)b * n + v) * 3;
            o[0] = cmd0; o[1] = cmd1; o[2] = cmd2;
          }
          if (modified) {
            if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 1;
            ++mine;
          }
        }
      }
    }
    if (lane == 0 && mine) atomicAdd(nca, mine);
#if ACL_CA_PROF
    CPROF_T(cw1);
    if (P.stamps && lane == 0) {
      unsigned long long* ps = P.stamps + (size_t)b * kStampStride + kStampSec;
      atomicAdd(ps + 8, cp_build);
      atomicAdd(ps + 9, cp_res);
      atomicAdd(ps + 10, (cw1 - cw0) - cp_build - cp_res);
      atomicAdd(ps + 11, cp_cnt);
    }
#endif
    __syncthreads();
    // the workgroup owns the swarm's status word here (the control kernels
    // before it are stream-ordered): n_ca is the high half of the word at
    // byte offset 8
    if (tid == 0 && *nca) {
      reinterpret_cast<unsigned*>(&P.status[b])[2] += *nca << 16;
      P.status[b].flags |= (uint32_t)ACL_SWARM_CA_ACTIVE;
    }
  }
  ca_list_release(P, count);
}

// ---- collisionAvoidance by pairs (n <= 128) ----------------------------------
//
// ca_kernel gives every close vehicle a wave whose lanes run over the other
// vehicles: in a crowded swarm a vehicle has a handful of neighbours inside
// d_avoid_thresh, so the atan2 / asin of the sector edges (the kernel's fp64
// bulk) ran on a few lanes of two 64-lane chunks. ca_pair_kernel works by
// (vehicle, neighbour) pairs instead: one workgroup per listed swarm
//   A  lanes over the swarm's close vehicles: the saturated command and psi
//   B  a wave per close vehicle: its candidates (distance test, lanes over
//      the others) as mask words and counts; a prefix gives each vehicle a
//      contiguous run of pairs
//   C  lanes over the pairs (64 per instruction): theta, alpha and the
//      sector's two edges (beg, +1), (end, -1) at slots 2p, 2p + 1; a wrapped
//      sector adds (-pi, +1), (pi, -1) -- identical for every wrap, so only
//      counted per vehicle and synthesized where a vehicle's edges are read
//   D  the union and closest safe edge of up to 4 vehicles per wave: 16-,
//      32- or 64-lane segments by edge count (bitonic sort of (angle, sign)
//      keys, prefix count, ballots per segment); more than 64 edges or a NaN
//      angle: one vehicle at a time on the general / serial paths
//   E  lanes over the close vehicles: cos / sin of the chosen edge, u_safe,
//      ca_flag
// The same math as ca_kernel in the same operation order (identical results).
// Pairs are processed in batches of at most kCaPairCap (a vehicle has at most
// n - 1 <= 127), so the LDS image stays bounded.
constexpr int kCaPairCap = 1024;
constexpr int kCaPT = 256;
// diagnostic builds only (-DACL_CA_DIAG_FASTTRIG: wrong results): the pair
// kernel's atan2 / asin / cos / sin in f32, to bound what the f64 library
// calls cost
#ifdef ACL_CA_DIAG_FASTTRIG
#define CA_ATAN2(y, x) ((double)atan2f((float)(y), (float)(x)))
#define CA_ASIN(x) ((double)asinf((float)(x)))
#define CA_COS(x) ((double)cosf((float)(x)))
#define CA_SIN(x) ((double)sinf((float)(x)))
#else
#define CA_ATAN2(y, x) atan2(y, x)
#define CA_ASIN(x) asin(x)
#define CA_COS(x) cos(x)
#define CA_SIN(x) sin(x)
#endif

struct CaPairLayout {
  int q, cl, cmd, psi, cnt, off, wr, flg, edge, cmk, lists, pairs, ang, sA, sS, tA, tS, misc,
      total;
};
__host__ __device__ inline CaPairLayout ca_pair_layout(int n) {
  CaPairLayout L;
  int o = 0;
  L.q = o;     o = cal16(o + n * 24);
  L.cl = o;    o = cal16(o + n * 2);        // close vehicles (ascending)
  L.cmd = o;   o = cal16(o + n * 24);       // saturated commands
  L.psi = o;   o = cal16(o + n * 8);
  L.cnt = o;   o = cal16(o + n * 4);        // candidates per close vehicle
  L.off = o;   o = cal16(o + (n + 1) * 4);  // exclusive prefix of cnt
  L.wr = o;    o = cal16(o + n * 4);        // wrapped sectors
  L.flg = o;   o = cal16(o + n * 4);        // NaN edge (bit 0); result: 1 edge, 2 stop (bits 8..)
  L.edge = o;  o = cal16(o + n * 8);        // the chosen edge
  L.cmk = o;   o = cal16(o + n * 2 * 8);    // candidate masks [k][2]
  L.lists = o; o = cal16(o + 5 * n * 2);    // vehicles per resolve class (8/16/32/64/general)
  L.pairs = o; o = cal16(o + kCaPairCap * 2);   // neighbour of each pair (u8 k | u8 j)
  L.ang = o;   o = cal16(o + kCaPairCap * 2 * 8);
  L.sA = o;    o = cal16(o + 4 * n * 8);    // general / serial paths: one vehicle's slots
  L.sS = o;    o = cal16(o + 4 * n);
  L.tA = o;    o = cal16(o + 4 * n * 8);
  L.tS = o;    o = cal16(o + 4 * n);
  L.misc = o;  o = cal16(o + 16 * 4);
  L.total = o;
  return L;
}

// The value of lane ^ J (J = 1 ... 32) without the LDS unit (ds_bpermute:
// a dependent chain of LDS round trips per sorting stage): quad_perm for 1
// and 2, row_half_mirror after a quad reversal for 4 (l ^ 3 ^ 7), row_ror:8
// for 8, and for 16 / 32 gfx950's permlane swaps of a copy with itself,
// which leave {x[l], x[l ^ J]} in the lane's two registers in some order:
// the one that is not x[l] is the partner's (equal values: either is).
template <int J>
__device__ __forceinline__ unsigned xlane_u32(unsigned x) {
  if constexpr (J == 1) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
  else if constexpr (J == 2) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);
  else if constexpr (J == 4)
    return (unsigned)__builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp((int)x, 0x1B, 0xF, 0xF, true),
                                              0x141, 0xF, 0xF, true);
  else if constexpr (J == 8) return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, true);
  else {
    static_assert(J == 16 || J == 32, "lane xor 1 ... 32");
    const auto v = J == 16 ? __builtin_amdgcn_permlane16_swap(x, x, false, false)
                           : __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return v[0] == x ? v[1] : v[0];
  }
}
template <int J>
__device__ __forceinline__ unsigned long long xlane_u64(unsigned long long x) {
  return ((unsigned long long)xlane_u32<J>((unsigned)(x >> 32)) << 32) | xlane_u32<J>((unsigned)x);
}
// runtime j (a power of two <= 32; unrolled loops fold it to a constant)
__device__ __forceinline__ unsigned long long xlane64(unsigned long long x, int j) {
  switch (j) {
    case 1: return xlane_u64<1>(x);
    case 2: return xlane_u64<2>(x);
    case 4: return xlane_u64<4>(x);
    case 8: return xlane_u64<8>(x);
    case 16: return xlane_u64<16>(x);
    default: return xlane_u64<32>(x);
  }
}
__device__ __forceinline__ unsigned xlane32(unsigned x, int j) {
  switch (j) {
    case 1: return xlane_u32<1>(x);
    case 2: return xlane_u32<2>(x);
    case 4: return xlane_u32<4>(x);
    case 8: return xlane_u32<8>(x);
    case 16: return xlane_u32<16>(x);
    default: return xlane_u32<32>(x);
  }
}

// Segmented resolution: S-lane segments (S = 16, 32, 64), one vehicle each;
// lane e of a segment holds element e of its vehicle (m elements, e >= m an
// unused slot sorting last). As ca_resolve_wave, per segment. Returns the
// outcome for the lane's vehicle: 0 safe, 1 new direction `edge`, 2 stop.
// A vehicle's edge x (m = c2 + 2 wraps of them): its pairs' edges from av
// (beg, end alternating), then the wraps' (-pi, +1), (pi, -1).
__device__ __forceinline__ double ca_edge_of(const double* av, int c2, int x) {
  return x < c2 ? av[x] : (((x - c2) & 1) ? kPi : -kPi);
}
template <int S>
__device__ __forceinline__ int ca_resolve_seg(int lane, int m, int c2, const double* av,
                                              bool didWrap, double psi, double& edge) {
  const int e = lane & (S - 1), base = lane & ~(S - 1);
  const unsigned long long segm = S == 64 ? ~0ull : (((1ull << S) - 1ull) << base);
  // bitonic network on (key, sign): the key travels with the slot and its
  // sign packed as slot << 2 | sign + 1 (an edge's sign is its slot's parity:
  // c2 is even), and the angle itself -- -0.0 included, which the later
  // steps read -- is fetched by slot once sorted
  unsigned long long mk = ~0ull;
  unsigned sv = (unsigned)e << 2 | 1u;  // unused slot: sign 0, sorting last
  if (e < m) {
    mk = ca_key(ca_edge_of(av, c2, e), 1);
    sv = (unsigned)e << 2 | ((e & 1) ? 0u : 2u);
  }
#pragma unroll
  for (int k = 2; k <= S; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const unsigned long long pk = xlane64(mk, j);
      const unsigned ps = xlane32(sv, j);
      const bool pless = pk < mk || (pk == mk && (ps & 3u) < (sv & 3u));
      const bool mless = mk < pk || (mk == pk && (sv & 3u) < (ps & 3u));
      const bool take_min = ((e & k) == 0) == ((e & j) == 0);
      if (take_min ? pless : mless) {
        sv = ps;
        mk = pk;
      }
    }
  }
  const int sg = (int)(sv & 3u) - 1;
  const double a = sg != 0 ? ca_edge_of(av, c2, (int)(sv >> 2)) : 0.0;
  // inclusive prefix of the signs within the segment: row_shr 1, 2, 4, 8
  // (zero past the row's start; S = 8 masks the other half row), then
  // row_bcast 15 / 31 into the next row(s)
  int incl = sg;
  if constexpr (S == 8) {
    int y = __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xF, 0xF, true);
    incl += e >= 1 ? y : 0;
    y = __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xF, 0xF, true);
    incl += e >= 2 ? y : 0;
    y = __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xF, 0xF, true);
    incl += e >= 4 ? y : 0;
  } else {
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xF, 0xF, true);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xF, 0xF, true);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xF, 0xF, true);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xF, 0xF, true);
  }
  if constexpr (S >= 32) incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xA, 0xF, false);
  if constexpr (S == 64) incl += __builtin_amdgcn_update_dpp(0, incl, 0x143, 0xC, 0xF, false);
  const int excl = incl - sg;
  const bool isEnd = sg != 0 && incl == 0;
  const unsigned long long endMask = __ballot(isEnd) & segm;
  const unsigned long long below = endMask & ((1ull << lane) - 1ull) & segm;
  const int sLane = below ? 64 - __clzll(below) : base;
  const double zs = __shfl(a, sLane, 64);
  const bool inside = isEnd && psi > zs && psi < a;
  if (!endMask || !(__ballot(inside) & segm)) return 0;
  const int lastEnd = 63 - __clzll(endMask);
  const bool isStart = sg != 0 && excl == 0 && lane < lastEnd;
  const bool keep = (isStart || isEnd) && !(didWrap && fabs(a) == kPi);
  const unsigned long long km = __ballot(keep) & segm;
  const int m2 = __popcll(km);
  if (m2 == 0) return 2;
  // std::lower_bound: the segment is sorted, so the kept edges below psi are
  // the first `it` kept lanes -- the (it - 1)-th kept edge is the highest of
  // them, the it-th the lowest kept lane above
  const unsigned long long kb = __ballot(keep && a < psi) & segm;
  const int it = __popcll(kb);
  const unsigned long long ka = km & ~kb;
  // (the shuffles are wave-wide: every lane computes its own segment's indices)
  int idx;
  const int lo_l = it > 0 ? 63 - __clzll(kb) : __ffsll((long long)km) - 1;
  const int hi_l = it < m2 ? __ffsll((long long)ka) - 1 : 63 - __clzll(km);
  const double lo = __shfl(a, lo_l, 64), hi = __shfl(a, hi_l, 64);
  if (it == 0) idx = 0;
  else if (it == m2) idx = it - 1;
  else idx = fabs(lo - psi) < fabs(hi - psi) ? it - 1 : it;
  edge = idx == it ? hi : lo;
  if (it == 0) edge = hi;  // nth(0): the first kept edge
  return fabs(wrap_to_pi(edge - psi)) <= kPi / 2 ? 1 : 2;
}

#ifndef ACL_CA_OCC
#define ACL_CA_OCC 4  // ca_pair_kernel's occupancy bound (waves per SIMD)
#endif
// diagnostic builds only (-DACL_CA_STOP=k, wrong results): ca_pair_kernel
// without its phases after k (0: nothing, 1: A + B and the prefix, 2: the pair lists,
// 3: C, 4: D and the general paths), to split the launch's time by phase
#ifndef ACL_CA_STOP
#define ACL_CA_STOP 9
#endif
__global__ void __launch_bounds__(kCaPT, ACL_CA_OCC) ca_pair_kernel(const CtlParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int kW = kCaPT / 64;
  const CaPairLayout L = ca_pair_layout(n);
  double* q = reinterpret_cast<double*>(smem + L.q);
  uint16_t* cl = reinterpret_cast<uint16_t*>(smem + L.cl);
  double* cmd = reinterpret_cast<double*>(smem + L.cmd);
  double* psiv = reinterpret_cast<double*>(smem + L.psi);
  int* cnt = reinterpret_cast<int*>(smem + L.cnt);
  int* off = reinterpret_cast<int*>(smem + L.off);
  int* wr = reinterpret_cast<int*>(smem + L.wr);
  int* flg = reinterpret_cast<int*>(smem + L.flg);
  double* edg = reinterpret_cast<double*>(smem + L.edge);
  unsigned long long* cmk = reinterpret_cast<unsigned long long*>(smem + L.cmk);
  uint16_t* lists = reinterpret_cast<uint16_t*>(smem + L.lists);
  uint16_t* pairs = reinterpret_cast<uint16_t*>(smem + L.pairs);
  double* ang = reinterpret_cast<double*>(smem + L.ang);
  double* sA = reinterpret_cast<double*>(smem + L.sA);
  signed char* sS = reinterpret_cast<signed char*>(smem + L.sS);
  double* tA = reinterpret_cast<double*>(smem + L.tA);
  signed char* tS = reinterpret_cast<signed char*>(smem + L.tS);
  // [0] nc, [5] modified, [6] pairs handed out, [8..12] class counts
  int* misc = reinterpret_cast<int*>(smem + L.misc);
  const acl_safety_params_t sp = P.s;
  const unsigned count = ca_list_count(P);
  for (unsigned itb = blockIdx.x; itb < (ACL_CA_STOP < 1 ? 0u : count); itb += gridDim.x) {
    const int b = (int)P.ca_list[itb];
    const double* gq = P.q + (size_t)b * n * 3;
    for (int k = tid; k < 3 * n; k += kCaPT) q[k] = gq[k];
    if (wave == 0) {  // the close vehicles in ascending order
      const uint64_t* cmask = P.ca_mask + (size_t)b * NW;
      int base = 0;
      for (int w = 0; w < NW; ++w) {
        const unsigned long long mw = cmask[w];
        if ((mw >> lane) & 1ull)
          cl[base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mw >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((unsigned)mw, 0u))] =
              (uint16_t)(64 * w + lane);
        base += __popcll(mw);
      }
      if (lane == 0) {
        misc[0] = base;
        misc[5] = 0;
        misc[6] = 0;
      }
    }
    __syncthreads();
    const int nc = misc[0];
    // A: saturated commands and psi (lanes over the close vehicles)
    #pragma unroll 1
    for (int k = tid; k < nc; k += kCaPT) {
      const int v = cl[k];
      const double* gu = P.u + ((size_t)b * n + v) * 3;
      double c0 = gu[0], c1 = gu[1], c2 = gu[2];
      saturate(sp, c0, c1, c2);
      cmd[3 * k] = c0; cmd[3 * k + 1] = c1; cmd[3 * k + 2] = c2;
      psiv[k] = CA_ATAN2(c1, c0);
      wr[k] = 0;
      flg[k] = 0;
    }
    // B: candidates of every close vehicle (a wave per vehicle, lanes over j;
    // the lane's own points j held in registers). The squared distance
    // decides outside a 2^-40 band around the threshold; inside it (and for
    // NaN) the exact test of safety.cpp:421 runs
    {
      const double thr = sp.d_avoid_thresh;
      const bool band = thr > 0.0 && thr < 1e150;  // (else always the exact test)
      const double lo2 = band ? (thr * (1.0 - 0x1p-40)) * (thr * (1.0 - 0x1p-40)) : -1.0;
      const double hi2 = band ? (thr * (1.0 + 0x1p-40)) * (thr * (1.0 + 0x1p-40)) : __builtin_inf();
      double qj0[2], qj1[2];
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const int j = lane + 64 * w;
        qj0[w] = (w < NW && j < n) ? q[3 * j] : 0.0;
        qj1[w] = (w < NW && j < n) ? q[3 * j + 1] : 0.0;
      }
    for (int k = wave; k < nc; k += kW) {
      const int v = cl[k];
      const double qv0 = q[3 * v], qv1 = q[3 * v + 1];
      unsigned long long mw[2] = {0ull, 0ull};
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        if (w >= NW) break;
        const int j = lane + 64 * w;
        bool cand = false;
        if (j < n && j != v) {
          const double dx = qj0[w] - qv0, dy = qj1[w] - qv1;
          const double d2 = dx * dx + dy * dy;
          cand = d2 < lo2;
          if (!cand && !(d2 > hi2)) cand = !(sqrt(d2) > thr);
        }
        mw[w] = __ballot(cand);
      }
      const int c = __popcll(mw[0]) + __popcll(mw[1]);
      // the vehicle's run of pairs: any order of vehicles serves (each
      // vehicle's sectors are resolved on their own), so a running total
      // hands out the runs; when every pair fits one batch (the usual case)
      // the list is written here and the prefix and list passes are skipped
      int o = 0;
      if (lane == 0) {
        cmk[2 * k] = mw[0];
        cmk[2 * k + 1] = mw[1];
        cnt[k] = c;
        o = atomicAdd(&misc[6], c);
        off[k] = o;
      }
      o = __builtin_amdgcn_readfirstlane(o);
      if (o + c <= kCaPairCap) {
        int base = o;
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          const unsigned long long m = mw[w];
          if ((m >> lane) & 1ull)
            pairs[base + (int)__builtin_amdgcn_mbcnt_hi(
                             (unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                (uint16_t)((k << 8) | (64 * w + lane));
          base += __popcll(m);
        }
      }
    }
    }
    __syncthreads();
    const int npairs = misc[6];
    const bool one = npairs <= kCaPairCap;  // workgroup-uniform: one batch, listed in B
    if (!one && wave == 0) {  // exclusive prefix of the counts (nc <= 128: two per lane)
      int base = 0;
      for (int k0 = 0; k0 < nc; k0 += 64) {
        const int k = k0 + lane;
        const int c = k < nc ? cnt[k] : 0;
        int x = c;
        for (int o = 1; o < 64; o <<= 1) {
          const int y = __shfl_up(x, o, 64);
          if (lane >= o) x += y;
        }
        if (k < nc) off[k] = base + x - c;
        base += __shfl(x, 63, 64);
      }
      if (lane == 0) off[nc] = base;
    }
    if (!one) __syncthreads();
    unsigned mine = 0;  // commands this thread modified (E)
    // batches of whole vehicles with at most kCaPairCap pairs
    for (int k0 = ACL_CA_STOP < 2 ? nc : 0; k0 < nc;) {
      int k1 = k0 + 1;
      if (one) k1 = nc;
      else
        while (k1 < nc && off[k1 + 1] - off[k0] <= kCaPairCap) ++k1;
      const int p0 = one ? 0 : off[k0], np = one ? npairs : off[k1] - p0;
      // the batch's pair list (a wave per vehicle; listed in B when `one`)
      for (int k = k0 + wave; k < (one ? k0 : k1); k += kW) {
        int base = off[k] - p0;
        for (int w = 0; w < NW; ++w) {
          const unsigned long long m = cmk[2 * k + w];
          if ((m >> lane) & 1ull)
            pairs[base + (int)__builtin_amdgcn_mbcnt_hi(
                             (unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                (uint16_t)(((k - k0) << 8) | (64 * w + lane));
          base += __popcll(m);
        }
      }
      if (tid < 5) misc[8 + tid] = 0;
      if (!one) __syncthreads();  // (one: the barrier after B ordered the list)
      if (ACL_CA_STOP < 3) {
        k0 = k1;
        continue;
      }
      // C: the sector edges of every pair
      #pragma unroll 1
      for (int p = tid; p < np; p += kCaPT) {
        const int pr = pairs[p];
        const int k = k0 + (pr >> 8), j = pr & 0xFF;
        const int v = cl[k];
        const double dx = q[3 * j] - q[3 * v], dy = q[3 * j + 1] - q[3 * v + 1];
        const double dd = sqrt(dx * dx + dy * dy);
        const double theta = CA_ATAN2(dy, dx);
        const double x = sp.r_keep_out / dd;
        const double alpha = fabs(CA_ASIN(x < 1.0 ? x : 1.0));
        const double beg = wrap_to_pi(theta - alpha);
        const double end = wrap_to_pi(theta + alpha);
        ang[2 * p] = beg;
        ang[2 * p + 1] = end;
        if (beg > end) atomicAdd(&wr[k], 1);
        if (beg != beg || end != end) atomicOr(&flg[k], 1);
      }
      __syncthreads();
      // resolve classes: edges m = 2 cnt + 2 wraps
      for (int k = k0 + tid; k < k1; k += kCaPT) {
        const int m = 2 * (cnt[k] + wr[k]);
        const int cls =
            (flg[k] & 1) || m > 64 ? 4 : (m > 32 ? 3 : (m > 16 ? 2 : (m > 8 ? 1 : 0)));
        if (m > 0) lists[cls * n + atomicAdd(&misc[8 + cls], 1)] = (uint16_t)k;
      }
      __syncthreads();
      if (ACL_CA_STOP < 4) {
        k0 = k1;
        continue;
      }
      // D: 8 / 4 / 2 / 1 vehicles per wave
      {
        const int n8 = misc[8], n16 = misc[9], n32 = misc[10], n64 = misc[11];
        const int g8 = (n8 + 7) >> 3, g16 = (n16 + 3) >> 2, g32 = (n32 + 1) >> 1;
        for (int item = wave; item < g8 + g16 + g32 + n64; item += kW) {
          int cls, slot, S;
          if (item < g8) { cls = 0; S = 8; slot = 8 * item + (lane >> 3); }
          else if (item < g8 + g16) { cls = 1; S = 16; slot = 4 * (item - g8) + (lane >> 4); }
          else if (item < g8 + g16 + g32) {
            cls = 2; S = 32; slot = 2 * (item - g8 - g16) + (lane >> 5);
          } else { cls = 3; S = 64; slot = item - g8 - g16 - g32; }
          const int ncls = misc[8 + cls];
          const bool has = slot < ncls;
          const int k = has ? lists[cls * n + slot] : k0;
          const int c2 = has ? 2 * cnt[k] : 0, m = has ? c2 + 2 * wr[k] : 0;
          const int e = lane & (S - 1);
          const double* av = ang + 2 * (off[k] - p0);
          double edge = 0.0;
          const double psi = psiv[k];
          int res;
          if (S == 8) res = ca_resolve_seg<8>(lane, m, c2, av, wr[k] > 0, psi, edge);
          else if (S == 16) res = ca_resolve_seg<16>(lane, m, c2, av, wr[k] > 0, psi, edge);
          else if (S == 32) res = ca_resolve_seg<32>(lane, m, c2, av, wr[k] > 0, psi, edge);
          else res = ca_resolve_seg<64>(lane, m, c2, av, wr[k] > 0, psi, edge);
          if (has && e == 0) {
            flg[k] |= res << 8;
            edg[k] = edge;
          }
        }
      }
      // more than 64 edges or a NaN angle: one vehicle at a time (wave 0) on
      // the general and serial paths over its slots in sA / sS
      if (wave == 0) {
        const int ng = misc[12];
        for (int s = 0; s < ng; ++s) {
          const int k = lists[4 * n + s];
          const int c2 = 2 * cnt[k], m = c2 + 2 * wr[k];
          for (int e = lane; e < m; e += 64) {
            if (e < c2) {
              sA[e] = ang[2 * (off[k] - p0) + e];
              sS[e] = (e & 1) ? -1 : +1;
            } else {
              sA[e] = ((e - c2) & 1) ? kPi : -kPi;
              sS[e] = ((e - c2) & 1) ? -1 : +1;
            }
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
          double c0 = cmd[3 * k], c1 = cmd[3 * k + 1], c2d = cmd[3 * k + 2];
          const double u0 = c0, u1 = c1;
          bool mod = false;
          if (flg[k] & 1) {
            if (lane == 0) mod = ca_resolve_serial(m, sA, sS, wr[k] > 0, c0, c1, c2d);
            mod = __shfl(mod ? 1 : 0, 0, 64) != 0;
            c0 = __shfl(c0, 0, 64);
            c1 = __shfl(c1, 0, 64);
            c2d = __shfl(c2d, 0, 64);
          } else {
            mod = ca_resolve_general(lane, m, sA, sS, tA, tS, wr[k] > 0, c0, c1, c2d);
          }
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
          if (lane == 0 && mod) {
            // the paths applied the command themselves: store it as a
            // resolved outcome (3: explicit command in cmd)
            flg[k] |= 3 << 8;
            cmd[3 * k] = c0; cmd[3 * k + 1] = c1; cmd[3 * k + 2] = c2d;
          }
          (void)u0; (void)u1;
        }
      }
      __syncthreads();
      // E: the modified commands
      #pragma unroll 1
      for (int k = k0 + tid; k < (ACL_CA_STOP < 5 ? k0 : k1); k += kCaPT) {
        const int res = flg[k] >> 8;
        if (!res) continue;
        const int v = cl[k];
        double c0 = cmd[3 * k], c1 = cmd[3 * k + 1], c2 = cmd[3 * k + 2];
        if (res == 1) {
          const double edge = edg[k];
          const double umag = sqrt(c0 * c0 + c1 * c1);
          c0 = umag * CA_COS(edge);
          c1 = umag * CA_SIN(edge);
        } else if (res == 2) {
          c0 = c1 = 0.0;
          c2 = 0.0;
        }
        if (P.u_safe) {
          double* o = P.u_safe + ((size_t)b * n + v) * 3;
          o[0] = c0; o[1] = c1; o[2] = c2;
        }
        if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 1;
        ++mine;
      }
      __syncthreads();  // the batch's arrays are reused
      k0 = k1;
    }
    const unsigned long long mm = __ballot(mine != 0u);
    unsigned tot = mine;
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    if (lane == 0 && mm) atomicAdd(reinterpret_cast<unsigned*>(&misc[5]), tot);
    __syncthreads();
    if (tid == 0 && misc[5]) {
      reinterpret_cast<unsigned*>(&P.status[b])[2] += (unsigned)misc[5] << 16;
      P.status[b].flags |= (uint32_t)ACL_SWARM_CA_ACTIVE;
    }
    __syncthreads();  // q, cl and misc are rewritten for the next listed swarm
  }
  ca_list_release(P, count);
}

// acl_control_batch's hand-off: P must be a permutation (else BAD_INPUT and
// zero commands, as for the auction's P_in); the inverse assignment is the
// shared row the gain kernel reads. Episodes: swarms flagged in P.keep keep
// their per-vehicle rows.
__global__ void __launch_bounds__(256) control_prep_kernel(const CtlParams P,
                                                           const uint16_t* Pg) {
  __shared__ unsigned long long seen[kMaxNWide / 64];
  __shared__ int bad;
  const int n = P.n, b = blockIdx.x, tid = threadIdx.x;
  if (tid < kMaxNWide / 64) seen[tid] = 0ull;
  if (tid == 0) bad = 0;
  __syncthreads();
  if (P.keep && P.keep[(size_t)b * P.keep_stride]) {
    // an episode swarm flying per-vehicle tables (already in wsRows)
    if (tid == 0) {
      const_cast<uint8_t*>(P.wsMode)[b] = 1;
      P.status[b] = acl_swarm_status_t{};
    }
    return;
  }
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
// n > 128: every swarm in the directed walk on 1024-thread workgroups
// (ACL_WIDE_DIRECTED=0, diagnostic builds: the 256-thread pair kernel)
#ifndef ACL_WIDE_DIRECTED
#define ACL_WIDE_DIRECTED 1
#endif

hipError_t launch_control(const CtlParams& P, int nb, int which, hipStream_t stream) {
  // the control kernels' dynamic-LDS limit, once per device (not per launch)
  static PerDeviceOnce once;
  const hipError_t ea = once.run([] {
    for (const void* k :
         {(const void*)gain_pair_kernel<true, true, kCtlBlock>,
          (const void*)gain_pair_kernel<true, false, kCtlBlock>,
          (const void*)gain_pair_kernel<false, true, kCtlBlock>,
          (const void*)gain_pair_kernel<false, false, kCtlBlock>,
          (const void*)gain_kernel<5, true, 1024>, (const void*)gain_kernel<5, false, 1024>,
          (const void*)gain_kernel<9, true, 1024>, (const void*)gain_kernel<9, false, 1024>,
          (const void*)gain_kernel<5, true, kCtlBlock>, (const void*)gain_kernel<5, false, kCtlBlock>,
          (const void*)gain_kernel<9, true, kCtlBlock>, (const void*)gain_kernel<9, false, kCtlBlock>,
          (const void*)ca_pair_kernel, (const void*)ca_kernel}) {
      hipFuncAttributes fa;
      hipError_t r = hipFuncGetAttributes(&fa, k);
      if (r != hipSuccess) return r;
      r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - (int)fa.sharedSizeBytes);
      if (r != hipSuccess) return r;
    }
    return hipSuccess;
  });
  if (ea != hipSuccess) return ea;
  if (which == 0 || which == 2) {
    CtlParams Q = P;
    Q.nb = nb;
    Q.only_nonuniform = which == 2 ? 1 : 0;
    if (which == 0 && P.gain_planes == 5 && ACL_GAIN_PAIR && (P.n <= kMaxN || !ACL_WIDE_DIRECTED)) {
      // uniform swarms: one evaluation per undirected edge; then gain_kernel
      // for the swarms whose vehicles hold different assignments
      const bool tiled = P.gains_tiled != nullptr && P.n <= kMaxN;
#ifndef ACL_PAIR_SMALL_BLOCK
#define ACL_PAIR_SMALL_BLOCK 64  // threads per swarm for n <= 32 (one wave; episode n = 20: 81 -> 70 us per step)
#endif
      constexpr int kSB = ACL_PAIR_SMALL_BLOCK > 0 ? ACL_PAIR_SMALL_BLOCK : kCtlBlock;
      const bool small = ACL_PAIR_SMALL_BLOCK > 0 && P.n <= 32;
      const int pw = small ? kSB / 64 : kCtlWaves;
      const PairLayout PL = make_pair_layout(P.n, pw, tiled);
      const int lds = std::max(PL.total, make_gain_layout(P.n, pw).total);
      const bool gm = P.gate_margin != nullptr;
#define ACL_PAIR(T_, G_)                                                                     \
  do {                                                                                       \
    if (small)                                                                               \
      hipLaunchKernelGGL((gain_pair_kernel<T_, G_, kSB>), dim3(nb), dim3(kSB), lds, stream, Q); \
    else                                                                                     \
      hipLaunchKernelGGL((gain_pair_kernel<T_, G_, kCtlBlock>), dim3(nb), dim3(kCtlBlock), lds, \
                         stream, Q);                                                         \
  } while (0)
      if (tiled && gm) ACL_PAIR(true, true);
      else if (tiled) ACL_PAIR(true, false);
      else if (gm) ACL_PAIR(false, true);
      else ACL_PAIR(false, false);
#undef ACL_PAIR
      return hipGetLastError();  // the pair kernel also took the per-vehicle swarms
    }
    // n > 128: 16 waves per swarm (the directed walk keeps per-lane sums;
    // the pair kernel's per-wave accumulators would not fit the LDS)
    const bool big = P.n > kMaxN;
    const GainLayout L = make_gain_layout(P.n, big ? 16 : kCtlWaves);
    const bool gm = P.gate_margin != nullptr;
    const int gb = nb;
#define ACL_GAIN(NP_, G_)                                                                    \
  do {                                                                                       \
    if (big) {                                                                               \
      hipLaunchKernelGGL((gain_kernel<NP_, G_, 1024>), dim3(gb), dim3(1024), L.total, stream, Q); \
    } else {                                                                                 \
      hipLaunchKernelGGL((gain_kernel<NP_, G_, kCtlBlock>), dim3(gb), dim3(kCtlBlock), L.total, \
                         stream, Q);                                                         \
    }                                                                                        \
  } while (0)
    if (P.gain_planes == 5 && gm) ACL_GAIN(5, true);
    else if (P.gain_planes == 5) ACL_GAIN(5, false);
    else if (gm) ACL_GAIN(9, true);
    else ACL_GAIN(9, false);
#undef ACL_GAIN
  } else {
    // a fixed grid striding over the device-side count of listed swarms
#ifndef ACL_CA_PAIR_MIN_N
#define ACL_CA_PAIR_MIN_N 33  // smaller swarms: the per-vehicle ca_kernel (episode n = 20: 81 -> 77 us per step)
#endif
    if (P.n <= kMaxN && P.n >= ACL_CA_PAIR_MIN_N) {
      const int lp = ca_pair_layout(P.n).total;
      hipLaunchKernelGGL(ca_pair_kernel, dim3(nb < ACL_CA_PAIR_GRID ? nb : ACL_CA_PAIR_GRID), dim3(kCaPT), lp,
                         stream, P);
      return hipGetLastError();
    }
    const int lds = ca_layout(P.n).total;
    hipLaunchKernelGGL(ca_kernel, dim3(nb < ACL_CA_GRID ? nb : ACL_CA_GRID), dim3(64 * kCaWaves),
                       lds, stream, P);
  }
  return hipGetLastError();
}

}  // namespace acl_amd
