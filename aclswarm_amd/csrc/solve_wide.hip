// solve_wide.hip -- the batched auction for 128 < n <= 512 (config C4, N=500).
//
// Same algorithm and exactness as solve.hip (alignment, prices, CBAA to the
// fixed point, adoption; see that file and SURVEY.md App. A), re-laid out
// for swarms whose CBAA tables do not fit LDS. Only the `who` table lives in
// the solve workspace (HBM; 0.5 MB per swarm at n = 500, so the resident
// swarms' tables stay within the last-level cache):
//
//   T  [j][u] u16   `who` table in 8 x 8 tiles (one 128-byte line: tasks
//                   j..j+7 x vehicles u..u+7, tix): a dirty-column update
//                   reads and rewrites its column in place (8 lines per 64
//                   vehicles), a re-select reads its vehicle's row (8 lines
//                   per 64 tasks instead of 64 with a column-major table)
//
// Sparse columns (round 5). A column whose update leaves at most kWSparseK
// vehicles holding something other than one base `who` is kept in LDS
// instead: the base (cuw[j]) and the exceptions (vehicle, who) -- the table
// T is not written for it and is stale there. A bid on a sparse column is
// appended to the select phase's bid list (LDS) and applied by the column's
// next update; a column with more exceptions is written to T in full and
// read from it (dense) until an update makes it sparse again. At N = 500
// nearly every column update leaves 0-2 exceptions (a vehicle misses ~1 of
// 499 neighbours), so the column reads and write-backs that moved most of
// the table's HBM traffic (one 128-byte line per 8 vehicles, 16 bytes of it
// used) leave the memory system; START needs no table reset.
//
// The price matrix (1 MB per swarm at n = 500) is not stored: a price is
// recomputed from LDS where it is needed (wprice: vehicle v's alignment
// applied to formation point j, the same f64 operations as the n <= 128
// kernel's price phase, so every price is bit-identical). Recomputing costs
// ~40 f64 operations; reading a stored price was a random HBM access.
//
// Two launches (round 4). align_wide_kernel (one 1 024-thread workgroup per
// swarm) loads the formation, checks P_in, and leaves in the workspace every
// vehicle's alignment (R, t), the vehicle-space closed-neighbourhood masks
// (8 words per vehicle) and the smallest alignment gap. solve_wide_kernel
// (8 waves per swarm) keeps only what the CBAA rounds touch in LDS -- points,
// q, the neighbourhood masks, the column price cache and the masks: ~62 KB at
// n = 500, so two swarms share a CU and one's round barriers and table
// latency hide behind the other's work (the kernel waited half its time with
// one 16-wave swarm per CU) -- and reads the alignments from the workspace
// (24 KB per swarm, L2-resident; wave-uniform in the selects). Indices are
// u16 (the reference's u8 vehidx_t caps N at 255; widened as SURVEY.md 8d
// prescribes for C4).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/aclswarm_amd.h"
#include "common.h"
#include "control_params.h"
#include "pair_fused.h"
#include "umeyama_dev.h"

namespace acl_amd {

enum { W_RCH = 3 /* misc[3..4]: a column changed in a round of that parity */,
       W_BIG = 12 /* a coordinate or alignment entry is not below 1e100 */,
       W_TCOL = 13 /* the round's next dirty column (ticket) */,
       W_TSEL = 14 /* the round's next re-select (ticket) */,
       W_NBID = 16 /* misc[16..17]: bids in the bid list of that parity */ };

// exceptions a sparse column holds (LDS: 4 bytes each per column)
constexpr int kWSparseK = 4;


constexpr int kWBlock = 512;    // solve_wide_kernel: 8 waves per swarm, 2 swarms per CU
constexpr int kWWaves = kWBlock / 64;
constexpr int kWABlock = 512;   // align_wide_kernel: a lane per vehicle, two swarms per CU
constexpr int kWMaxW = kMaxNWide / 64;  // 64-bit words per bitmask row
constexpr int kWLevels = 3;

// align_wide_kernel's results in the workspace (WsLayout::align, per swarm)
struct WsWide {
  size_t out, vadj, gal, flags;
};
__host__ __device__ inline WsWide ws_wide(int n) {
  const int NW = (n + 63) >> 6;
  WsWide w;
  w.out = 0;                                   // [n][6] f64 R, t per vehicle
  w.vadj = (size_t)n * 48;                     // [NW][n] u64 closed neighbourhoods
  w.gal = w.vadj + (size_t)NW * n * 8;         // u64 bits of the smallest alignment gap
  w.flags = w.gal + 8;                         // u32: bit 0 bad input, bit 1 p not finite
  return w;
}

// index of entry (task j, vehicle u) of the tiled `who` table
__host__ __device__ __forceinline__ size_t tix(int n, int j, int u) {
  const int n8 = (n + 7) >> 3;
  return (((size_t)(j >> 3) * n8 + (u >> 3)) << 6) + ((j & 7) << 3) + (u & 7);
}
__host__ __device__ __forceinline__ int tix_size(int n) {
  const int n8 = (n + 7) >> 3;
  return n8 * n8 * 64;
}

__host__ __device__ inline int wal(int x) { return (x + 15) & ~15; }

// align_wide_kernel's LDS
struct WALayout {
  int p, qf, adjF, Pin, seen, misc, total;
};
__host__ __device__ inline WALayout make_walayout(int n) {
  const int NW = (n + 63) >> 6;
  WALayout L;
  int o = 0;
  L.p = o;     o = wal(o + n * 24);
  L.qf = o;    o = wal(o + n * 24);   // q in formation order
  L.adjF = o;  o = wal(o + n * NW * 8);
  L.Pin = o;   o = wal(o + n * 2);
  L.seen = o;  o = wal(o + NW * 8);   // permutation check
  L.misc = o;  o = wal(o + 64);
  L.total = o;
  return L;
}

// solve_wide_kernel's LDS
struct WLayout {
  int p, qv, vadj, Pin, Ptin, ccw, ccp, cuw, valid, masks, seen, misc, ecnt, elist, bids, xcnt, total;
};

__host__ __device__ inline WLayout make_wlayout(int n) {
  const int NW = (n + 63) >> 6;
  WLayout L;
  int o = 0;
  L.p = o;     o = wal(o + n * 24);
  L.qv = o;    o = wal(o + n * 24);   // q in vehicle order
  L.vadj = o;  o = wal(o + n * NW * 8);  // [word][vehicle]: conflict-free per-lane reads
  L.Pin = o;   o = wal(o + n * 2);
  L.Ptin = o;  o = wal(o + n * 2);
  L.ccw = o;   o = wal(o + n * 2);    // column price cache: a holder of task j
  L.ccp = o;   o = wal(o + n * 4);    // and its price for j
  L.cuw = o;   o = wal(o + n * 2);    // a sparse column's base `who` (unif: every vehicle's)
  L.valid = o; o = wal(o + n);
  L.masks = o; o = wal(o + 6 * NW * 8);  // dmask[2][NW], obm[2][NW], unif[NW], spm[NW]
  L.seen = o;  o = wal(o + kWWaves * NW * 8);         // per-wave validity checks
  L.misc = o;  o = wal(o + 128);
  L.ecnt = o;  o = wal(o + n);                         // exceptions of a sparse column
  L.elist = o; o = wal(o + n * kWSparseK * 4);         // [j][K] vehicle << 16 | who
  L.bids = o;  o = wal(o + 2 * n * 4);                 // [2][n] bid lists: vehicle << 16 | task
  L.xcnt = o;  o = wal(o + n * 4);                     // [n] sparse columns a vehicle is an exception in
  L.total = o;
  return L;
}

// The price of task j for vehicle v (C[v][j] of the n <= 128 kernel, bit for
// bit): v's alignment (R, t) = out[6 v..] applied to formation point j, the
// squared distance to v's position qv[3 v..], then acl_price (common.h).
// pfin: every formation coordinate is finite, so the 0 * p terms of the
// aligned point drop (auction.hip phase 2).
struct WPrice {
  const double* out;
  const double* qv;
  const double* p;
  bool pfin;
  __device__ __forceinline__ float operator()(int v, int j) const {
    const double* o = out + 6 * v;
    const double* q = qv + 3 * v;
    const double px = p[3 * j], py = p[3 * j + 1], pz = p[3 * j + 2];
    double dx, dy, dz;
    if (pfin) {
      dx = q[0] - ((o[0] * px + o[1] * py) + o[4]);
      dy = q[1] - ((o[2] * px + o[3] * py) + o[5]);
      dz = q[2] - pz;
    } else {
      const double ax = ((o[0] * px + o[1] * py) + 0.0 * pz) + o[4];
      const double ay = ((o[2] * px + o[3] * py) + 0.0 * pz) + o[5];
      const double az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0;
      dx = q[0] - ax; dy = q[1] - ay; dz = q[2] - az;
    }
    return acl_price((dx * dx + dy * dy) + dz * dz);
  }
};

// selectTaskAssignment (auctioneer.cpp:517-542) on vehicle v's row: the
// first task j maximizing C[v][j] among C[v][j] > 0 and C[v][j] > price_j
// (price_j = C[w][j] of the task's holder w in v's table).
// `fresh`: the row is all `none` (the START bid). Tracks the margin of the
// decisive comparisons (include/aclswarm_amd.h) in m.
// Entry (task j, vehicle u) of the table: a sparse column's exception or its
// base, else T (see the header).
struct WTable {
  const uint16_t* T;
  const uint16_t* cuw;
  const unsigned char* ecnt;
  const unsigned* elist;
  const unsigned long long* spm;
  const unsigned* xcnt;  // [u]: sparse columns whose exception list holds vehicle u
  int n;
  __device__ __forceinline__ bool sparse(int j) const { return (spm[j >> 6] >> (j & 63)) & 1ull; }
  __device__ __forceinline__ unsigned sparse_entry(int j, int u) const {
    unsigned w = cuw[j];
    const int ne = ecnt[j];
    const uint4 e4 = *reinterpret_cast<const uint4*>(elist + j * kWSparseK);
    const unsigned e[4] = {e4.x, e4.y, e4.z, e4.w};
    static_assert(kWSparseK == 4, "one 16-byte read per column");
#pragma unroll
    for (int k = 0; k < kWSparseK; ++k)
      if (k < ne && (e[k] >> 16) == (unsigned)u) w = e[k] & 0xFFFFu;
    return w;
  }
  __device__ __forceinline__ unsigned operator()(int j, int u) const {
    return sparse(j) ? sparse_entry(j, u) : (unsigned)T[tix(n, j, u)];
  }
};

template <bool MG>
__device__ int wide_select(int n, int NW, int v, int lane, const WPrice& price,
                           const uint16_t* T, const uint16_t* ccw, const float* ccp,
                           const WTable& tab, bool fresh, MarginPair& m) {
  unsigned key[kWMaxW];
  float cvs[kWMaxW], prs[kWMaxW];
  bool other[kWMaxW];
  unsigned lm = 0u;
  int wv[kWMaxW];
  // row v of the tiled table: task j = lane + 64 c at Tv[lo + c * 512 n8];
  // a sparse column's entry comes from LDS -- its base, unless v is one of
  // its exceptions (only looked up when v is an exception somewhere) -- so
  // only the dense columns' entries are read from the table
  const int n8 = (n + 7) >> 3;
  const uint16_t* Tv = T + (((v >> 3) << 6) + (v & 7));
  const int lo = (((lane >> 3) * n8) << 6) + ((lane & 7) << 3);
  const bool vx = !fresh && tab.xcnt[v] != 0;  // wave-uniform
  if (vx) {
#pragma unroll
    for (int c = 0; c < kWMaxW; ++c) {
      const int j = lane + 64 * c;
      if (c >= NW || j >= n) {
        wv[c] = n;
      } else {
        const bool spl = (tab.spm[c] >> lane) & 1ull;
        wv[c] = spl ? (int)tab.sparse_entry(j, v) : (int)Tv[lo + c * (n8 << 9)];
      }
    }
  } else {
#pragma unroll
    for (int c = 0; c < kWMaxW; ++c) {
      const int j = lane + 64 * c;
      if (fresh || c >= NW || j >= n) {
        wv[c] = n;
      } else {
        const bool spl = (tab.spm[c] >> lane) & 1ull;
        wv[c] = spl ? (int)tab.cuw[j] : (int)Tv[lo + c * (n8 << 9)];
      }
    }
  }
#pragma unroll
  for (int c = 0; c < kWMaxW; ++c) {
    key[c] = 0u;
    cvs[c] = 0.0f;
    prs[c] = 0.0f;
    other[c] = false;
    const int j = lane + 64 * c;
    if (c < NW && j < n) {
      const float cv = price(v, j);
      const int w = wv[c];
      // the column price cache (ccw, ccp: one holder of task j and its
      // price, a pure function of the pair) saves most holder prices
      const float pr = w < n ? (w == ccw[j] ? ccp[j] : price(w, j)) : 0.0f;
      if (cv > 0.0f && cv > pr) key[c] = __float_as_uint(cv);
      cvs[c] = cv;
      prs[c] = pr;
      other[c] = w != v;
    }
    lm = lm > key[c] ? lm : key[c];
  }
  const unsigned M = wave_max_u32(lm);
  int js = -1;
  if (M != 0u) {
#pragma unroll
    for (int c = 0; c < kWMaxW; ++c) {
      const unsigned long long e = __ballot(key[c] == M);
      if (js < 0 && e) js = 64 * c + __ffsll((long long)e) - 1;
    }
  }
  const float cmax = __uint_as_float(M);
#pragma unroll
  for (int c = 0; c < kWMaxW; ++c) {
    // branch-free (margin_track_sel, common.h): the selected task vs its
    // price; an eligible task that lost vs the maximum; a task that would
    // win if it became eligible vs its price
    const int j = lane + 64 * c;
    const bool isjs = other[c] && j == js;
    const bool elig = other[c] && !isjs && key[c] != 0u;
    const bool near = other[c] && !isjs && key[c] == 0u && cvs[c] > 0.0f &&
                      (js < 0 || cvs[c] > cmax || (cvs[c] == cmax && j < js));
    if (MG)
      margin_track_sel(m, isjs ? cvs[c] : (elig ? cmax : prs[c]), isjs ? prs[c] : cvs[c],
                       isjs || elig || near);
  }
  return js;
}

// ---- the fused control phase (n > 128, FUSE) --------------------------------
// DistCntrl::compute (distcntrl.cpp:46-102), saturation (safety.cpp:185-196)
// and the first collision test (safety.cpp:412-430) of a swarm whose
// vehicles all adopted one assignment, in the auction's workgroup right after
// its adoption: with two swarms per CU one swarm's gain stream (the HBM
// bytes) runs beside the other's latency-bound rounds, instead of all of it
// in a launch after every auction. The directed walk: a wave per formation
// row i (vehicle Pt[i]), lanes over the 64 columns of one adjacency word per
// pass, a lane's record = the row's base + the bits below it (v_mbcnt), the
// next pass's 40-byte records loaded before this pass's math; the wave's sums
// by DPP. p and q (vehicle order) stay where the auction left them; the rest
// of the image overlays the auction's dead tables (<= 80 KB at n = 512, so two
// swarms still share a CU). Parity as the other gain kernels: gates and gate
// margin on the same expressions (pair_e, gate_decide_t), u / u_safe 1e-5.
struct WCLayout {
  int adj, rowbase, Pt, uo, atab, cst, flags, gmw, caw, total;
};
__host__ __device__ inline WCLayout make_wclayout(int n, int start) {
  const int NW = (n + 63) >> 6;
  WCLayout L;
  int o = start;
  L.adj = o;     o = wal(o + n * NW * 8);   // formation rows (masked past n)
  L.rowbase = o; o = wal(o + (n + 1) * 4);  // record base of every row
  L.Pt = o;      o = wal(o + n * 2);        // formation point -> vehicle
  L.uo = o;      o = wal(o + n * 24);       // DistCntrl's u per vehicle
  L.atab = o;    o = wal(o + ACL_ATAB_N * 8);
  L.cst = o;     o = wal(o + FC_N * 8);     // the walk's constants (pair_fused.h FC_*)
  L.flags = o;   o = wal(o + 4);            // bit 0: a q coordinate is not finite
  L.gmw = o;     o = o + 8;
  L.caw = o;     o = wal(o + 4);
  L.total = o;
  return L;
}

template <bool GM>
__device__ __forceinline__ void wide_control(KCtlParams* Pp, int b, int f, unsigned char* smem,
                                             const double* p, const double* q, int cstart,
                                             const uint16_t* wsPt) {
  KCtlParams& P = *Pp;
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const WCLayout L = make_wclayout(n, cstart);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adj);
  int* rowbase = reinterpret_cast<int*>(smem + L.rowbase);
  uint16_t* Pt = reinterpret_cast<uint16_t*>(smem + L.Pt);
  double* uo = reinterpret_cast<double*>(smem + L.uo);
  double* atab = reinterpret_cast<double*>(smem + L.atab);
  double* cst = reinterpret_cast<double*>(smem + L.cst);
  unsigned* flags = reinterpret_cast<unsigned*>(smem + L.flags);
  unsigned long long& gmw = *reinterpret_cast<unsigned long long*>(smem + L.gmw);
  unsigned* caw = reinterpret_cast<unsigned*>(smem + L.caw);
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;

  for (int k = tid; k < ACL_ATAB_N; k += kWBlock) atab[k] = ACL_ATAB_AT(k);
  if (tid == 0) {
    *flags = 0u;
    *caw = 0u;
    if (GM) gmw = (unsigned long long)__double_as_longlong(__builtin_inf());
  }
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
    const uint64_t* ga = P.adj + (size_t)f * n * NW;
    for (int k = tid; k < n * NW; k += kWBlock) {
      unsigned long long x = ga[k];
      if (k % NW == NW - 1) x &= lastmask;
      adjF[k] = x;
    }
    bool qbad = false;
    for (int i = tid; i < n; i += kWBlock) {
      Pt[i] = wsPt[i];
      qbad |= !(__builtin_isfinite(q[3 * i]) && __builtin_isfinite(q[3 * i + 1]) &&
                __builtin_isfinite(q[3 * i + 2]));
    }
    if (__any(qbad) && lane == 0) atomicOr(flags, 1u);
  }
  __syncthreads();
  if (wave == 0) {  // record base of every row: a scan of the row popcounts
    int base = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      int cnt = 0;
      if (i < n)
        for (int w = 0; w < NW; ++w) cnt += __popcll(adjF[i * NW + w]);
      // inclusive prefix on DPP (row_shr 1, 2, 4, 8, then row_bcast 15 / 31)
      int x = cnt;
      x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);
      x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);
      x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);
      x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);
      x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
      x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
      if (i < n) rowbase[i] = base + x - cnt;
      base += __builtin_amdgcn_readlane(x, 63);
    }
    if (lane == 0) rowbase[n] = base;
  }
  __syncthreads();
  const bool qfin = (*flags & 1u) == 0u;
  const int E = __builtin_amdgcn_readfirstlane(rowbase[n]);
  const double* G = P.gains + 5 * P.gain_off[f];
  const __amdgpu_buffer_rsrc_t grs =
      __builtin_amdgcn_make_buffer_rsrc((void*)G, (short)0, 5 * E * 8, 0x00020000);
  double gmxy = __builtin_inf(), gmz = __builtin_inf();
  for (int i = wave; i < n; i += kWWaves) {
    const int v = Pt[i];
    const double pix = p[3 * i], piy = p[3 * i + 1], piz = p[3 * i + 2];
    const double Ni = pix * pix + piy * piy, Nzi = piz * piz;
    const double qv0 = q[3 * v], qv1 = q[3 * v + 1], qv2 = q[3 * v + 2];
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    int eb = __builtin_amdgcn_readfirstlane(rowbase[i]);  // the pass's first record
    unsigned long long word = uni_u64(adjF[i * NW]);
    Rec5 X;
    load_rec5(grs, lanebit_u64(word) ? (int)__umul24((unsigned)eb + __builtin_amdgcn_mbcnt_hi(
                                                         (unsigned)(word >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)word, 0u)),
                                                     40u)
                                     : 0x40000000, X);
    int deg = 0;
#pragma unroll 1
    for (int t = 0; t < NW; ++t) {
#pragma clang fp contract(fast)
      const unsigned long long wc = word;
      const int ebn = eb + __popcll(wc);
      deg += __popcll(wc);
      Rec5 Xn;
      if (t + 1 < NW) {  // the next pass's records, before this pass's math
        word = uni_u64(adjF[i * NW + t + 1]);
        load_rec5(grs, lanebit_u64(word) ? (int)__umul24((unsigned)ebn + __builtin_amdgcn_mbcnt_hi(
                                                             (unsigned)(word >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((unsigned)word, 0u)),
                                                         40u)
                                         : 0x40000000, Xn);
      }
      if (lanebit_u64(wc)) {
        const int j = 64 * t + lane;
        const int u = Pt[j];
        const double q0 = q[3 * u] - qv0, q1 = q[3 * u + 1] - qv1, q2 = q[3 * u + 2] - qv2;
        const double pjx = p[3 * j], pjy = p[3 * j + 1], pjz = p[3 * j + 2];
        double Nj, Nzj;
        {
#pragma clang fp contract(off)
          Nj = pjx * pjx + pjy * pjy;
          Nzj = pjz * pjz;
        }
        double Fxy = 0.0, Fz = 0.0;
        if (!ACL_DIAG_NOPAIR) {
          double e_xy, e_z;
          pair_e(q0, q1, q2, Ni, Nj, Nzi, Nzj, pix, piy, piz, pjx, pjy, pjz, pair_s2(q0, q1), e_xy,
                 e_z);
          bool gxy, gz;
          gate_decide_t<GM>(fcst(cst, FC_TXY), fcst(cst, FC_TZ), fcst(cst, FC_WIN), e_xy, e_z, q0,
                            q1, q2, Ni, Nj, Nzi, Nzj, pix, piy, piz, pjx, pjy, pjz, gxy, gz, gmxy,
                            gmz);
          if (gxy) Fxy = fcst(cst, FC_K1XY) * ACL_GAIN_ATAN(fcst(cst, FC_K2XY) * e_xy, atab);
          if (gz) Fz = fcst(cst, FC_K1Z) * ACL_GAIN_ATAN(fcst(cst, FC_K2Z) * e_z, atab);
        }
        if (qfin) {  // A q + F q (kp per vehicle); the structural zeros drop (pair_fused.h)
          a0 += X.a[1] * q1 + (X.a[0] * q0 + Fxy * q0);
          a1 += X.a[3] * q1 + (X.a[2] * q0 + Fxy * q1);
          a2 += X.a[4] * q2 + Fz * q2;
        } else {
          a0 += ((X.a[0] * q0 + X.a[1] * q1) + 0.0 * q2) + Fxy * q0;
          a1 += ((X.a[2] * q0 + X.a[3] * q1) + 0.0 * q2) + Fxy * q1;
          a2 += ((0.0 * q0 + 0.0 * q1) + X.a[4] * q2) + Fz * q2;
        }
      }
      eb = ebn;
      X = Xn;
    }
    a0 = wave_sum(a0);
    a1 = wave_sum(a1);
    a2 = wave_sum(a2);
    if (lane == 0) {
      const double kp = P.g.kp, kd = P.g.kd;
      double u0 = kp * a0, u1 = kp * a1, u2 = kp * a2;
      if (deg) {  // + kd (-vel) once per edge of the row (distcntrl.cpp:85-95)
        const double* gv = P.vel + ((size_t)b * n + v) * 3;
        const double cn = (double)deg;
        u0 += cn * (kd * (-gv[0]));
        u1 += cn * (kd * (-gv[1]));
        u2 += cn * (kd * (-gv[2]));
      }
      uo[3 * v] = u0; uo[3 * v + 1] = u1; uo[3 * v + 2] = u2;
    }
  }
  if (GM) {
    const acl_cntrl_gains_t g = kgains(P);
    gate_margin_reduce(&gmw, gate_margin_of(g, gmxy, gmz));
  }
  __syncthreads();
  if (GM && tid == 0) P.gate_margin[b] = __longlong_as_double((long long)gmw);
  // per vehicle: the command, saturation, the first collision test
  // (gain_epilogue's semantics, control_dev.h)
  const acl_safety_params_t sp = ksafety(P);
  const double thr_hi = sp.d_avoid_thresh * (1.0 + 0x1p-40);
  const double thr2hi = thr_hi * thr_hi;
  for (int v = tid; v < n; v += kWBlock) {
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
        const double d2 = dx * dx + dy * dy;
        if (j != v && !(d2 > thr2hi)) close |= !(sqrt(d2) > sp.d_avoid_thresh);
      }
    }
    if (P.u_safe) {
      double* o = P.u_safe + ((size_t)b * n + v) * 3;
      o[0] = cmd0; o[1] = cmd1; o[2] = cmd2;
    }
    if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 0;
    const unsigned long long cm = __ballot(close);
    if (lane == 0) {
      P.ca_mask[(size_t)b * NW + (v >> 6)] = cm;
      if (cm && atomicOr(caw, 1u) == 0u) P.ca_list[atomicAdd(P.ca_count, 1u)] = (unsigned)b;
    }
  }
}

// diagnostic: s_memtime at phase ends into P.stamps[b][k] (scripts/phase_profile.py)
template <class SP>
__device__ __forceinline__ void wstamp(SP& P, int b, int k) {
  if (P.stamps && threadIdx.x == 0)
    P.stamps[(size_t)b * kStampStride + k] =
        k >= kStampRt0 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
}

// diagnostic build (-DACL_WIDE_PROF=1, scripts/phase_profile.py): CBAA
// section cycles summed over the swarm's waves into P.stamps[b][kStampSec +
// 0..3] and counts into [kStampSec + 4] (columns | exact scans << 21 | re-selects << 42), [12]
// rounds
#ifndef ACL_WIDE_PROF
#define ACL_WIDE_PROF 0
#endif
#if ACL_WIDE_PROF
#define WPROF_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define WPROF_ADD(acc, x) acc += (x)
#else
#define WPROF_T(v)
#define WPROF_ADD(acc, x)
#endif

// Phases 0-1 of the n > 128 solve, one 512-thread workgroup per swarm (a
// ~58 KB LDS image: two swarms per CU): load, the permutation check, the
// vehicle-space closed neighbourhoods and every vehicle's 2-D Umeyama
// alignment (Auctioneer::alignFormation, auctioneer.cpp:347-415; Eigen's two
// sequential passes, bit for bit), left in the workspace for
// solve_wide_kernel (WsWide). The alignment: a lane per vehicle, its four
// sums of each pass as four independent chains over the same members (the
// members' values are wave-uniform LDS broadcasts, one ds_read2 per pair).
__global__ void __launch_bounds__(kWABlock, 2) align_wide_kernel(const SolveParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const WALayout L = make_walayout(n);
  const int b = P.b0 + blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  constexpr int kAW = kWABlock / 64;

  double* p = reinterpret_cast<double*>(smem + L.p);
  double* qf = reinterpret_cast<double*>(smem + L.qf);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adjF);
  uint16_t* Pin = reinterpret_cast<uint16_t*>(smem + L.Pin);
  unsigned long long* seen = reinterpret_cast<unsigned long long*>(smem + L.seen);
  int* misc = reinterpret_cast<int*>(smem + L.misc);
  const WsWide WW = ws_wide(n);
  unsigned char* wsa = P.ws + P.W.align + (size_t)b * P.W.align_stride;
  double* out = reinterpret_cast<double*>(wsa + WW.out);
  unsigned long long* vadj = reinterpret_cast<unsigned long long*>(wsa + WW.vadj);

  // a formation index out of range is a bad input like a bad P_in (nothing
  // of the formation table is read for it)
  const int f_in = P.fidx[b];
  const bool fbad = f_in < 0 || f_in >= P.F;
  const int f = fbad ? 0 : f_in;
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  bool pbad = false;  // a formation coordinate is not finite (the prices' fast path)
  {
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += kWABlock) {
      const double x = gp[k];
      pbad |= !__builtin_isfinite(x);
      p[k] = x;
    }
    const uint64_t* ga = P.adj + (size_t)f * n * NW;
    for (int k = tid; k < n * NW; k += kWABlock) {
      unsigned long long x = ga[k];
      if (k % NW == NW - 1) x &= lastmask;
      adjF[k] = x;
    }
    for (int k = tid; k < NW; k += kWABlock) seen[k] = 0ull;
    if (tid < 16) misc[tid] = 0;
  }
  __syncthreads();
  if (tid == 0 && fbad) misc[M_BAD] = 1;
  if (__any(pbad) && lane == 0) misc[M_PINF] = 1;
  for (int v = tid; v < n; v += kWABlock) {
    const unsigned pv = P.P_in[(size_t)b * n + v];
    Pin[v] = (uint16_t)pv;
    if (pv >= (unsigned)n) {
      misc[M_BAD] = 1;
    } else {
      const unsigned long long bit = 1ull << (pv & 63);
      const unsigned long long prev = atomicOr(&seen[pv >> 6], bit);
      if (prev & bit) misc[M_BAD] = 1;
      const double* gq = P.q + ((size_t)b * n + v) * 3;
      qf[3 * pv] = gq[0]; qf[3 * pv + 1] = gq[1]; qf[3 * pv + 2] = gq[2];
    }
  }
  __syncthreads();
  unsigned* wflags = reinterpret_cast<unsigned*>(wsa + WW.flags);
  if (misc[M_BAD]) {  // solve_wide_kernel writes the BAD_INPUT outputs
    if (tid == 0) *wflags = 1u;
    return;
  }
  unsigned long long* gw = reinterpret_cast<unsigned long long*>(misc + 12);  // (8-byte aligned)
  if (P.P_rows != nullptr && P.P_rows_on[b] != 0) {  // workgroup-uniform
    // the vehicles hold their own assignments (acl_solve_args_t::P_rows):
    // thread v checks its row, builds its neighbourhood and aligns with it
    double galign = 1.0;
    if (tid == 0) *gw = (unsigned long long)__double_as_longlong(1.0);
    __syncthreads();
    for (int v = tid; v < n; v += kWABlock) {
      const int i = Pin[v];
      const uint16_t* row = P.P_rows + ((size_t)b * n + v) * n;
      unsigned long long nbm[kWMaxW];
      const bool ok = align_own_row<kWMaxW>(
          n, NW, v, i, adjF + (size_t)i * NW, p, [&](int j) { return (int)row[j]; },
          [&](int u, double& x, double& y) {
            x = qf[3 * Pin[u]];
            y = qf[3 * Pin[u] + 1];
          },
          nbm, out + 6 * v, galign);
      if (!ok) misc[M_BAD] = 1;
#pragma unroll
      for (int c = 0; c < kWMaxW; ++c)
        if (c < NW) vadj[c * n + v] = nbm[c];
    }
    block_min_gap(gw, galign);
    __syncthreads();
    if (tid == 0) {
      *reinterpret_cast<unsigned long long*>(wsa + WW.gal) = *gw;
      *wflags = misc[M_BAD] ? 1u : (misc[M_PINF] ? 2u : 0u);
    }
    return;
  }
  // vehicle-space closed neighbourhoods (bidIterComplete, auctioneer.cpp:419-437)
  for (int v = wave; v < n; v += kAW) {
    const int i = Pin[v];
    for (int c = 0; c < NW; ++c) {
      const int u = lane + 64 * c;
      bool e = false;
      if (u < n) {
        const int pu = Pin[u];
        e = (u == v) || ((adjF[i * NW + (pu >> 6)] >> (pu & 63)) & 1ull);
      }
      const unsigned long long m = __ballot(e);
      if (lane == 0) vadj[c * n + v] = m;  // word-major: lanes over vehicles read consecutive words
    }
  }
  // alignment sums, ascending members: a lane adds a member's terms only if
  // the member is in its neighbourhood (exec narrowed to those lanes around
  // the four adds, masked_add4: no selects), starting from -0.0, the exact
  // identity of IEEE addition (-0 + x == x for every x, signed zeros
  // included), which gives the bits of "first term, then acc + term". Lane =
  // vehicle v; the four chains of a pass (x and y of p, of q) are independent.
  double galign = 1.0;
  for (int v = tid; v < n; v += kWABlock) {
    const int i = Pin[v];
    unsigned long long rowb[kWMaxW];
    int k = 0;
#pragma unroll
    for (int w = 0; w < kWMaxW; ++w) {
      unsigned long long bits = w < NW ? adjF[i * NW + w] : 0ull;
      if (w == (i >> 6)) bits |= 1ull << (i & 63);
      if (w == NW - 1 && (n & 63)) bits &= (1ull << (n & 63)) - 1ull;
      rowb[w] = bits;
      k += __popcll(bits);
    }
    double s0 = -0.0, s1 = -0.0, s2 = -0.0, s3 = -0.0;
#pragma unroll
    for (int w = 0; w < kWMaxW; ++w) {
      if (w >= NW) break;
      for (int hf = 0; hf < 2; ++hf) {
        const unsigned h = (unsigned)(rowb[w] >> (32 * hf));
#pragma unroll 4
        for (int jb = 0; jb < 32; ++jb) {
          int j = 64 * w + 32 * hf + jb;
          j = j < n ? j : 0;
          const double px = p[3 * j], py = p[3 * j + 1], qx = qf[3 * j], qy = qf[3 * j + 1];
          masked_add4(__ballot((h >> jb) & 1u), s0, s1, s2, s3, px, py, qx, qy);
        }
      }
    }
    const double oon = 1.0 / (double)k;
    const double sm[2] = {s0 * oon, s1 * oon};
    const double dm[2] = {s2 * oon, s3 * oon};
    const bool lazy = (k + 4) < 20;
    // lazy: the first product is the sum's first term (start from -0.0, the
    // exact additive identity); otherwise the sum starts at +0.0 (0 + the
    // first product); a non-neighbour adds -0.0 (no change, bit for bit).
    // c = 2 di + sj: (q_di - dm_di) (p_sj - sm_sj)
    const double z0 = lazy ? -0.0 : 0.0;
    double c0 = z0, c1 = z0, c2 = z0, c3 = z0;
    // lazy lanes scale the q deviations by 1/k; 1.0 * x == x bit for bit, so
    // the others multiply by 1.0, and a wave without a lazy lane (every one
    // at C4's k ~ 500) skips the products (no per-lane selects either way)
    const double scale = lazy ? oon : 1.0;
    auto pass2 = [&](auto scaled) {
#pragma unroll
      for (int w = 0; w < kWMaxW; ++w) {
        if (w >= NW) break;
        for (int hf = 0; hf < 2; ++hf) {
          const unsigned h = (unsigned)(rowb[w] >> (32 * hf));
#pragma unroll 4
          for (int jb = 0; jb < 32; ++jb) {
            int j = 64 * w + 32 * hf + jb;
            j = j < n ? j : 0;
            const double e0 = p[3 * j] - sm[0], e1 = p[3 * j + 1] - sm[1];
            double d0 = qf[3 * j] - dm[0], d1 = qf[3 * j + 1] - dm[1];
            if (decltype(scaled)::value) {
              d0 = scale * d0;
              d1 = scale * d1;
            }
            masked_add4(__ballot((h >> jb) & 1u), c0, c1, c2, c3, d0 * e0, d0 * e1, d1 * e0,
                        d1 * e1);
          }
        }
      }
    };
    if (__any(lazy)) pass2(std::true_type{});
    else pass2(std::false_type{});
    if (!lazy) {
      c0 = c0 * oon; c1 = c1 * oon; c2 = c2 * oon; c3 = c3 * oon;
    }
    const double S[4] = {c0, c2, c1, c3};
    double R[4], t[2], ga;
    umeyama_finish(S, sm, dm, R, t, &ga);
    galign = ga < galign ? ga : galign;
    double* o = out + 6 * v;
    o[0] = R[0]; o[1] = R[1]; o[2] = R[2]; o[3] = R[3]; o[4] = t[0]; o[5] = t[1];
  }
  // the swarm's smallest alignment gap and the flags
  if (tid == 0) *gw = (unsigned long long)__double_as_longlong(1.0);
  __syncthreads();
  block_min_gap(gw, galign);
  __syncthreads();
  if (tid == 0) {
    *reinterpret_cast<unsigned long long*>(wsa + WW.gal) = *gw;
    *wflags = misc[M_PINF] ? 2u : 0u;
  }
}

// FUSE: the control phase of a swarm whose vehicles all adopted one
// assignment runs in this workgroup after its adoption (wide_control);
// GM: it also reports the gate margin.
// ACL_WIDE_KARG (default 1): the kernel reads its parameters through a
// pointer to the kernarg segment, laundered so the compiler reloads a field
// by a scalar load where it is used instead of holding every pointer and
// layout offset in SGPRs for the whole kernel (it spilled ~130 of them to
// VGPR lanes and read them back inside the CBAA rounds).
#ifndef ACL_WIDE_KARG
#define ACL_WIDE_KARG 1
#endif
typedef const __attribute__((address_space(4))) SolveParams KSolveParams;

// MG false (acl_solve_args_t::skip_margin): no decision margin -- the level
// walk stops once every vehicle has its winning level (the runner-up levels
// only bound the margin), the selects and scans track nothing
template <bool FUSE, bool GM, bool MG>
__global__ void __launch_bounds__(kWBlock, 4) solve_wide_kernel(const SolveParams P_) {
#if ACL_WIDE_KARG
  KSolveParams* Pk = (KSolveParams*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(Pk));
  KSolveParams& P = *Pk;
#else
  const SolveParams& P = P_;
#endif
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const int NW = (n + 63) >> 6;
  const WLayout L = make_wlayout(n);
  const int b = P.b0 + blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;

  double* p = reinterpret_cast<double*>(smem + L.p);
  double* qv = reinterpret_cast<double*>(smem + L.qv);
  unsigned long long* vadj = reinterpret_cast<unsigned long long*>(smem + L.vadj);
  uint16_t* Pin = reinterpret_cast<uint16_t*>(smem + L.Pin);
  uint16_t* Ptin = reinterpret_cast<uint16_t*>(smem + L.Ptin);
  uint16_t* ccw = reinterpret_cast<uint16_t*>(smem + L.ccw);
  float* ccp = reinterpret_cast<float*>(smem + L.ccp);
  uint16_t* cuw = reinterpret_cast<uint16_t*>(smem + L.cuw);
  unsigned char* validv = smem + L.valid;
  unsigned long long* dmask = reinterpret_cast<unsigned long long*>(smem + L.masks);
  unsigned long long* obm = dmask + 2 * NW;
  // unif bit j: column j holds one `who` for every vehicle (as of its last
  // update; a bid written into it clears the bit and dirties the column), so
  // at the fixed point all tables agree <=> every bit is set
  unsigned long long* unif = dmask + 4 * NW;
  unsigned long long* spm = dmask + 5 * NW;  // sparse columns (see the header)
  unsigned long long* seen = reinterpret_cast<unsigned long long*>(smem + L.seen);
  int* misc = reinterpret_cast<int*>(smem + L.misc);
  unsigned char* ecnt = smem + L.ecnt;
  unsigned* elist = reinterpret_cast<unsigned*>(smem + L.elist);
  unsigned* bids = reinterpret_cast<unsigned*>(smem + L.bids);  // [2][n]
  unsigned* xcnt = reinterpret_cast<unsigned*>(smem + L.xcnt);

  unsigned char* wsb = P.ws + P.W.wide + (size_t)b * P.W.wide_stride;
  uint16_t* T = reinterpret_cast<uint16_t*>(wsb);
  const WsWide WW = ws_wide(n);
  const unsigned char* wsa = P.ws + P.W.align + (size_t)b * P.W.align_stride;
  const double* out = reinterpret_cast<const double*>(wsa + WW.out);  // global, L2-resident
  const unsigned wflags = *reinterpret_cast<const unsigned*>(wsa + WW.flags);

  const int f_in = P.fidx[b];
  const int f = (f_in < 0 || f_in >= P.F) ? 0 : f_in;
  MarginPair mp;
  margin_init(mp);
  wstamp(P, b, 0);
  wstamp(P, b, kStampRt0);

  // ---------------- phase 0: load (align_wide_kernel's results) -------------
  if (wflags & 1u) {
    // P_in is not a permutation (or fidx is out of range): nothing is solved
    for (int v = tid; v < n; v += kWBlock) {
      P.P_out[(size_t)b * n + v] = P.P_in[(size_t)b * n + v];
      if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 0;
    }
    for (int k = tid; k < 3 * n; k += kWBlock) {
      if (P.u) P.u[(size_t)b * n * 3 + k] = 0.0;
      if (P.u_safe) P.u_safe[(size_t)b * n * 3 + k] = 0.0;
    }
    if (P.who)
      for (int k = tid; k < n * n; k += kWBlock) P.who[(size_t)b * n * n + k] = 0xFFFF;
    if (P.gate_margin && tid == 0) P.gate_margin[b] = __builtin_inf();
    if (tid == 0) {
      acl_swarm_status_t st = {};
      st.flags = ACL_SWARM_BAD_INPUT;
      st.rounds = (uint16_t)(2 * n);
      st.margin = 1.0f;
      P.status[b] = st;
    }
    return;
  }
  {
    const double* gp = P.p + (size_t)f * n * 3;
    const double* gq = P.q + (size_t)b * n * 3;
    for (int k = tid; k < 3 * n; k += kWBlock) {
      p[k] = gp[k];
      qv[k] = gq[k];
    }
    const unsigned long long* gv = reinterpret_cast<const unsigned long long*>(wsa + WW.vadj);
    for (int k = tid; k < NW * n; k += kWBlock) vadj[k] = gv[k];
    for (int v = tid; v < n; v += kWBlock) {
      const unsigned pv = P.P_in[(size_t)b * n + v];  // a permutation (checked)
      Pin[v] = (uint16_t)pv;
      Ptin[pv] = (uint16_t)v;
    }
    for (int k = tid; k < 4 * NW; k += kWBlock) dmask[k] = 0ull;
    // every column all `none`: sparse, base `none`, no exceptions (T is not
    // reset: no column reads it before an update writes it in full)
    for (int k = tid; k < NW; k += kWBlock) unif[k] = spm[k] = ~0ull;
    for (int k = tid; k < n; k += kWBlock) {
      ccw[k] = cuw[k] = (uint16_t)n;
      ecnt[k] = 0;
      xcnt[k] = 0;
    }
    if (tid < 32) misc[tid] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    misc[M_AGREE] = 1;
    if (wflags & 2u) misc[M_PINF] = 1;
    // the margin word starts at the smallest alignment gap
    *reinterpret_cast<unsigned long long*>(misc + M_MARG) =
        *reinterpret_cast<const unsigned long long*>(wsa + WW.gal);
  }
  wstamp(P, b, 1);
  wstamp(P, b, 2);
  if (P.align_Rt)
    for (int k = tid; k < 6 * n; k += kWBlock) P.align_Rt[(size_t)b * n * 6 + k] = out[k];
  __syncthreads();

  // ---------------- phase 2: prices -----------------------------------------
  // Not stored (see the header): the NaN-price test. A price is NaN only if
  // its squared distance is (acl_price is finite on [0, inf]); with every
  // coordinate, rotation and translation entry finite and below 1e100 in
  // magnitude no product overflows, so no distance is NaN. Otherwise every
  // price is evaluated once.
  const WPrice price{out, qv, p, misc[M_PINF] == 0};
  {
    bool big = false;
    for (int k = tid; k < 6 * n; k += kWBlock) big |= !(fabs(out[k]) < 1e100);
    for (int k = tid; k < 3 * n; k += kWBlock) big |= !(fabs(p[k]) < 1e100) || !(fabs(qv[k]) < 1e100);
    if (__any(big) && lane == 0) misc[W_BIG] = 1;
    __syncthreads();
    if (misc[W_BIG]) {
      int nonfin = 0;
      for (int e = tid; e < n * n; e += kWBlock) {
        const float c = price(e / n, e % n);
        nonfin |= c != c;
      }
      if (__any(nonfin) && lane == 0) misc[M_NONFIN] = 1;
    }
  }
  __syncthreads();
  const bool nonfinite = misc[M_NONFIN] != 0;
  const WTable tab{T, cuw, ecnt, elist, spm, xcnt, n};
  wstamp(P, b, 3);

  // ---------------- phase 3: CBAA ------------------------------------------
  // a bid: into T for a dense column, else into the bid list of this
  // select phase's parity (the column's next update applies it)
  auto place_bid = [&](int v, int task, int bpar) {
    if (tab.sparse(task)) {
      const int k = atomicAdd(&misc[W_NBID + bpar], 1);
      bids[bpar * n + k] = ((unsigned)v << 16) | (unsigned)task;
    } else {
      T[tix(n, task, v)] = (uint16_t)v;
    }
    atomicOr(&dmask[(bpar ^ 1) * NW + (task >> 6)], 1ull << (task & 63));
    atomicAnd(&unif[task >> 6], ~(1ull << (task & 63)));
  };
  for (int v = wave; v < n; v += kWWaves) {
    const int task = wide_select<MG>(n, NW, v, lane, price, T, ccw, ccp, tab, true, mp);
    if (task >= 0 && lane == 0) place_bid(v, task, 0);  // round 1 (parity 1) reads list 0
  }
  __syncthreads();
  int eff = 0;
#if ACL_WIDE_PROF
  unsigned long long pf_col = 0, pf_scan = 0, pf_sel = 0, pf_bar = 0, pf_cnt = 0, pf_rounds = 0;
  unsigned long long pf_cload = 0, pf_clvl = 0, pf_cwb = 0;
  unsigned long long pf_sparse = 0;  // sparse-column updates | dense ones << 21 | sparse->dense << 42
#endif
  unsigned obf = 0u;  // per-lane outbid bits (bit c: vehicle lane + 64 c), one round
  const int max_rounds = 2 * n;
  int lastpar = 0;  // the parity of the last select phase's bid list
  for (int r = 1; r <= max_rounds; ++r) {
    const int par = r & 1, npar = par ^ 1;
    lastpar = par;
    // the round's dirty columns, a ticket at a time: a wave takes the next
    // one when it finishes its last (column updates differ in cost; the
    // updates of one round touch disjoint columns, so the order is free)
    int ncol = 0;
    for (int w = 0; w < NW; ++w) ncol += __popcll(dmask[par * NW + w]);
    for (;;) {
      const int tk = wave_ticket(misc, W_TCOL, lane);
      if (tk >= ncol) break;
      {
        const int j = kth_bit(dmask + par * NW, NW, tk);
        WPROF_T(pc0);
        WPROF_ADD(pf_cnt, 1ull);
        // column j of the tiled table: vehicle u = lane + 64 c at Tj[tlo + 512 c]
        uint16_t* Tj = T + (((size_t)(j >> 3) * ((n + 7) >> 3)) << 6) + ((j & 7) << 3);
        const int tlo = ((lane >> 3) << 6) + (lane & 7);
        unsigned wu[kWMaxW], key[kWMaxW], nw[kWMaxW], k1[kWMaxW], k2[kWMaxW];
        // per vehicle (bit c of a per-lane VGPR word, not an SGPR lane mask
        // per c: eight of each would not fit the scalar file): s1m -- a
        // winner level found (k1), s2m -- done (k2 = the next level its
        // neighbourhood holds, 0 = none; also the lanes past n), needm --
        // exact ordered scan (ties, NaN, levels exhausted)
        unsigned s1m = 0u, s2m = 0u, needm = 0u;
        // the column's entries: a sparse column from its base, exceptions
        // and the last select phase's bids on it (LDS); a dense one from T
        const bool spj = tab.sparse(j);  // wave-uniform
        const unsigned base = spj ? (unsigned)cuw[j] : 0u;
#pragma unroll
        for (int c = 0; c < kWMaxW; ++c) {
          const int u = lane + 64 * c;
          const bool ok = c < NW && u < n;
          wu[c] = ok ? (spj ? base : (unsigned)Tj[tlo + (c << 9)]) : (unsigned)n;
          key[c] = ok ? 1u : 0u;  // + the holder's price bits below (1: none)
          nw[c] = (unsigned)n;
          k1[c] = k2[c] = 0u;
          s2m |= (ok ? 0u : 1u) << c;
        }
        if (spj) {
          // vehicle u's entry is `who` (u wave-uniform, in a scalar register:
          // the chunk is chosen by a scalar branch, one select per entry)
          auto set_entry = [&](unsigned u, unsigned who) {
            const int cu = (int)(u >> 6);
            const bool me = lane == (int)(u & 63u);
            switch (cu) {
#define ACL_SET_CHUNK(c_) \
  case c_:                \
    if (c_ < kWMaxW) wu[c_ < kWMaxW ? c_ : 0] = me ? who : wu[c_ < kWMaxW ? c_ : 0]; \
    break;
              ACL_SET_CHUNK(0) ACL_SET_CHUNK(1) ACL_SET_CHUNK(2) ACL_SET_CHUNK(3)
              ACL_SET_CHUNK(4) ACL_SET_CHUNK(5) ACL_SET_CHUNK(6) ACL_SET_CHUNK(7)
#undef ACL_SET_CHUNK
              default: break;
            }
          };
          static_assert(kWMaxW <= 8, "set_entry covers 8 chunks");
          const int ne = ecnt[j];
          for (int k = 0; k < ne; ++k) {
            const unsigned e =
                (unsigned)__builtin_amdgcn_readfirstlane((int)elist[j * kWSparseK + k]);
            set_entry(e >> 16, e & 0xFFFFu);
          }
          // (the list is rewritten below: its vehicles' counts drop here)
          if (lane < ne) atomicSub(&xcnt[elist[j * kWSparseK + lane] >> 16], 1u);
          const int nb = misc[W_NBID + npar];
          const unsigned* bl = bids + npar * n;
          for (int k0 = 0; k0 < nb; k0 += 64) {
            const unsigned e = k0 + lane < nb ? bl[k0 + lane] : 0xFFFFFFFFu;
            unsigned long long m = __ballot((e & 0xFFFFu) == (unsigned)j);
            while (m) {
              const int k = __ffsll((long long)m) - 1;
              m &= m - 1;
              const unsigned v = (unsigned)__builtin_amdgcn_readlane((int)e, k) >> 16;
              set_entry(v, v);  // the bid: v holds its own bid
            }
          }
        }
        {
          // entries of one holder share its price: one (lane-uniform) price
          // per distinct holder, the first few holders; any further ones per
          // entry
          unsigned pendm = 0u;
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c) pendm |= (wu[c] < (unsigned)n ? 1u : 0u) << c;
          for (int it = 0; it < 4; ++it) {
            int lw = -1;
#pragma unroll
            for (int c = 0; c < kWMaxW; ++c) {
              const unsigned long long bl = __ballot((pendm >> c) & 1u);
              if (lw < 0 && bl) lw = __builtin_amdgcn_readlane((int)wu[c], __ffsll((long long)bl) - 1);
            }
            if (lw < 0) break;
            const unsigned kk = __float_as_uint(price(lw, j)) + 1u;
#pragma unroll
            for (int c = 0; c < kWMaxW; ++c)
              if (((pendm >> c) & 1u) && wu[c] == (unsigned)lw) {
                key[c] = kk;
                pendm &= ~(1u << c);
              }
          }
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c)
            if ((pendm >> c) & 1u) key[c] = __float_as_uint(price((int)wu[c], j)) + 1u;
        }
        WPROF_T(pk);
        WPROF_ADD(pf_cload, pk - pc0);
        unsigned cap = 0xFFFFFFFFu;
        bool exhausted = false;
        int wk0 = -1;  // the top level's holder and key (the column price cache)
        unsigned Mk0 = 0u;
        for (int k = 0; k < kWLevels + 1; ++k) {
          unsigned lm = 0u;
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c) {
            const unsigned x = key[c] < cap ? key[c] : 0u;
            lm = lm > x ? lm : x;
          }
          const unsigned Mk = wave_max_u32(lm);
          if (Mk == 0u) {
            exhausted = true;
            break;
          }
          unsigned long long h[kWMaxW];
          int wk = -1;
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c) {
            h[c] = __ballot(key[c] == Mk);
            if (wk < 0 && h[c]) wk = __builtin_amdgcn_readlane((int)wu[c], __ffsll((long long)h[c]) - 1);
          }
          bool tl = false;
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c) tl |= key[c] == Mk && wu[c] != (unsigned)wk;
          const bool tk = nonfinite || __ballot(tl) != 0ull;
          // hit: the vehicle's closed neighbourhood holds a vehicle of this
          // level; holder-word outer loop, so the vehicle words' LDS loads
          // issue together, stopping once every active vehicle is hit
          // (MG false: done at the winner; s2m then only marks the lanes past n)
          const unsigned actm = ~((MG ? s2m : (s1m | s2m)) | needm) & ((1u << kWMaxW) - 1u);
          unsigned hitm = 0u;
#pragma unroll
          for (int w2 = 0; w2 < kWMaxW; ++w2) {
            if (!h[w2]) continue;
            if (__ballot((actm & ~hitm) != 0u) == 0ull) break;
#pragma unroll
            for (int c = 0; c < kWMaxW; ++c)
              if (((actm & ~hitm) >> c) & 1u)
                hitm |= ((vadj[w2 * n + lane + 64 * c] & h[w2]) != 0ull ? 1u : 0u) << c;
          }
          if (k == 0 && wk >= 0 && wk < n) {
            wk0 = wk;
            Mk0 = Mk;
          }
          const unsigned took = actm & hitm;   // st 0 -> 1 or 1 -> 2
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c) {
            if ((took >> c) & 1u) {
              if (!((s1m >> c) & 1u)) {
                nw[c] = (unsigned)wk;
                k1[c] = Mk;
              } else {
                k2[c] = Mk;
              }
            }
          }
          const unsigned first = took & ~s1m, second = took & s1m;
          s1m |= first;
          s2m |= second;
          if (tk) needm |= first;
          const bool open = (~((MG ? s2m : (s1m | s2m)) | needm) & ((1u << kWMaxW) - 1u)) != 0u;
          if (__ballot(open) == 0ull) break;
          cap = Mk;
        }
        WPROF_T(pl);
        WPROF_ADD(pf_clvl, pl - pk);
        // undecided, or the runner-up level not found before the level cap
        needm |= ~(s1m | s2m) & ((1u << kWMaxW) - 1u);
        if (MG && !exhausted) needm |= s1m & ~s2m;
        if (MG) {
          const unsigned donem = s2m & ~needm;
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c)
            if (((donem >> c) & 1u) && k2[c] != 0u)
              margin_track(mp, __uint_as_float(k1[c] - 1u), __uint_as_float(k2[c] - 1u));
        }
        WPROF_T(ps0);
        bool tvalid = !spj;  // T holds the column's entries (before this update)
        if (__ballot(needm != 0u) != 0ull) {
          WPROF_ADD(pf_cnt, 1ull << 21);
          if (!tvalid) {  // (rare) the exact scan reads T: write the column in full
#pragma unroll
            for (int c = 0; c < kWMaxW; ++c)
              if (c < NW && lane + 64 * c < n) Tj[tlo + (c << 9)] = (uint16_t)wu[c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            tvalid = true;
          }
          // exact ordered scan (ascending vehid, strict >): ties, NaN prices,
          // vehicles no tracked level decides; the runner-up is the best
          // price of another `who` (entries of one `who` share its price)
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c) {
            if ((needm >> c) & 1u) {
              const int u = lane + 64 * c;
              float bp = 0.0f, p2 = 0.0f;
              unsigned bw = (unsigned)n;
              bool first = true, have2 = false;
              for (int w2 = 0; w2 < NW; ++w2) {
                unsigned long long mm = vadj[w2 * n + u];
                while (mm) {
                  const int uu = 64 * w2 + __ffsll((long long)mm) - 1;
                  mm &= mm - 1;
                  const unsigned wx = T[tix(n, j, uu)];
                  const float px = wx < (unsigned)n ? price((int)wx, j) : 0.0f;
                  if (first) {
                    bp = px; bw = wx; first = false;
                  } else if (px > bp) {
                    p2 = bp; have2 = true;  // the old winner's `who` differs
                    bp = px; bw = wx;
                  } else if (wx != bw) {
                    if (!have2 || px > p2) p2 = px;
                    have2 = true;
                  }
                }
              }
              nw[c] = bw;
              if (MG && have2) margin_track(mp, bp, p2);
            }
          }
        }
        WPROF_T(ps1);
        WPROF_ADD(pf_scan, ps1 - ps0);
        __builtin_amdgcn_wave_barrier();
        bool ch = false, mx = false;
        const unsigned nw0 = (unsigned)__builtin_amdgcn_readfirstlane((int)nw[0]);  // vehicle 0
        // the new state: sparse around the top level's `who` (the entry most
        // vehicles take) when at most kWSparseK vehicles hold another, else
        // dense in T (all entries written if T was stale, else the changed ones)
        unsigned nbase = (wk0 < 0 || wk0 >= n) ? nw0 : (unsigned)wk0;
        unsigned long long em[kWMaxW];
        int nexc = 0;
#pragma unroll
        for (int c = 0; c < kWMaxW; ++c) {
          const bool ok = c < NW && lane + 64 * c < n;
          em[c] = __ballot(ok && nw[c] != nbase);
          nexc += __popcll(em[c]);
        }
        if (nexc == n && nbase != nw0) {
          // (rare: no vehicle holds the top level's `who`, a tie) around
          // vehicle 0's entry instead
          nbase = nw0;
          nexc = 0;
#pragma unroll
          for (int c = 0; c < kWMaxW; ++c) {
            const bool ok = c < NW && lane + 64 * c < n;
            em[c] = __ballot(ok && nw[c] != nbase);
            nexc += __popcll(em[c]);
          }
        }
        // every vehicle holds one `who` <=> no exception around nbase (when
        // some vehicle holds nbase; else it is vehicle 0's entry, above)
        const bool uniformj = nexc == 0;
        const bool nsparse = nexc <= kWSparseK;
        WPROF_ADD(pf_sparse, spj ? 1ull : (1ull << 21));
        WPROF_ADD(pf_sparse, (spj && !nsparse) ? (1ull << 42) : 0ull);
        int erank = 0;
#pragma unroll
        for (int c = 0; c < kWMaxW; ++c) {
          const int u = lane + 64 * c;
          const bool ok = c < NW && u < n;
          if (nsparse) {
            if ((em[c] >> lane) & 1ull) {
              const int k = erank + (int)__builtin_amdgcn_mbcnt_hi(
                                        (unsigned)(em[c] >> 32),
                                        __builtin_amdgcn_mbcnt_lo((unsigned)em[c], 0u));
              elist[j * kWSparseK + k] = ((unsigned)u << 16) | nw[c];
              atomicAdd(&xcnt[u], 1u);
            }
            erank += __popcll(em[c]);
          } else if (ok && (!tvalid || nw[c] != wu[c])) {
            Tj[tlo + (c << 9)] = (uint16_t)nw[c];
          }
          // outbid (:502): a per-lane bit, published once per wave and round
          obf |= (vflag(ok) & vflag(wu[c] == (unsigned)u) & vflag(nw[c] != (unsigned)u)) << c;
          ch |= nw[c] != wu[c];
        }
        mx = !uniformj;
        if (lane == 0) {
          if (nsparse) {
            cuw[j] = (uint16_t)nbase;
            ecnt[j] = (unsigned char)nexc;
            if (!spj) atomicOr(&spm[j >> 6], 1ull << (j & 63));
          } else if (spj) {
            atomicAnd(&spm[j >> 6], ~(1ull << (j & 63)));
          }
        }
        // a column left holding one `who` everywhere is a fixed point with no
        // runner-up: not dirty next round unless a re-select writes it (as in
        // auction.hip); the change still counts for eff_rounds
        if (wk0 >= 0 && lane == 0) {
          ccw[j] = (uint16_t)wk0;
          ccp[j] = __uint_as_float(Mk0 - 1u);
        }
        const bool anych = __ballot(ch) != 0ull, anymx = __ballot(mx) != 0ull;
        if (anych && lane == 0) {
          misc[W_RCH + par] = 1;
          if (anymx || nonfinite) atomicOr(&dmask[npar * NW + (j >> 6)], 1ull << (j & 63));
        }
        if (lane == 0) {  // (a column without exceptions: cuw[j] = nw0, set above)
          if (anymx) atomicAnd(&unif[j >> 6], ~(1ull << (j & 63)));
          else atomicOr(&unif[j >> 6], 1ull << (j & 63));
        }
        WPROF_T(pc1);
        WPROF_ADD(pf_col, pc1 - pc0 - (ps1 - ps0));
        WPROF_ADD(pf_cwb, pc1 - ps1);
      }
    }
#pragma unroll
    for (int c = 0; c < kWMaxW; ++c) {
      const unsigned long long ob = __ballot((obf >> c) & 1u);
      if (ob && lane == 0) atomicOr(&obm[par * NW + c], ob);
    }
    obf = 0u;
    WPROF_T(pb0);
    __syncthreads();
    WPROF_T(pb1);
    WPROF_ADD(pf_bar, pb1 - pb0);
    WPROF_ADD(pf_rounds, 1ull);
    if (tid < NW) {
      dmask[par * NW + tid] = 0ull;
      obm[npar * NW + tid] = 0ull;
    }
    if (tid == 0) {
      misc[W_RCH + npar] = 0;  // round r+1's change flag (round r-1's was read)
      misc[W_TCOL] = 0;        // every wave has left this round's column loop
      misc[W_NBID + npar] = 0; // the bid list this round's updates read: round r+1's selects refill it
    }
    {
      // outbid vehicles, a ticket at a time (a re-select writes only its own
      // row's entry: any order)
      int nsel = 0;
      for (int w = 0; w < NW; ++w) nsel += __popcll(obm[par * NW + w]);
      for (;;) {
        const int tk = wave_ticket(misc, W_TSEL, lane);
        if (tk >= nsel) break;
        {
          const int v = kth_bit(obm + par * NW, NW, tk);
          WPROF_T(pr0);
          WPROF_ADD(pf_cnt, 1ull << 42);
          const int task = wide_select<MG>(n, NW, v, lane, price, T, ccw, ccp, tab, false, mp);
          if (task >= 0 && lane == 0) place_bid(v, task, par);
          WPROF_T(pr1);
          WPROF_ADD(pf_sel, pr1 - pr0);
        }
      }
    }
    WPROF_T(pb2);
    __syncthreads();
    WPROF_T(pb3);
    WPROF_ADD(pf_bar, pb3 - pb2);
    if (tid == 0) misc[W_TSEL] = 0;  // every wave has left this round's re-selects
    bool next = false;
    for (int w = 0; w < NW; ++w) next |= dmask[npar * NW + w] != 0ull;
    if (next || misc[W_RCH + par]) eff = r;
    // no dirty column and no re-select: round r+1 changes nothing (the
    // fixed point every later round repeats); early_exit = 0 iterates the
    // remaining (empty) rounds, the reference's literal schedule
    if (!next && P.early_exit) break;
  }
#if ACL_WIDE_PROF
  if (P.stamps && lane == 0) {
    unsigned long long* ps =
        reinterpret_cast<unsigned long long*>(P.stamps) + (size_t)b * kStampStride + kStampSec;
    atomicAdd(ps + 0, pf_col);
    atomicAdd(ps + 1, pf_scan);
    atomicAdd(ps + 2, pf_sel);
    atomicAdd(ps + 3, pf_bar);
    atomicAdd(ps + 4, pf_cnt);
    if (wave == 0) ps[5] = pf_rounds;
    atomicAdd(ps + 6, pf_cload);
    atomicAdd(ps + 7, pf_clvl);
    atomicAdd(ps + 8, pf_cwb);
    atomicAdd(ps + 9, pf_sparse);
  }
#endif

  // Bids of the last select phase that no column update applied (the rounds
  // ran to the 2n limit with re-selects in the last one): fold them into
  // their columns -- an exception entry while there is room, else the
  // column is written to T in full (dense). One wave, bid by bid.
  if (wave == 0) {
    const int nb = misc[W_NBID + lastpar];
    const unsigned* bl = bids + lastpar * n;
    for (int k = 0; k < nb; ++k) {
      const unsigned e = bl[k];
      const int v = (int)(e >> 16), task = (int)(e & 0xFFFFu);
      if (!tab.sparse(task)) {
        if (lane == 0) T[tix(n, task, v)] = (uint16_t)v;  // (dense bids went to T already)
        continue;
      }
      const int ne = ecnt[task];
      int slot = -1;
      for (int q = 0; q < ne; ++q)
        if ((elist[task * kWSparseK + q] >> 16) == (unsigned)v) slot = q;
      if (slot < 0 && ne < kWSparseK) slot = ne;
      if (slot >= 0) {
        if (lane == 0) {
          elist[task * kWSparseK + slot] = ((unsigned)v << 16) | (unsigned)v;
          if (slot == ne) ecnt[task] = (unsigned char)(ne + 1);
        }
      } else {
        for (int u = lane; u < n; u += 64)
          T[tix(n, task, u)] = (uint16_t)(u == v ? (unsigned)v : tab.sparse_entry(task, u));
        if (lane == 0) atomicAnd(&spm[task >> 6], ~(1ull << (task & 63)));
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  }
  __syncthreads();
  wstamp(P, b, 4);
  // swarm margin: min over every thread's CBAA pair (the alignment gaps are
  // in the word already)
  if (MG) block_min_gap(reinterpret_cast<unsigned long long*>(misc + M_MARG), margin_gap(mp));

  // ---------------- phase 4: adoption --------------------------------------
  // Do all vehicles hold vehicle 0's table? T is column-major, so compare
  // each column with its row-0 entry (coalesced). Then one table decides
  // every vehicle's validity (isValidAssignment of row 0, as auction.hip).
  // Do all vehicles hold vehicle 0's table? <=> every column is uniform
  // (the unif bits; no pass over the n^2 table)
  if (tid == 0) {
    bool agree = true;
    for (int w = 0; w < NW; ++w) {
      const unsigned long long need =
          (w == NW - 1 && (n & 63)) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
      agree &= (unif[w] & need) == need;
    }
    if (!agree) misc[M_AGREE] = 0;
  }
  __syncthreads();
  const bool allagree = misc[M_AGREE] != 0;
  if (allagree) {
    // row 0 = column entries T[j][0]: a permutation <=> every entry < n and
    // each vehicle holds exactly one task
    unsigned long long* sw = seen;  // [NW] words
    if (tid < NW) sw[tid] = 0ull;
    __syncthreads();
    for (int j = tid; j < n; j += kWBlock) {
      const int w = cuw[j];  // every column uniform: its one `who`
      if (w >= n) misc[M_NINV] = n;
      else atomicOr(&sw[w >> 6], 1ull << (w & 63));
    }
    __syncthreads();
    if (tid == 0) {
      int cnt = 0;
      for (int w = 0; w < NW; ++w) cnt += __popcll(sw[w]);
      if (cnt != n) misc[M_NINV] = n;
    }
    __syncthreads();
    const bool valid0 = misc[M_NINV] == 0;
    for (int j = tid; j < n; j += kWBlock) {
      const int v = valid0 ? (int)cuw[j] : Ptin[j];
      validv[v] = valid0;
      if (j != Pin[v]) misc[M_CHANGED] = 1;
      P.P_out[(size_t)b * n + v] = (uint16_t)j;
    }
  }
  for (int v = wave; !allagree && v < n; v += kWWaves) {
    unsigned long long* sw = seen + wave * NW;
    if (lane < NW) sw[lane] = 0ull;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    bool bad = false, diff = false;
    int mine = -1;
    for (int c = 0; c < NW; ++c) {
      const int jj = lane + 64 * c;
      bool ismine = false;
      if (jj < n) {
        const int w = (int)tab(jj, v);
        if (w >= n) bad = true;
        else atomicOr(&sw[w >> 6], 1ull << (w & 63));
        diff |= w != (int)tab(jj, 0);
        ismine = w == v;
      }
      const unsigned long long mm = __ballot(ismine);
      if (mine < 0 && mm) mine = 64 * c + __ffsll((long long)mm) - 1;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    int cnt = 0;
    for (int w = 0; w < NW; ++w) cnt += __popcll(sw[w]);
    const bool valid = !__any(bad) && cnt == n && mine >= 0;
    const bool agree = !__any(diff);
    const int adopted = valid ? mine : Pin[v];
    if (lane == 0) {
      validv[v] = valid;
      if (!valid) atomicAdd(&misc[M_NINV], 1);
      if (!agree) misc[M_AGREE] = 0;
      if (adopted != Pin[v]) misc[M_CHANGED] = 1;
      P.P_out[(size_t)b * n + v] = (uint16_t)adopted;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  if (P.who) {
    for (int k = tid; k < n * n; k += kWBlock) {
      const int v = k / n, jj = k - v * n;
      const int w = (int)tab(jj, v);
      P.who[(size_t)b * n * n + k] = (w >= n) ? (uint16_t)0xFFFF : (uint16_t)w;
    }
  }
  __syncthreads();
  wstamp(P, b, 5);
  {
    const bool allvalid = misc[M_NINV] == 0;
    // (own rows: a vehicle without a valid table keeps its own row)
    const bool rowsm = P.P_rows != nullptr && P.P_rows_on[b] != 0;
    const bool uniform = (allvalid && misc[M_AGREE]) || (misc[M_NINV] == n && !rowsm);
    uint16_t* wsPt = reinterpret_cast<uint16_t*>(P.ws + P.W.pt) + (size_t)b * n;
    if (tid == 0) P.ws[P.W.mode + b] = uniform ? 0 : 1;
    if (uniform) {
      for (int jj = tid; jj < n; jj += kWBlock) wsPt[jj] = allvalid ? (uint16_t)tab(jj, 0) : Ptin[jj];
    } else {
      uint16_t* rows = reinterpret_cast<uint16_t*>(P.ws + P.W.rows) + (size_t)b * n * n;
      for (int k = tid; k < n * n; k += kWBlock) {
        const int v = k / n, jj = k - v * n;
        rows[k] = validv[v] ? (uint16_t)tab(jj, v)
                  : rowsm ? P.P_rows[(size_t)b * n * n + k] : Ptin[jj];
      }
      for (int v = tid; v < n; v += kWBlock) P.ws[P.W.vvalid + (size_t)b * n + v] = validv[v];
    }
  }
  const bool uniform_all = (misc[M_NINV] == 0 && misc[M_AGREE]) || misc[M_NINV] == n;
  if (tid == 0) {
    acl_swarm_status_t st = {};
    uint32_t fl = 0;
    if (misc[M_NINV] == 0) fl |= ACL_SWARM_VALID;
    if (misc[M_AGREE]) fl |= ACL_SWARM_AGREE;
    if (misc[M_CHANGED]) fl |= ACL_SWARM_CHANGED;
    if (nonfinite) fl |= ACL_SWARM_NONFINITE;
    // (MG false: skip_margin -- not tracked, -1)
    const double g = !MG ? -1.0 : nonfinite ? 0.0
        : __longlong_as_double((long long)*reinterpret_cast<unsigned long long*>(misc + M_MARG));
    if (MG && g < ACL_FRAGILE_MARGIN) fl |= ACL_SWARM_FRAGILE;
    st.flags = fl;
    st.eff_rounds = (uint16_t)eff;
    st.rounds = (uint16_t)(2 * n);
    st.n_invalid = (uint16_t)misc[M_NINV];
    st.margin = (float)g;
    P.status[b] = st;
  }
  wstamp(P, b, 6);
  if constexpr (FUSE) {
    if (!uniform_all) return;  // workgroup-uniform: gain_kernel takes per-vehicle rows
#ifdef ACL_EXP_SKIP_GAIN
    return;  // diagnostic builds: the fused kernel without its control phase
#endif
    __syncthreads();           // the auction's tables and the hand-off reads are done
    KCtlParams* pc = (KCtlParams*)((const __attribute__((address_space(4))) char*)
                                       __builtin_amdgcn_kernarg_segment_ptr() +
                                   offsetof(SolveParams, ctl));
    asm volatile("" : "+s"(pc));
    wide_control<GM>(pc, b, f, smem, p, qv, L.qv + wal(n * 24),
                     reinterpret_cast<const uint16_t*>(P.ws + P.W.pt) + (size_t)b * n);
    wstamp(P, b, 7);
  }
  wstamp(P, b, kStampRt1);
}

hipError_t launch_wide(const SolveParams& P, int nb, hipStream_t stream, bool fuse) {
  static PerDeviceOnce once;
  const hipError_t e = once.run([] {
    for (const void* k : {(const void*)align_wide_kernel,
                          (const void*)solve_wide_kernel<false, false, true>,
                          (const void*)solve_wide_kernel<true, false, true>,
                          (const void*)solve_wide_kernel<true, true, true>,
                          (const void*)solve_wide_kernel<false, false, false>,
                          (const void*)solve_wide_kernel<true, false, false>,
                          (const void*)solve_wide_kernel<true, true, false>}) {
      const hipError_t r =
          hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (r != hipSuccess) return r;
    }
    return hipSuccess;
  });
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(align_wide_kernel, dim3(nb), dim3(kWABlock), make_walayout(P.n).total, stream,
                     P);
  const WLayout L = make_wlayout(P.n);
  int lds = L.total;
  if (fuse) {
    const int c = make_wclayout(P.n, L.qv + wal(P.n * 24)).total;
    lds = c > lds ? c : lds;
  }
#define ACL_WIDE_LAUNCH(MG_)                                                                   \
  do {                                                                                         \
    if (!fuse)                                                                                 \
      hipLaunchKernelGGL((solve_wide_kernel<false, false, MG_>), dim3(nb), dim3(kWBlock), lds,   \
                         stream, P);                                                           \
    else if (P.ctl.gate_margin)                                                                \
      hipLaunchKernelGGL((solve_wide_kernel<true, true, MG_>), dim3(nb), dim3(kWBlock), lds,     \
                         stream, P);                                                           \
    else                                                                                       \
      hipLaunchKernelGGL((solve_wide_kernel<true, false, MG_>), dim3(nb), dim3(kWBlock), lds,    \
                         stream, P);                                                           \
  } while (0)
  if (P.skip_margin) ACL_WIDE_LAUNCH(false);
  else ACL_WIDE_LAUNCH(true);
#undef ACL_WIDE_LAUNCH
  return hipGetLastError();
}

}  // namespace acl_amd
