// solve.hip -- the fused batched solve kernel for gfx950 (MI355X).
//
// One workgroup (256 threads = 4 wave64) owns one swarm of n <= 128 vehicles
// for the whole solve; every per-swarm table lives in LDS:
//
//   phase 0  load q, p, adjacency bits, P_in (coalesced, ~10 KB/swarm)
//   phase 1  per-vehicle 2-D Umeyama alignment, one thread per vehicle
//            (Auctioneer::alignFormation, auctioneer.cpp:347-415)
//   phase 2  price matrix C[v][j] (getPrice, auctioneer.cpp:546-549), fp64
//            math, f32 result, n x n in LDS
//   phase 3  CBAA rounds (auctioneer.cpp:182-306,469-542). A table entry is
//            the pair (price, who); since price == C[who][j] always (an entry
//            is created by `who` bidding C[who][j] and only ever copied), the
//            tables store `who` only (u8), 2 x n x n bytes.
//            Per round:  A) per task j: the maximum price over ALL vehicles,
//            its owner and the holder bitmask H_j;  B) per (vehicle v, task j):
//            if some holder of the maximum is in v's closed neighbourhood and
//            the maximum is owned by one `who` only, the winner is that `who`
//            (no tie-break needed); otherwise the exact ordered scan of the
//            reference (ascending vehid, strict >). Then the outbid ->
//            selectTaskAssignment step as a wave argmax.
//            The loop stops at the first round that changes no table: the
//            update is a deterministic function of the tables, so rounds
//            after a fixed point are identical (exact early exit).
//   phase 4  adoption: each vehicle's table -> validity, own formation point
//   phase 5  DistCntrl::compute per vehicle (distcntrl.cpp:46-102): one wave
//            per vehicle, lanes over formation neighbours, 3x3 gain blocks
//            streamed from HBM as 9 coalesced f64 planes; then
//            Safety::cmdinCb saturation and collisionAvoidance
//            (safety.cpp:172-197, 412-541).
//
// Compiled with -ffp-contract=off: every f64 op is one IEEE rounding, so the
// alignment, prices and therefore the assignment are bit-identical to the
// CPU restatement (oracle/).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "../../include/aclswarm_amd.h"
#include "common.h"
#include "umeyama_dev.h"
#include "control_params.h"

namespace acl_amd {

constexpr int kBlock = 512;  // 8 waves per swarm
constexpr int kWaves = kBlock / 64;
constexpr int kMinWavesPerEU = 6;  // 3 swarms x 8 waves per CU (LDS <= 160 KiB / 3)

// LDS layout (byte offsets, 16-byte aligned). The CBAA table T (n x n u8,
// who per vehicle row) is written after the prices are known and overlays
// the arrays only phases 0-2 read (formation-ordered q, p, the alignments,
// the formation adjacency), so one swarm needs ~53 KB at n = 100 and three
// swarms fit a CU.
struct Layout {
  int C;                                  // n x n f32 prices; alignment-sum scratch first
  int A, qf, p, out, adjF;                // region A (phases 0-2) ...
  int T;                                  // ... reused by the CBAA table (phase 3-4)
  int vadj, Pin, Ptin, myi, valid, H, misc;
  int total;
};

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

#ifndef ACL_CBAA_LEVELS
#define ACL_CBAA_LEVELS 3
#endif
constexpr int kLevels = ACL_CBAA_LEVELS;  // price levels resolved per dirty column before the exact scan

__host__ __device__ inline Layout make_layout(int n) {
  Layout L;
  int o = 0;
  L.C = o;
  {
    const int csz = n * n * 4, sc = 64 * n;  // prices / alignment sums [n][8] f64
    o = align16(o + (csz > sc ? csz : sc));
  }
  L.A = o;
  L.qf = o;     o = align16(o + n * 3 * 8);   // q in formation order: qf[j] = q[Pt[j]]
  L.p = o;      o = align16(o + n * 3 * 8);
  L.out = o;    o = align16(o + n * 6 * 8);   // R, t per vehicle
  L.adjF = o;   o = align16(o + n * 2 * 8);
  L.T = L.A;
  if (L.A + n * n > o) o = align16(L.A + n * n);
  L.vadj = o;   o = align16(o + n * 2 * 8);
  L.Pin = o;    o = align16(o + n);
  L.Ptin = o;   o = align16(o + n);
  L.myi = o;    o = align16(o + n);
  L.valid = o;  o = align16(o + n);
  L.H = o;      o = align16(o + 96);
  L.misc = o;   o = align16(o + 64);
  L.total = o;
  return L;
}

__device__ __forceinline__ void stamp(const SolveParams& P, int b, int tid, int k) {
  if (P.stamps && tid == 0) P.stamps[(size_t)b * 16 + k] = __builtin_amdgcn_s_memtime();
}

// Price of a table entry: C[who][j], 0 for `none` (who == n; reset,
// auctioneer.cpp:448-465, price 0).
__device__ __forceinline__ float entry_price(const float* C, int n, int w, int j) {
  const float c = C[(w < n ? w : 0) * n + j];
  return w < n ? c : 0.0f;
}

// selectTaskAssignment (auctioneer.cpp:517-542) for vehicle v as a wave
// argmax: the first task j maximizing C[v][j] among tasks with
// C[v][j] > 0 and C[v][j] > price_j (price_j = C[who_j][j]); nw[c] is this
// lane's entry for task lane+64c. Returns the selected task (wave-uniform) or -1.
__device__ __forceinline__ int wave_select(int n, int v, int lane, const float* C,
                                           const int (&nw)[2], MarginPair& m) {
  unsigned key[2];
  float cvs[2], prs[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int j = lane + 64 * c;
    key[c] = 0u;
    cvs[c] = prs[c] = 0.0f;
    if (j < n) {
      const float cv = C[v * n + j];
      const float pr = entry_price(C, n, nw[c], j);
      if (cv > 0.0f && cv > pr) key[c] = __float_as_uint(cv);
      cvs[c] = cv;
      prs[c] = pr;
    }
  }
  const unsigned M = wave_max_u32(key[0] > key[1] ? key[0] : key[1]);
  int js = -1;
  if (M != 0u) {
    const unsigned long long e0 = __ballot(key[0] == M), e1 = __ballot(key[1] == M);
    js = e0 ? __ffsll((long long)e0) - 1 : 64 + __ffsll((long long)e1) - 1;
  }
  // margin of the decisive comparisons (include/aclswarm_amd.h)
  const float cmax = __uint_as_float(M);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int j = lane + 64 * c;
    if (j >= n || nw[c] == v) continue;
    if (j == js) margin_track(m, cvs[c], prs[c]);
    else if (key[c] != 0u) margin_track(m, cmax, cvs[c]);
    else if (cvs[c] > 0.0f && (js < 0 || cvs[c] > cmax || (cvs[c] == cmax && j < js)))
      margin_track(m, prs[c], cvs[c]);
  }
  return js;
}

__global__ void __launch_bounds__(kBlock, kMinWavesPerEU) solve_kernel(const SolveParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const Layout L = make_layout(n);
  const int b = P.b0 + blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;

  float* C = reinterpret_cast<float*>(smem + L.C);
  double* qf = reinterpret_cast<double*>(smem + L.qf);
  double* p = reinterpret_cast<double*>(smem + L.p);
  double* out = reinterpret_cast<double*>(smem + L.out);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adjF);
  unsigned long long* vadj = reinterpret_cast<unsigned long long*>(smem + L.vadj);
  unsigned long long* H = reinterpret_cast<unsigned long long*>(smem + L.H);
  unsigned char* const T = smem + L.T;
  unsigned char* Pin = smem + L.Pin;
  unsigned char* Ptin = smem + L.Ptin;
  unsigned char* myi = smem + L.myi;
  unsigned char* validv = smem + L.valid;
  int* misc = reinterpret_cast<int*>(smem + L.misc);

  // a formation index out of range is a bad input like a bad P_in
  const int f_in = P.fidx[b];
  const bool fbad = f_in < 0 || f_in >= P.F;
  const int f = fbad ? 0 : f_in;
  MarginPair mp;
  margin_init(mp);
  double galign = 1.0;
  const int gw = (n + 63) >> 6;  // words per row in the global table
  const unsigned long long lastmask =
      (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  stamp(P, b, tid, 0);

  // ---------------- phase 0: load -----------------------------------------
  {
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += kBlock) p[k] = gp[k];
    const uint64_t* ga = P.adj + (size_t)f * n * gw;
    for (int k = tid; k < n * 2; k += kBlock) {
      const int i = k >> 1, w = k & 1;
      unsigned long long x = 0;
      if (w < gw) {
        x = ga[(size_t)i * gw + w];
        if (w == gw - 1) x &= lastmask;
      }
      adjF[k] = x;
    }
    if (tid < 16) misc[tid] = 0;
    if (tid < 2) H[tid] = 0ull;  // "seen" mask for the permutation check
  }
  __syncthreads();
  if (tid == 0) {
    misc[M_AGREE] = 1;
    if (fbad) misc[M_BAD] = 1;
    *reinterpret_cast<unsigned long long*>(misc + M_MARG) =
        (unsigned long long)__double_as_longlong(1.0);
  }
  __syncthreads();
  for (int v = tid; v < n; v += kBlock) {
    const unsigned pv = P.P_in[(size_t)b * n + v];
    Pin[v] = (unsigned char)pv;
    if (pv >= (unsigned)n) {
      misc[M_BAD] = 1;
    } else {
      // two vehicles claiming the same point -> not a permutation
      const unsigned long long bit = 1ull << (pv & 63);
      const unsigned long long prev = atomicOr(&H[pv >> 6], bit);
      if (prev & bit) misc[M_BAD] = 1;
      Ptin[pv] = (unsigned char)v;
    }
  }
  __syncthreads();
  if (misc[M_BAD]) {
    // P_in is not a permutation: the reference never holds such a P.
    for (int v = tid; v < n; v += kBlock) {
      P.P_out[(size_t)b * n + v] = P.P_in[(size_t)b * n + v];
      if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 0;
    }
    for (int k = tid; k < 3 * n; k += kBlock) {
      if (P.u) P.u[(size_t)b * n * 3 + k] = 0.0;
      if (P.u_safe) P.u_safe[(size_t)b * n * 3 + k] = 0.0;
    }
    if (P.who)
      for (int k = tid; k < n * n; k += kBlock) P.who[(size_t)b * n * n + k] = 0xFFFF;
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

  // q in formation order: qf[j] = q[Pt[j]] (the alignment reads the
  // formation-ordered xy, the prices read qf[P[v]] = q[v])
  {
    const double* gq = P.q + (size_t)b * n * 3;
    for (int k = tid; k < 3 * n; k += kBlock) {
      const int j = k / 3, c = k - 3 * j;
      qf[k] = gq[3 * Ptin[j] + c];
    }
  }
  // vehicle-space closed neighbourhoods: u ~ v iff u == v or adj(P[v], P[u])
  // (bidIterComplete, auctioneer.cpp:419-437); one wave per vehicle, lanes
  // over u, one ballot per 64-bit word
  {
    const int pu0 = (lane < n) ? Pin[lane] : 0;
    const int pu1 = (64 + lane < n) ? Pin[64 + lane] : 0;
    for (int v = wave; v < n; v += kWaves) {
      const int i = Pin[v];
      const unsigned long long a0 = adjF[2 * i], a1 = adjF[2 * i + 1];
      const bool e0 = (lane < n) && ((lane == v) || (((pu0 < 64 ? a0 : a1) >> (pu0 & 63)) & 1ull));
      const bool e1 = (64 + lane < n) &&
                      ((64 + lane == v) || (((pu1 < 64 ? a0 : a1) >> (pu1 & 63)) & 1ull));
      const unsigned long long m0 = __ballot(e0), m1 = __ballot(e1);
      if (lane == 0) {
        vadj[2 * v] = m0;
        vadj[2 * v + 1] = m1;
      }
    }
  }
  __syncthreads();
  stamp(P, b, tid, 1);

  // ---------------- phase 1: alignment -------------------------------------
  // Eigen::umeyama's sums run sequentially in ascending neighbour order; each
  // of the 4 sums of a pass is one thread's sequential loop (4 threads per
  // vehicle), so the order -- and every rounding -- is the reference's.
  double* sums = reinterpret_cast<double*>(C);  // [n][8] scratch (C is filled later)
  {
    const int v = tid >> 2, c = tid & 3;
    const bool act = v < n;
    const int i = act ? Pin[v] : 0;
    unsigned long long r0 = adjF[2 * i], r1 = adjF[2 * i + 1];
    if (i < 64) r0 |= 1ull << i; else r1 |= 1ull << (i - 64);
    // pass 1: rowwise().sum() of src (p) and dst (q in formation space).
    // Branch-free: the sum starts at -0.0, the additive identity of IEEE
    // addition (x + -0.0 == x for every x, +0.0 and NaN included), and a
    // point outside the neighbourhood adds -0.0 -- the same roundings as
    // Eigen's "first element, then += the rest".
    const double* src = (c < 2) ? (p + c) : (qf + (c - 2));
    double acc = -0.0;
    for (int jb = 0; jb < n; jb += 32) {
      const unsigned m = (unsigned)((jb < 64 ? r0 : r1) >> (jb & 63));
#pragma unroll
      for (int x = 0; x < 32; ++x) {
        const int j = jb + x < n ? jb + x : n - 1;
        const double val = src[j * 3];
        acc += ((m >> x) & 1u) ? val : -0.0;  // bits past n are 0
      }
    }
    if (act) sums[8 * v + c] = acc;
  }
  __syncthreads();
  stamp(P, b, tid, 8);
  {
    const int v = tid >> 2, c = tid & 3;
    const bool act = v < n;
    const int i = act ? Pin[v] : 0;
    unsigned long long r0 = adjF[2 * i], r1 = adjF[2 * i + 1];
    if (i < 64) r0 |= 1ull << i; else r1 |= 1ull << (i - 64);
    const int k = __popcll(r0) + __popcll(r1);
    const double oon = 1.0 / (double)k;
    // pass 2: a_(di,sj) = sum_j dst_demean[di] * src_demean[sj]; c = 2*di + sj
    const int di = c >> 1, sj = c & 1;
    const double smj = act ? sums[8 * v + sj] * oon : 0.0;
    const double dmi = act ? sums[8 * v + 2 + di] * oon : 0.0;
    // sigma = one_over_n * dst_demean * src_demean^T: lazy product (scaled
    // lhs) when k + 4 < 20, GEMM (alpha after the sum) otherwise
    const bool lazy = (k + 4) < 20;
    // branch-free as pass 1: the lazy product starts at its first term
    // (-0.0 start), the GEMM form at 0.0; excluded points add -0.0; the
    // lazy scaling multiplies by oon, the other form by 1.0 (exact)
    const double scale = lazy ? oon : 1.0;
    double acc = lazy ? -0.0 : 0.0;
    // 1.0 * x == x exactly: a wave with no lazy-product vehicle skips the
    // scaling multiply (every vehicle with k + 4 >= 20, e.g. all at n = 100)
    auto pass2 = [&](auto scaled) {
      for (int jb = 0; jb < n; jb += 32) {
        const unsigned m = (unsigned)((jb < 64 ? r0 : r1) >> (jb & 63));
#pragma unroll
        for (int x = 0; x < 32; ++x) {
          const int j = jb + x < n ? jb + x : n - 1;
          const double s0 = p[3 * j + sj] - smj;
          const double dd = qf[3 * j + di] - dmi;
          const double d0 = decltype(scaled)::value ? scale * dd : dd;
          const double pr = d0 * s0;
          acc += ((m >> x) & 1u) ? pr : -0.0;
        }
      }
    };
    if (__ballot(act && lazy) != 0ull)
      pass2(std::true_type{});
    else
      pass2(std::false_type{});
    if (act) sums[8 * v + 4 + c] = lazy ? acc : acc * oon;
  }
  __syncthreads();
  stamp(P, b, tid, 9);
  for (int v = tid; v < n; v += kBlock) {
    const int i = Pin[v];
    unsigned long long r0 = adjF[2 * i], r1 = adjF[2 * i + 1];
    if (i < 64) r0 |= 1ull << i; else r1 |= 1ull << (i - 64);
    const int k = __popcll(r0) + __popcll(r1);
    const double oon = 1.0 / (double)k;
    const double sm[2] = {sums[8 * v] * oon, sums[8 * v + 1] * oon};
    const double dm[2] = {sums[8 * v + 2] * oon, sums[8 * v + 3] * oon};
    // column-major sigma: S(di, sj) = a_(di, sj)
    const double S[4] = {sums[8 * v + 4], sums[8 * v + 6], sums[8 * v + 5], sums[8 * v + 7]};
    double R[4], t[2], ga;
    umeyama_finish(S, sm, dm, R, t, &ga);
    galign = ga < galign ? ga : galign;
    double* o = out + 6 * v;
    o[0] = R[0]; o[1] = R[1]; o[2] = R[2]; o[3] = R[3]; o[4] = t[0]; o[5] = t[1];
  }
  __syncthreads();
  if (P.align_Rt)
    for (int k = tid; k < 6 * n; k += kBlock) P.align_Rt[(size_t)b * n * 6 + k] = out[k];
  stamp(P, b, tid, 2);

  // ---------------- phase 2: prices ---------------------------------------
  {
    // thread -> fixed task j, vehicles v0, v0 + per, ... (no per-entry
    // index division; p_j stays in registers)
    int nonfin = 0;
    const int per = kBlock / n;
    const int j = tid % n, v0 = tid / n;
    const double px = p[3 * j], py = p[3 * j + 1], pz = p[3 * j + 2];
    for (int v = v0; v0 < per && v < n; v += per) {
      const int k = v * n + j;
      const double* o = out + 6 * v;
      const double* qv = qf + 3 * Pin[v];
      const double ax = ((o[0] * px + o[1] * py) + 0.0 * pz) + o[4];
      const double ay = ((o[2] * px + o[3] * py) + 0.0 * pz) + o[5];
      const double az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0;
      const double dx = qv[0] - ax, dy = qv[1] - ay, dz = qv[2] - az;
      const double nrm = sqrt((dx * dx + dy * dy) + dz * dz);
      const float c = (float)(1.0 / (nrm + 1e-8));
      C[k] = c;
      nonfin |= (c != c);
    }
    if (__any(nonfin) && lane == 0) misc[M_NONFIN] = 1;
  }
  // closed neighbourhood masks of this lane's vehicles (lane, lane + 64)
  unsigned long long vmy0[2], vmy1[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int v = lane + 64 * c;
    vmy0[c] = (v < n) ? vadj[2 * v] : 0ull;
    vmy1[c] = (v < n) ? vadj[2 * v + 1] : 0ull;
  }
  __syncthreads();  // region A (q, p, alignments) is dead from here: T overlays it
  const bool nonfinite = misc[M_NONFIN] != 0;
  // initial tables: every entry unassigned (reset, auctioneer.cpp:448-465)
  for (int k = tid; k < n * n; k += kBlock) T[k] = (unsigned char)n;
  // CBAA state: dirty-column masks and outbid-vehicle masks by round parity
  unsigned long long* dmask = H;      // [2][2]
  unsigned long long* obm = H + 4;    // [2][2]
  if (tid < 8) H[tid] = 0ull;
  __syncthreads();
  stamp(P, b, tid, 3);

  // ---------------- phase 3: CBAA ------------------------------------------
  // round 0: START bid = select from the zero table (start, auctioneer.cpp:105);
  // every column that received a bid is dirty for round 1
  for (int v = wave; v < n; v += kWaves) {
    int nw[2] = {n, n};
    const int task = wave_select(n, v, lane, C, nw, mp);
    if (task >= 0 && lane == 0) {
      T[v * n + task] = (unsigned char)v;
      atomicOr(&dmask[2 * 1 + (task >> 6)], 1ull << (task & 63));
    }
  }
  __syncthreads();

  int eff = 0;
  const int max_rounds = 2 * n;  // cbaa_max_iter_ = n * diameter (:50-51)
  const bool ok0 = lane < n, ok1 = lane + 64 < n;
  // diagnostic counters (stamps only): cycles of the column part and of the
  // select part as seen by thread 0, dirty columns, outbid vehicles
  unsigned long long tA = 0, tB = 0, nDirty = 0, nOut = 0;
  for (int r = 1; r <= max_rounds; ++r) {
    const int par = r & 1, npar = par ^ 1;
    const unsigned long long D0 = dmask[2 * par], D1 = dmask[2 * par + 1];
    const unsigned long long t0 = P.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
    if (P.stamps) nDirty += __popcll(D0) + __popcll(D1);
    // One wave per dirty column j, lanes = vehicles (two chunks of 64). A
    // column none of whose entries changed last round is a fixed point of
    // updateTaskAssignment (it reads only that column, and a select always
    // changes the entry it writes), so only dirty columns are recomputed.
    // Each column is read whole into registers before it is rewritten in
    // place; no other wave touches it this round.
    int idx = 0;
    for (int w = 0; w < 2; ++w) {
      unsigned long long m = w ? D1 : D0;
      while (m) {
        const int j = 64 * w + __ffsll((long long)m) - 1;
        m &= m - 1;
        if ((idx++ & (kWaves - 1)) != wave) continue;
        const int wu0 = ok0 ? T[lane * n + j] : n;
        const int wu1 = ok1 ? T[(lane + 64) * n + j] : n;
        // key = price bits + 1 (prices are >= 0); 0 = no vehicle in this lane
        const unsigned key0 = ok0 ? __float_as_uint(entry_price(C, n, wu0, j)) + 1u : 0u;
        const unsigned key1 = ok1 ? __float_as_uint(entry_price(C, n, wu1, j)) + 1u : 0u;
        // A) price levels of the column, highest first, computed lazily:
        //    level k = (max key below level k-1, holder mask, `who`, tie).
        // B) vehicle v takes the `who` of the highest level one of its
        //    closed neighbours holds, unless that level is tied; vehicles
        //    no tracked level decides fall back to the exact ordered scan
        //    (ascending vehid, strict >).
        // per vehicle: st 0 = undecided, 1 = winner level found (k1), 2 =
        // done (k2 = the next level its neighbourhood holds, the margin's
        // runner-up; 0 = none); need = exact ordered scan
        int nw0 = n, nw1 = n;
        int st0 = ok0 ? 0 : 2, st1 = ok1 ? 0 : 2;
        unsigned k10 = 0u, k11 = 0u, k20 = 0u, k21 = 0u;
        bool need0 = false, need1 = false, exhausted = false;
        unsigned cap = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < kLevels + 1; ++k) {
          const unsigned Mk = wave_max_u32(max(key0 < cap ? key0 : 0u, key1 < cap ? key1 : 0u));
          if (Mk == 0u) {  // no further level
            exhausted = true;
            break;
          }
          const bool e0 = key0 == Mk, e1 = key1 == Mk;
          const unsigned long long h0 = __ballot(e0), h1 = __ballot(e1);
          const int wk = h0 ? __builtin_amdgcn_readlane(wu0, __ffsll((long long)h0) - 1)
                            : __builtin_amdgcn_readlane(wu1, __ffsll((long long)h1) - 1);
          const bool tk = nonfinite || __ballot((e0 && wu0 != wk) || (e1 && wu1 != wk)) != 0ull;
          const bool hit0 = st0 < 2 && !need0 && ((h0 & vmy0[0]) | (h1 & vmy1[0])) != 0ull;
          const bool hit1 = st1 < 2 && !need1 && ((h0 & vmy0[1]) | (h1 & vmy1[1])) != 0ull;
          if (hit0) {
            if (st0 == 0) { nw0 = wk; k10 = Mk; need0 = tk; st0 = 1; }
            else { k20 = Mk; st0 = 2; }
          }
          if (hit1) {
            if (st1 == 0) { nw1 = wk; k11 = Mk; need1 = tk; st1 = 1; }
            else { k21 = Mk; st1 = 2; }
          }
          if (__ballot((st0 < 2 && !need0) || (st1 < 2 && !need1)) == 0ull) break;
          cap = Mk;
        }
        need0 |= st0 == 0 || (st0 == 1 && !exhausted);
        need1 |= st1 == 0 || (st1 == 1 && !exhausted);
        if (!need0 && k20 != 0u) margin_track(mp, __uint_as_float(k10 - 1u), __uint_as_float(k20 - 1u));
        if (!need1 && k21 != 0u) margin_track(mp, __uint_as_float(k11 - 1u), __uint_as_float(k21 - 1u));
        if (__ballot(need0 || need1) != 0ull) {
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            if (c ? need1 : need0) {
              float bp = 0.0f, p2 = 0.0f;
              int bw = n;
              bool first = true, have2 = false;
#pragma unroll
              for (int w2 = 0; w2 < 2; ++w2) {
                unsigned long long mm = w2 ? vmy1[c] : vmy0[c];
                while (mm) {
                  const int u = 64 * w2 + __ffsll((long long)mm) - 1;
                  mm &= mm - 1;
                  const int wx = T[u * n + j];
                  const float px = entry_price(C, n, wx, j);
                  if (first) { bp = px; bw = wx; first = false; }
                  else if (px > bp) { p2 = bp; have2 = true; bp = px; bw = wx; }
                  else if (wx != bw) { if (!have2 || px > p2) p2 = px; have2 = true; }
                }
              }
              if (c) nw1 = bw; else nw0 = bw;
              if (have2) margin_track(mp, bp, p2);
            }
          }
        }
        // the exact scan above read the column: rewrite it only now
        __builtin_amdgcn_wave_barrier();
        if (ok0) T[lane * n + j] = (unsigned char)nw0;
        if (ok1) T[(lane + 64) * n + j] = (unsigned char)nw1;
        const unsigned long long ob0 = __ballot(ok0 && wu0 == lane && nw0 != lane);
        const unsigned long long ob1 = __ballot(ok1 && wu1 == lane + 64 && nw1 != lane + 64);
        const bool anych = __ballot(nw0 != wu0 || nw1 != wu1) != 0ull;
        if (lane == 0) {
          if (ob0) atomicOr(&obm[2 * par], ob0);  // outbid (auctioneer.cpp:502)
          if (ob1) atomicOr(&obm[2 * par + 1], ob1);
          if (anych) atomicOr(&dmask[2 * npar + (j >> 6)], 1ull << (j & 63));
        }
      }
    }
    __syncthreads();
    const unsigned long long t1 = P.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
    if (P.stamps) nOut += __popcll(obm[2 * par]) + __popcll(obm[2 * par + 1]);
    // outbid vehicles re-select on their updated rows (auctioneer.cpp:224)
    {
      if (tid == 0) {
        dmask[2 * par] = 0ull;        // consumed; becomes round r+2's mask
        dmask[2 * par + 1] = 0ull;
        obm[2 * npar] = 0ull;         // round r+1's outbid mask
        obm[2 * npar + 1] = 0ull;
      }
      const unsigned long long O0 = obm[2 * par], O1 = obm[2 * par + 1];
      int idx2 = 0;
      for (int w = 0; w < 2; ++w) {
        unsigned long long m = w ? O1 : O0;
        while (m) {
          const int v = 64 * w + __ffsll((long long)m) - 1;
          m &= m - 1;
          if ((idx2++ & (kWaves - 1)) != wave) continue;
          int nw[2];
          nw[0] = ok0 ? T[v * n + lane] : n;
          nw[1] = ok1 ? T[v * n + lane + 64] : n;
          const int task = wave_select(n, v, lane, C, nw, mp);
          if (task >= 0 && lane == 0) {
            T[v * n + task] = (unsigned char)v;
            atomicOr(&dmask[2 * npar + (task >> 6)], 1ull << (task & 63));
          }
        }
      }
    }
    __syncthreads();
    if (P.stamps) {
      const unsigned long long t2 = __builtin_amdgcn_s_memtime();
      tA += t1 - t0;
      tB += t2 - t1;
    }
    const bool changed = (dmask[2 * npar] | dmask[2 * npar + 1]) != 0ull;
    if (changed) eff = r;
    else if (P.early_exit) break;  // fixed point
  }
  {  // swarm margin: every thread's CBAA pair and alignment gaps
    const double gc = margin_gap(mp);
    block_min_gap(reinterpret_cast<unsigned long long*>(misc + M_MARG),
                  gc < galign ? gc : galign);
  }
  stamp(P, b, tid, 4);
  if (P.stamps && tid == 0) {
    unsigned long long* st = P.stamps + (size_t)b * 16;
    st[10] = tA; st[11] = tB; st[12] = nDirty; st[13] = nOut;
  }

  // ---------------- phase 4: adoption --------------------------------------
  // AGREE: is every vehicle's table equal to vehicle 0's?
  for (int v = wave; v < n; v += kWaves) {
    bool diff = false;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int jj = lane + 64 * c;
      if (jj < n) diff |= T[v * n + jj] != T[jj];
    }
    if (__any(diff) && lane == 0) misc[M_AGREE] = 0;
  }
  __syncthreads();
  const bool allagree = misc[M_AGREE] != 0;
  // isValidAssignment (auctioneer.cpp:325-343) of a table row: one wave,
  // lanes over tasks; a permutation <=> every entry < n and the OR of the
  // one-hot entries has n bits
  auto row_valid = [&](const unsigned char* row) -> bool {
    unsigned lo[4] = {0u, 0u, 0u, 0u};
    bool bad = false;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int jj = lane + 64 * c;
      if (jj < n) {
        const int w = row[jj];
        if (w >= n) bad = true;
        else lo[w >> 5] |= 1u << (w & 31);
      }
    }
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) cnt += __popc(wave_or_u32(lo[k]));
    return !__any(bad) && cnt == n;
  };
  // with all tables equal, vehicle 0's verdict is every vehicle's (each
  // wave checks row 0 itself: no further barrier)
  const bool valid0 = allagree && row_valid(T);
  for (int v = wave; v < n; v += kWaves) {
    const unsigned char* row = T + v * n;
    bool ismine[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int jj = lane + 64 * c;
      ismine[c] = (jj < n) && (row[jj] == v);
    }
    const unsigned long long mm0 = __ballot(ismine[0]), mm1 = __ballot(ismine[1]);
    const bool valid = (allagree ? valid0 : row_valid(row)) && (mm0 | mm1) != 0ull;
    const int mine = valid ? (mm0 ? __ffsll((long long)mm0) - 1 : 64 + __ffsll((long long)mm1) - 1)
                           : Pin[v];
    if (lane == 0) {
      validv[v] = valid;
      myi[v] = (unsigned char)mine;
      if (!valid) atomicAdd(&misc[M_NINV], 1);
      if (mine != Pin[v]) misc[M_CHANGED] = 1;
      P.P_out[(size_t)b * n + v] = (uint16_t)mine;
    }
  }
  if (P.who) {
    for (int k = tid; k < n * n; k += kBlock) {
      const int w = T[k];
      P.who[(size_t)b * n * n + k] = (w >= n) ? (uint16_t)0xFFFF : (uint16_t)w;
    }
  }
  __syncthreads();
  stamp(P, b, tid, 5);

  // ---------------- hand-off to the control kernel ------------------------
  // Each vehicle's adopted inverse assignment (formation point -> vehicle):
  // one shared row when every vehicle adopts the same one (all tables valid
  // and identical, or none valid), else one row per vehicle.
  {
    const bool allvalid = misc[M_NINV] == 0;
    const bool uniform = (allvalid && misc[M_AGREE]) || misc[M_NINV] == n;
    uint16_t* wsPt = reinterpret_cast<uint16_t*>(P.ws + P.W.pt) + (size_t)b * n;
    if (tid == 0) P.ws[P.W.mode + b] = uniform ? 0 : 1;
    if (uniform) {
      for (int jj = tid; jj < n; jj += kBlock) wsPt[jj] = allvalid ? T[jj] : Ptin[jj];
    } else {
      uint16_t* rows = reinterpret_cast<uint16_t*>(P.ws + P.W.rows) + (size_t)b * n * n;
      for (int k = tid; k < n * n; k += kBlock) {
        const int v = k / n, jj = k - v * n;
        rows[k] = validv[v] ? T[k] : Ptin[jj];
      }
    }
  }
  stamp(P, b, tid, 6);
  if (tid == 0) {
    acl_swarm_status_t st = {};
    uint32_t fl = 0;
    if (misc[M_NINV] == 0) fl |= ACL_SWARM_VALID;
    if (misc[M_AGREE]) fl |= ACL_SWARM_AGREE;
    if (misc[M_CHANGED]) fl |= ACL_SWARM_CHANGED;
    if (nonfinite) fl |= ACL_SWARM_NONFINITE;
    if (misc[M_NCA]) fl |= ACL_SWARM_CA_ACTIVE;
    const double g = nonfinite ? 0.0
        : __longlong_as_double((long long)*reinterpret_cast<unsigned long long*>(misc + M_MARG));
    if (g < ACL_FRAGILE_MARGIN) fl |= ACL_SWARM_FRAGILE;
    st.margin = (float)g;
    st.flags = fl;
    st.eff_rounds = (uint16_t)eff;
    st.rounds = (uint16_t)(2 * n);
    st.n_invalid = (uint16_t)misc[M_NINV];
    st.n_ca = (uint16_t)misc[M_NCA];
    P.status[b] = st;
  }
}
}  // namespace acl_amd

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" acl_status_t acl__set_error(const char* msg);

extern "C" int32_t acl_max_vehicles(void) { return acl_amd::kMaxNWide; }

// Diagnostic hook (not part of the public ABI): when set, the next solves
// record s_memtime at the end of each phase into stamps[B][8].
static unsigned long long* g_stamps = nullptr;
extern "C" void acl_internal_set_stamps(unsigned long long* stamps) { g_stamps = stamps; }

extern "C" size_t acl_solve_workspace_bytes(int32_t n, int32_t B) {
  if (n < 1 || B < 0) return 0;
  return acl_amd::ws_layout(n, B).total;
}

namespace {
// Diagnostic per-launch kernel timing (not part of the public ABI): events
// around each kernel launch, so bench.py can report every kernel's own time.
struct KTiming {
  bool on = false;
  int n[3] = {0, 0, 0};
  hipEvent_t ev[3][64][2] = {};
};
KTiming g_kt;

void kt_record(int kind, int which, hipStream_t s) {
  if (!g_kt.on) return;
  const int i = g_kt.n[kind];
  if (i >= 64) return;
  hipEvent_t& e = g_kt.ev[kind][i][which];
  if (!e) (void)hipEventCreate(&e);
  (void)hipEventRecord(e, s);
  if (which == 1) g_kt.n[kind] = i + 1;
}
}  // namespace

// enable != 0 starts a fresh timing window; 0 stops recording.
extern "C" void acl_internal_kernel_timing(int enable) {
  g_kt.on = enable != 0;
  if (enable) g_kt.n[0] = g_kt.n[1] = g_kt.n[2] = 0;
}

// Sums the recorded launches: ms[k]/count[k] for k = 0 auction kernel,
// 1 gain kernel, 2 collision-avoidance kernel. Synchronises on the events.
extern "C" int acl_internal_kernel_times(double* ms, int* count) {
  for (int k = 0; k < 3; ++k) {
    double t = 0.0;
    for (int i = 0; i < g_kt.n[k]; ++i) {
      float x = 0.f;
      if (hipEventSynchronize(g_kt.ev[k][i][1]) != hipSuccess ||
          hipEventElapsedTime(&x, g_kt.ev[k][i][0], g_kt.ev[k][i][1]) != hipSuccess)
        return -1;
      t += x;
    }
    ms[k] = t;
    count[k] = g_kt.n[k];
  }
  return 0;
}

// ACLSWARM_AMD_AUCTION=old selects the previous LDS auction kernel
// (solve_kernel) for n <= 128 (diagnostic A/B switch; read once).
static bool auction_v2_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("ACLSWARM_AMD_AUCTION");
    on = (e && e[0] == 'o') ? 0 : 1;
  }
  return on != 0;
}

// The batch runs as three stream-ordered launches: the auction kernel over
// all B swarms (solve_kernel for n <= 128, tables in LDS; solve_wide_kernel
// for n <= 512, tables in the workspace), the gain kernel, and the
// collision-avoidance kernel over the vehicles the gain kernel listed.
// (Overlapping the auction with the control stage on a second stream was
// measured slower: both compete for the same CU slots.)
extern "C" acl_status_t acl_solve_batch(const acl_formations_t* F, const acl_solve_args_t* a,
                                        void* stream) {
  using namespace acl_amd;
  if (!F || !a) return acl__set_error("acl_solve_batch: null argument");
  const int n = F->n;
  if (n < 1 || n > kMaxNWide) return acl__set_error("acl_solve_batch: n out of range [1, 512]");
  if (a->B < 0) return acl__set_error("acl_solve_batch: B < 0");
  if (a->B == 0) return ACL_OK;
  if (!F->p || !F->adj || !a->fidx || !a->q || !a->P_in || !a->P_out || !a->status)
    return acl__set_error("acl_solve_batch: required pointer is NULL");
  if (F->n_formations < 1) return acl__set_error("acl_solve_batch: n_formations < 1");
  if (!a->workspace)
    return acl__set_error("acl_solve_batch: workspace is NULL (acl_solve_workspace_bytes)");
  if (a->do_control && (!F->gains || !F->gain_off || !a->vel))
    return acl__set_error("acl_solve_batch: do_control needs gains, gain_off and vel");
  if (a->do_control && F->gain_planes != 0 && F->gain_planes != 9 && F->gain_planes != 5)
    return acl__set_error("acl_solve_batch: gain_planes must be 9 (or 0) or 5");
  SolveParams P;
  P.n = n; P.B = a->B; P.F = F->n_formations; P.b0 = 0;
  P.p = F->p; P.adj = F->adj; P.gains = F->gains; P.gain_off = F->gain_off;
  P.fidx = a->fidx; P.q = a->q; P.vel = a->vel; P.P_in = a->P_in; P.P_out = a->P_out;
  P.status = a->status; P.u = a->u; P.u_safe = a->u_safe; P.ca_flag = a->ca_flag;
  P.who = a->who; P.align_Rt = a->align_Rt; P.g = a->cntrl; P.s = a->safety;
  P.early_exit = a->early_exit; P.do_control = a->do_control;
  P.ws = (unsigned char*)a->workspace;
  P.W = ws_layout(n, a->B);
  P.stamps = g_stamps;
  P.gate_margin = a->do_control ? a->gate_margin : nullptr;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  kt_record(0, 0, s);
  if (n <= kMaxN && auction_v2_enabled()) {
    e = launch_auction(P, a->B, s);
  } else if (n <= kMaxN) {
    static int configured = 0;
    if (!configured) {
      if (hipFuncSetAttribute((const void*)solve_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
        return acl__set_error("hipFuncSetAttribute failed");
      configured = 1;
    }
    const Layout L = make_layout(n);
    hipLaunchKernelGGL(solve_kernel, dim3(a->B), dim3(kBlock), L.total, s, P);
    e = hipGetLastError();
  } else {
    e = launch_wide(P, a->B, s);
  }
  kt_record(0, 1, s);
  if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  if (!a->do_control) return ACL_OK;
  CtlParams C;
  C.n = n; C.B = a->B; C.b0 = 0;
  C.p = F->p; C.adj = F->adj; C.gains = F->gains; C.gain_off = F->gain_off;
  C.gain_planes = F->gain_planes == 5 ? 5 : 9;
  C.gains_tiled = (C.gain_planes == 5 && n <= kMaxN) ? F->gains_tiled : nullptr;
  C.fidx = a->fidx; C.q = a->q; C.vel = a->vel; C.P_out = a->P_out;
  C.status = a->status;
  C.u = a->u ? a->u : reinterpret_cast<double*>(P.ws + P.W.u);
  C.u_safe = a->u_safe; C.ca_flag = a->ca_flag;
  C.wsPt = reinterpret_cast<const uint16_t*>(P.ws + P.W.pt);
  C.wsMode = P.ws + P.W.mode;
  C.wsRows = reinterpret_cast<const uint16_t*>(P.ws + P.W.rows);
  C.ca_list = reinterpret_cast<unsigned*>(P.ws + P.W.calist);
  C.ca_count = reinterpret_cast<unsigned*>(P.ws + P.W.cacount);
  C.g = a->cntrl; C.s = a->safety;
  C.only_nonuniform = 0;
  C.all_uniform = 0;
  C.F = F->n_formations;
  C.gate_margin = a->gate_margin;
  if (hipMemsetAsync(C.ca_count, 0, sizeof(unsigned), s) != hipSuccess)
    return acl__set_error("hipMemsetAsync failed");
  for (int which = 0; which < 2; ++which) {
    kt_record(1 + which, 0, s);
    e = launch_control(C, a->B, which, s);
    kt_record(1 + which, 1, s);
    if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  }
  return ACL_OK;
}

acl_status_t acl_amd::run_control(const acl_formations_t* F, const acl_control_args_t* a,
                                  hipStream_t s, int flags) {
  using namespace acl_amd;
  if (!F || !a) return acl__set_error("acl_control_batch: null argument");
  const int n = F->n;
  if (n < 1 || n > kMaxNWide) return acl__set_error("acl_control_batch: n out of range [1, 512]");
  if (a->B < 0) return acl__set_error("acl_control_batch: B < 0");
  if (a->B == 0) return ACL_OK;
  if (!F->p || !F->adj || !F->gains || !F->gain_off || !a->fidx || !a->q || !a->vel || !a->P ||
      !a->status || !a->workspace)
    return acl__set_error("acl_control_batch: required pointer is NULL");
  if (F->gain_planes != 0 && F->gain_planes != 9 && F->gain_planes != 5)
    return acl__set_error("acl_control_batch: gain_planes must be 9 (or 0) or 5");
  if (F->n_formations < 1) return acl__set_error("acl_control_batch: n_formations < 1");
  const WsLayout W = ws_layout(n, a->B);
  unsigned char* ws = (unsigned char*)a->workspace;
  CtlParams C;
  C.n = n; C.B = a->B; C.b0 = 0;
  C.p = F->p; C.adj = F->adj; C.gains = F->gains; C.gain_off = F->gain_off;
  C.gain_planes = F->gain_planes == 5 ? 5 : 9;
  C.gains_tiled = (C.gain_planes == 5 && n <= kMaxN) ? F->gains_tiled : nullptr;
  C.fidx = a->fidx; C.q = a->q; C.vel = a->vel; C.P_out = a->P;
  C.status = a->status;
  C.u = a->u ? a->u : reinterpret_cast<double*>(ws + W.u);
  C.u_safe = a->u_safe; C.ca_flag = a->ca_flag;
  C.wsPt = reinterpret_cast<const uint16_t*>(ws + W.pt);
  C.wsMode = ws + W.mode;
  C.wsRows = reinterpret_cast<const uint16_t*>(ws + W.rows);
  C.ca_list = reinterpret_cast<unsigned*>(ws + W.calist);
  C.ca_count = reinterpret_cast<unsigned*>(ws + W.cacount);
  C.g = a->cntrl; C.s = a->safety;
  C.only_nonuniform = 0;
  C.all_uniform = 1;  // the hand-off of a given P is one assignment per swarm
  C.F = F->n_formations;
  C.gate_margin = a->gate_margin;
  if ((flags & CTL_RESET) && hipMemsetAsync(C.ca_count, 0, sizeof(unsigned), s) != hipSuccess)
    return acl__set_error("hipMemsetAsync failed");
  hipError_t e = hipSuccess;
  if (flags & CTL_PREP) {
    e = launch_control_prep(C, a->P, a->B, s);
    if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  }
  for (int which = 0; which < 2; ++which) {
    e = launch_control(C, a->B, which, s);
    if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  }
  return ACL_OK;
}

extern "C" acl_status_t acl_control_batch(const acl_formations_t* F, const acl_control_args_t* a,
                                          void* stream) {
  return acl_amd::run_control(F, a, (hipStream_t)stream, acl_amd::CTL_PREP | acl_amd::CTL_RESET);
}

extern "C" acl_status_t acl_tile_gains(const acl_formations_t* F, double* out, void* stream) {
  using namespace acl_amd;
  if (!F || !out) return acl__set_error("acl_tile_gains: null argument");
  if (F->gain_planes != 5) return acl__set_error("acl_tile_gains: gain_planes must be 5");
  if (F->n < 1 || F->n > kMaxN) return acl__set_error("acl_tile_gains: n out of range [1, 128]");
  if (F->n_formations < 0) return acl__set_error("acl_tile_gains: n_formations < 0");
  if (F->n_formations == 0) return ACL_OK;
  if (!F->adj || !F->gains || !F->gain_off)
    return acl__set_error("acl_tile_gains: required pointer is NULL");
  if (out == F->gains) return acl__set_error("acl_tile_gains: out aliases gains");
  const hipError_t e = launch_tile_gains(F->n, F->n_formations, F->adj, F->gains, F->gain_off,
                                         out, (hipStream_t)stream);
  if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  return ACL_OK;
}
