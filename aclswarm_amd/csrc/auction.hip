// auction.hip -- the LDS-resident batched auction for n <= 128 (gfx950).
//
// One workgroup (512 threads = 8 wave64) owns one swarm for the whole
// auction; every per-swarm table lives in LDS (51.4 KiB at n = 100: three
// swarms per CU -- 53 KiB did not fit three after allocation rounding):
//
//   phase 0  load p, the adjacency bits, P_in (permutation check), q in
//            formation order; vehicle-space closed neighbourhoods and their
//            the alignment work list
//   phase 1  2-D Umeyama alignment (Auctioneer::alignFormation,
//            auctioneer.cpp:347-415). A vehicle's alignment depends only on
//            its closed formation neighbourhood N[P[v]] (the formation-ordered
//            q is shared), so one alignment per distinct neighbourhood: every
//            row with an incomplete neighbourhood plus one row for all the
//            complete ones (all of them at config C2, ~45% of the rows at C3).
//            One lane per work item runs both of Eigen's sequential passes
//            (ascending members; the loads are broadcast, non-members are
//            masked out of the wave by exec, not by selects) and the 2x2
//            JacobiSVD finish in registers.
//   phase 2  price matrix C[v][j] = getPrice (auctioneer.cpp:546-549), fp64
//            math, f32 result; row n of C is the `none` entry's price 0
//   phase 3  CBAA rounds (auctioneer.cpp:182-306,469-542) on the `who` table
//            T (u8, vehicle rows; price of an entry = C[who][j]): per round
//            the dirty columns (a clean column is a fixed point of
//            updateTaskAssignment), one wave per column, lanes = vehicles.
//            A column is resolved level by level: the highest price level of
//            the column, its holders H (ballot) and `who`; vehicle v takes it
//            iff H meets N(v) (a per-lane mask test: vector work, since the
//            scalar unit is the kernel's busiest) and the next level it meets
//            is its runner-up (decision
//            margin). Ties, NaN and vehicles no tracked level resolves take
//            the exact ordered scan. Then outbid vehicles re-select
//            (selectTaskAssignment) as wave argmaxes. Exact fixed-point exit.
//   phase 4  adoption (isValidAssignment, auctioneer.cpp:250-295): one
//            permutation check when every table agrees, per vehicle otherwise
//
// Compiled with -ffp-contract=off: every f64 op is one IEEE rounding, so the
// alignment, prices, assignments and decision margins are bit-identical to
// the CPU restatement (oracle/). Per-lane booleans are SGPR lane masks
// (inverse_ballot / ballot convert at no VALU cost).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/aclswarm_amd.h"
#include "common.h"
#include "control_dev.h"
#include "control_params.h"
#include "pair_fused.h"
#include "umeyama_dev.h"

namespace acl_amd {

// threads per swarm (kernel template parameter kAB): 512 for n > 64, 256 for
// 32 < n <= 64, 128 for n <= 32 -- a small swarm leaves most of a 512-thread
// workgroup idle in every phase, and the CU holds more small swarms
#ifndef ACL_AUCTION_LEVELS
#define ACL_AUCTION_LEVELS 4   // price levels per dirty column before the exact scan
#endif
constexpr int kAL = ACL_AUCTION_LEVELS;

__host__ __device__ inline int a16(int x) { return (x + 15) & ~15; }

// LDS layout (byte offsets). C's region first holds the alignment inputs
// (pq, adjF, items: phases 0-1 only); region A (p, qf, out: phases 0-2) is
// overlaid by the who table T from phase 3 on.
struct ALayout {
  int C, pq, adjF, items;
  int A, p, qf, out;
  int T, TS;
  int vadj, Pin, Ptin, itm, valid, H, misc, dummy, W1, total;
};

__host__ __device__ inline ALayout make_alayout(int n) {
  ALayout L;
  int o = 0;
  L.TS = (n + 3) & ~3;  // T row stride: rows compare as dwords
  L.C = o;
  {
    const int csz = (n + 1) * n * 4;
    const int pre = a16((n + 8) * 32) + a16(n * 16) + a16(n);
    o = a16(o + (csz > pre ? csz : pre));
  }
  L.pq = L.C;                      // [n + 8] {p.x, p.y, qf.x, qf.y} f64 (padded)
  L.adjF = L.pq + a16((n + 8) * 32);  // [n][2] u64 formation rows (no diagonal)
  L.items = L.adjF + a16(n * 16);  // [n] u8 alignment work list (rows)
  L.A = o;
  L.p = o;    o = a16(o + n * 24);
  L.qf = o;   o = a16(o + n * 24);
  L.out = o;  o = a16(o + n * 48);   // R, t per work item
  L.T = L.A;
  if (L.A + n * L.TS > o) o = a16(L.A + n * L.TS);
  L.vadj = o;  o = a16(o + n * 16);  // [v][2] closed neighbourhood of vehicle v
  L.Pin = o;   o = a16(o + n);
  L.Ptin = o;  o = a16(o + n);
  L.itm = o;   o = a16(o + n);       // work item of formation row i
  L.valid = o; o = a16(o + n);
  L.H = o;     o = a16(o + 16 * 8);  // dmask[2][2], obm[2][2], seen[2]
  L.misc = o;  o = a16(o + 16 * 4);
  L.dummy = o; o = a16(o + 64);      // write-back target of the lanes past n
  L.W1 = o;    o = a16(o + n * 8);   // [n] u64 START argmax words (phase 2)
  L.total = o;
  return L;
}

enum { A_NITEMS = 2, A_RCH = 3 /* [2]: a column changed in a round of that parity */ };

// diagnostic builds (-DACL_AUCTION_STOP=k): the kernel returns after phase
// k, for per-phase instruction counts (scripts/auction_phase_pmc.sh)
#ifndef ACL_AUCTION_STOP
#define ACL_AUCTION_STOP 0
#endif
#define ACL_AUCTION_STOP_AT(k) \
  if (ACL_AUCTION_STOP == (k)) return

// the four doubles of pq[j] (broadcast LDS reads)
__device__ __forceinline__ void load4(const double* pq, int j, double (&v)[4]) {
  const double2 a = *reinterpret_cast<const double2*>(pq + 4 * j);
  const double2 c = *reinterpret_cast<const double2*>(pq + 4 * j + 2);
  v[0] = a.x; v[1] = a.y; v[2] = c.x; v[3] = c.y;
}

// For j = 0 .. n-1 in order: f(mask, pq[j]) with mask = the lanes whose
// neighbourhood bits r hold j. pq[j] is a broadcast read issued four terms
// ahead (a ring of four buffers: the reads' latency, not the adds, would
// otherwise set the pace of the sequential sums). pq is padded to n + 4
// entries; terms past n have an empty mask (exec = 0: no lane adds).
template <int NC, typename F>
__device__ __forceinline__ void for_members(int n, const double* pq,
                                            const unsigned long long (&r)[2], F&& f) {
  double R0[4], R1[4], R2[4], R3[4];
  load4(pq, 0, R0);
  load4(pq, 1, R1);
  load4(pq, 2, R2);
  load4(pq, 3, R3);
#pragma unroll 1
  for (int j = 0; j < n; j += 4) {
    const unsigned long long w = j < 64 ? r[0] : r[1];
    const unsigned long long bits = w >> (j & 63);  // j % 4 == 0: four bits in one word
    f(__ballot(bits & 1ull), R0);
    load4(pq, j + 4, R0);
    f(__ballot(bits & 2ull), R1);
    load4(pq, j + 5, R1);
    f(__ballot(bits & 4ull), R2);
    load4(pq, j + 6, R2);
    f(__ballot(bits & 8ull), R3);
    load4(pq, j + 7, R3);
  }
}

// diagnostic: s_memtime at phase ends (scripts/phase_profile.py)
__device__ __forceinline__ void stamp_phase(const SolveParams& P, int b, int tid, int k) {
  if (P.stamps && tid == 0) P.stamps[(size_t)b * kStampStride + k] = __builtin_amdgcn_s_memtime();
}
// diagnostic: the shared 100 MHz clock into slot k (kStampRt0 / kStampRt1)
__device__ __forceinline__ void stamp_rt(const SolveParams& P, int b, int tid, int k) {
  if (P.stamps && tid == 0) P.stamps[(size_t)b * kStampStride + k] = __builtin_amdgcn_s_memrealtime();
}

// diagnostic builds (-DACL_AUCTION_PROF=1): s_memtime cycles of the CBAA
// column step's sections, summed over a swarm's waves into
// stamps[b][kStampSec + 0..8]
// (scripts/phase_profile.py; each mark waits for the wave's LDS operations,
// so the split is indicative)
#ifndef ACL_AUCTION_PROF
#define ACL_AUCTION_PROF 0
#endif
enum { PS_L0, PS_LV, PS_MB, PS_WALK, PS_SCAN, PS_WB, PS_SEL, PS_BAR, PS_N };
struct SecProf {
  unsigned long long acc[PS_N], last;
  unsigned cols, walks, scans, sels, selx;
  __device__ void start() {
    if (ACL_AUCTION_PROF) {
      for (int k = 0; k < PS_N; ++k) acc[k] = 0;
      cols = walks = scans = sels = selx = 0;
      last = __builtin_amdgcn_s_memtime();
    }
  }
  __device__ void mark(int k) {
    if (ACL_AUCTION_PROF) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc[k] += t - last;
      last = t;
    }
  }
  __device__ void flush(const SolveParams& P, int b, int lane) {
    if (ACL_AUCTION_PROF && P.stamps && lane == 0) {
      unsigned long long* s = P.stamps + (size_t)b * kStampStride + kStampSec;
      for (int k = 0; k < PS_N; ++k) atomicAdd(s + k, acc[k]);
      atomicAdd(s + PS_N, (unsigned long long)cols | ((unsigned long long)walks << 12) |
                              ((unsigned long long)scans << 24) |
                              ((unsigned long long)sels << 36) | ((unsigned long long)selx << 48));
    }
  }
};

// diagnostic builds (-DACL_AUCTION_NO_MARGIN): the CBAA rounds skip the
// decision-margin bookkeeping (a cost measurement only; margins then wrong)
#ifndef ACL_AUCTION_NO_MARGIN
#define ACL_AUCTION_NO_MARGIN 0
#endif
// diagnostic builds: -DACL_AUCTION_NO_SELMARGIN=1 skips the selects' margin
// tracking, -DACL_AUCTION_NO_PUBLISH=1 the per-round publication of the
// waves' gaps (cost measurements only; margins then wrong)
#ifndef ACL_AUCTION_NO_SELMARGIN
#define ACL_AUCTION_NO_SELMARGIN 0
#endif
#ifndef ACL_AUCTION_NO_PUBLISH
#define ACL_AUCTION_NO_PUBLISH 0
#endif

// Column maxima (ACL_CBAA_COLMAX, default on): an entry's price never falls
// (updateTaskAssignment keeps the best of a closed neighbourhood that holds
// the vehicle itself; a select raises it), so a column's highest key is the
// highest bid ever placed in it -- kept per column in LDS by one atomic max per
// bid, it is the column's level 0 without a wave reduction.
#ifndef ACL_CBAA_COLMAX
#define ACL_CBAA_COLMAX 1
#endif
// Lazy per-round margin work (ACL_CBAA_LAZY, default on): a wave with no
// dirty column skips the walk bound, and a wave publishes its gap bound only
// after a round in which it evaluated something.
#ifndef ACL_CBAA_LAZY
#define ACL_CBAA_LAZY 1
#endif

// Waves that take CBAA round work (ACL_CBAA_WAVES, a power of two <= the
// workgroup's waves): the others only pass the round barriers, so the
// per-round bookkeeping (work distribution, margin publication) is paid by
// fewer waves while the CU's other swarms keep its SIMDs busy.
#ifndef ACL_CBAA_WAVES
#define ACL_CBAA_WAVES 8
#endif
// Rounds in which the waves publish their gap bounds (ACL_PUBLISH_ROUNDS,
// default all): later rounds prune against the last published value (an
// upper bound of the swarm's minimum, so every pruning decision stays valid).
#ifndef ACL_PUBLISH_ROUNDS
#define ACL_PUBLISH_ROUNDS 0x7fffffff
#endif

// An upper bound of margin_gap(hi, lo) in f32 for the mid-auction
// publications of the margin word (the walk bound's Gpub): (hi - lo) is exact
// in f32 when lo >= hi / 2 (Sterbenz), the approximate reciprocal is padded
// by 2^-20; otherwise the gap is above 1/2 and 1 bounds it. A published value
// at least the exact gap of a tracked pair keeps every pruning decision
// valid, and the exact gaps published at the end make the final minimum.
__device__ __forceinline__ float gap_ub(float hi, float lo) {
  const float g = (hi - lo) * __builtin_amdgcn_rcpf(hi) * (1.0f + 0x1p-20f);
  return lo >= 0.5f * hi ? fminf(g, 1.0f) : 1.0f;
}

// publish a wave's upper-bounded smallest gap (lanes' pairs m, the wave's
// uniform pair) into the margin word: one u32 wave minimum, one LDS atomic
__device__ __forceinline__ void publish_gap_ub(unsigned long long* margw, const MarginPair& m,
                                               float uhi, float ulo) {
  const float g = fminf(gap_ub(m.hi, m.lo), gap_ub(uhi, ulo));
  const unsigned w = ~wave_max_u32(~__float_as_uint(g));  // non-negative floats: bit order
  if ((threadIdx.x & 63) == 0)
    atomicMin(margw, (unsigned long long)__double_as_longlong((double)__uint_as_float(w)));
}

// margin_gap of a (hi, lo) pair (common.h margin_gap)
__device__ __forceinline__ double margin_gap_pair(float hi, float lo) {
  MarginPair m;
  m.hi = hi;
  m.lo = lo;
  return margin_gap(m);
}

// margin_track on a wave-uniform pair, branch-free (selects)
__device__ __forceinline__ void margin_track_u(float& hi, float& lo, float h, float l) {
  const bool tie = l == h;
  const bool up = l < h && (double)l * (double)hi > (double)lo * (double)h;
  hi = tie ? 1.0f : (up ? h : hi);
  lo = tie ? 1.0f : (up ? l : lo);
}

enum { FL_OB = 0, FL_DIRTY = 2, FL_CH = 4 };

__device__ __forceinline__ bool lanebit(unsigned long long m) {
  return __builtin_amdgcn_inverse_ballot_w64(m);
}

// the who-table entry of lane-vehicle row `row`, task j, and its price key
// (price bits + 1; `none` = row n of C has price 0 -> key 1)
__device__ __forceinline__ unsigned entry_key(const float* C, int n, int w, int j) {
  // (24-bit multiply: w, n <= 128; v_mul_lo_u32 is a quarter-rate instruction)
  return __float_as_uint(C[__umul24(w, n) + j]) + 1u;
}

// selectTaskAssignment (auctioneer.cpp:517-542) for vehicle v as a wave
// argmax over its row (lanes = tasks), with the margin of its decisive
// comparisons (include/aclswarm_amd.h). fresh: the START bid on an all-`none`
// row. Returns the selected task (wave-uniform) or -1.
template <int NC, bool MG>
__device__ __forceinline__ int wave_select(int n, int TS, int v, int lane, const float* C,
                                           const unsigned char* T, bool fresh, MarginPair& m,
                                           unsigned* selx = nullptr) {
  unsigned key[NC];
  float cv[NC], pr[NC];
  bool oth[NC];
  unsigned lm = 0u;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int j = lane + 64 * c;
    const bool ok = j < n;
    const int jj = ok ? j : 0;
    const int w = fresh ? n : T[v * TS + jj];
    cv[c] = C[v * n + jj];
    pr[c] = C[__umul24(w, n) + jj];
    key[c] = (ok && cv[c] > 0.0f && cv[c] > pr[c]) ? __float_as_uint(cv[c]) : 0u;
    oth[c] = ok && w != v;
    lm = lm > key[c] ? lm : key[c];
  }
  const unsigned M = wave_max_u32(lm);
  int js = -1;
  if (M != 0u) {
#pragma unroll
    for (int c = NC - 1; c >= 0; --c) {
      const unsigned long long e = __ballot(key[c] == M);
      if (e) js = 64 * c + __ffsll((long long)e) - 1;
    }
  }
  const float cmax = __uint_as_float(M);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    // the selected task vs its price (cv, pr); an eligible task that lost vs
    // the maximum (cmax, cv); a task that would win if it became eligible vs
    // its price (pr, cv). (A filter against the published gap -- every pair
    // with a gap <= G has cmax - cv <= G cmax or |cv - pr| <= G max(cv, pr)
    // -- passed 92% of the selects at C3: the selects' gaps set the margin.)
    if (ACL_AUCTION_PROF && selx) ++*selx;
    if (MG && !ACL_AUCTION_NO_SELMARGIN) {
      const int j = lane + 64 * c;
      const bool isjs = oth[c] && j == js;
      const bool elig = oth[c] && !isjs && key[c] != 0u;
      const bool near = oth[c] && !isjs && key[c] == 0u && cv[c] > 0.0f &&
                        (js < 0 || cv[c] > cmax || (cv[c] == cmax && j < js));
      margin_track_sel(m, isjs ? cv[c] : (elig ? cmax : pr[c]), isjs ? pr[c] : cv[c],
                       isjs || elig || near);
    }
  }
  return js;
}

// `who` of the first holder (lowest vehicle index) of a level
template <int NC>
__device__ __forceinline__ int first_who(const unsigned long long (&h)[NC], const int (&wu)[NC]) {
  int hl = 0, src = wu[0];
#pragma unroll
  for (int c = NC - 1; c >= 0; --c)
    if (h[c]) {
      hl = __ffsll((long long)h[c]) - 1;
      src = wu[c];
    }
  return __builtin_amdgcn_readlane(src, hl);
}

// the highest price key of the column below `cap` (0: none)
template <int NC>
__device__ __forceinline__ unsigned level_key(const unsigned (&key)[NC], unsigned cap) {
  unsigned x = 0u;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const unsigned y = key[c] < cap ? key[c] : 0u;
    x = x > y ? x : y;
  }
  return wave_max_u32(x);
}

// vehicles (lane masks of `open`) whose closed neighbourhood holds a level
// held by h
template <int NC>
__device__ __forceinline__ void level_hits(const unsigned long long (&open)[NC],
                                           const unsigned long long (&h)[NC],
                                           const unsigned long long (&vm)[NC][NC],
                                           unsigned long long (&hitm)[NC]) {
  // a per-lane mask test (no branches on the holder set)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    unsigned long long t = 0ull;
#pragma unroll
    for (int w = 0; w < NC; ++w) t |= vm[c][w] & h[w];
    hitm[c] = __ballot(t != 0ull) & open[c];
  }
}

// The exact decision gaps of a column's level-resolved vehicles (k1 != 0):
// walk the levels again; a vehicle's runner-up is the first level below its
// winning level that its neighbourhood holds. The largest ratio among the
// vehicles that meet their runner-up at a level belongs to the lowest winning
// level among them (wave minimum of k1), tracked into the wave's pair.
template <int NC>
__device__ __forceinline__ void runner_up_walk(int n, const unsigned (&key)[NC],
                                               const unsigned (&k1)[NC],
                                               const unsigned long long (&Nd)[NC],
                                               const unsigned long long (&vm)[NC][NC],
                                               float& uhi, float& ulo) {
  unsigned long long D[NC];  // resolved by a level, runner-up not met yet
#pragma unroll
  for (int c = 0; c < NC; ++c) D[c] = __ballot(k1[c] != 0u) & ~Nd[c];
  unsigned cap = 0xFFFFFFFFu;
  int cum = 0;
  for (int k = 0; k < 2 * kMaxN + 2; ++k) {
    unsigned long long any = 0ull;
#pragma unroll
    for (int c = 0; c < NC; ++c) any |= D[c];
    if (!any || cum >= n) break;
    const unsigned Mk = level_key<NC>(key, cap);
    if (Mk == 0u) break;
    unsigned long long h[NC], open[NC], hitm[NC];
    int nh = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      h[c] = __ballot(key[c] == Mk);
      nh += __popcll(h[c]);
      open[c] = D[c] & __ballot(k1[c] > Mk);  // only below the winning level
    }
    cum += nh;
    level_hits<NC>(open, h, vm, hitm);
    unsigned lowest = 0u;  // ~min k1 over the vehicles meeting it here
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const unsigned x = lanebit(hitm[c]) ? ~k1[c] : 0u;
      lowest = lowest > x ? lowest : x;
      D[c] &= ~hitm[c];
    }
    lowest = wave_max_u32(lowest);
    if (lowest != 0u)
      margin_track_u(uhi, ulo, __uint_as_float(~lowest - 1u), __uint_as_float(Mk - 1u));
    cap = Mk;
  }
}

// ---- phase 1 as its own launch (align_kernel) --------------------------------
// The alignment is a chain of ~2n dependent sums per work item, ~55 items per
// swarm at C3: inside the auction workgroup it ran on one wave while the
// swarm's other seven waited at the barrier, for a fifth of the swarm's life.
// align_kernel gives each swarm one wave (LDS ~6 KB: many swarms per CU) and
// leaves, per swarm, the work items' (R, t), the item of every formation row
// and the smallest alignment gap in the workspace (WsLayout::align); the
// auction kernel reads them back. The arithmetic is the same code in the
// same order (bit-identical R, t).
struct AlignLayout {
  int pq, adjF, items, itm, Pin, seen, misc, total;
};
__host__ __device__ inline AlignLayout make_align_layout(int n) {
  AlignLayout L;
  int o = 0;
  L.pq = o;    o = a16(o + (n + 8) * 32);  // {p.x, p.y, qf.x, qf.y} per point (padded)
  L.adjF = o;  o = a16(o + n * 16);        // [n][2] formation rows (no diagonal)
  L.items = o; o = a16(o + n);
  L.itm = o;   o = a16(o + n);
  L.Pin = o;   o = a16(o + n);
  L.seen = o;  o = a16(o + 16);
  L.misc = o;  o = a16(o + 16);
  L.total = o;
  return L;
}

// The alignment work list (one wave): formation rows with an incomplete
// closed neighbourhood ascending, then one row standing for every complete
// one; itm[i] = the item of row i. Returns the item count.
template <int NC>
__device__ __forceinline__ int align_worklist(int n, const unsigned long long* adjF,
                                              unsigned char* items, unsigned char* itm, int lane) {
  unsigned long long cm[NC], im[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + 64 * c;
    bool comp = false;
    if (i < n) {
      unsigned long long r0 = adjF[2 * i], r1 = adjF[2 * i + 1];
      if (i < 64) r0 |= 1ull << i; else r1 |= 1ull << (i - 64);
      comp = (__popcll(r0) + __popcll(r1)) == n;
    }
    cm[c] = __ballot(comp);
    im[c] = __ballot(i < n && !comp);
  }
  int rep = -1;
#pragma unroll
  for (int c = NC - 1; c >= 0; --c)
    if (cm[c]) rep = 64 * c + __ffsll((long long)cm[c]) - 1;
  int ninc = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) ninc += __popcll(im[c]);
  int base = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + 64 * c;
    const int rk = base + (int)__builtin_amdgcn_mbcnt_hi(
                              (unsigned)(im[c] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)im[c], 0u));
    if (lanebit(im[c])) {
      items[rk] = (unsigned char)i;
      itm[i] = (unsigned char)rk;
    } else if (lanebit(cm[c])) {
      itm[i] = (unsigned char)ninc;
    }
    base += __popcll(im[c]);
  }
  if (rep >= 0 && lane == 0) items[ninc] = (unsigned char)rep;
  return ninc + (rep >= 0 ? 1 : 0);
}

// Eigen::umeyama (3.3.x) for work items k0 + lane (one wave, one lane per
// item): pass 1 rowwise sums of src (p) and dst (qf) over the members in
// ascending order, pass 2 sigma = one_over_n * dst_demean * src_demean^T --
// the lazy product (scaled lhs, from the first term) when k + 4 < 20, else
// the GEMM form (0.0 + every term, alpha after). A sum starts at -0.0, the
// identity of IEEE addition (x + -0.0 = x for every x), which is the
// first-element start exactly. The members' values are broadcast loads; a
// lane adds a term only for its members (exec-masked: asm keeps the compiler
// from turning it into selects). (R, t) of item k to out[6k]; galign takes
// the smallest decision gap.
template <int NC>
__device__ __forceinline__ void align_chunk(int n, const double* pq, const unsigned long long* adjF,
                                            const unsigned char* items, int nitems, int k0,
                                            int lane, double* out, double& galign) {
  const int k = k0 + lane;
  const bool act = k < nitems;
  const int i = act ? items[k] : 0;
  unsigned long long r[2] = {adjF[2 * i], adjF[2 * i + 1]};
  if (i < 64) r[0] |= 1ull << i; else r[1] |= 1ull << (i - 64);
  if (!act) r[0] = r[1] = 0ull;
  const int cnt = __popcll(r[0]) + __popcll(r[1]);
  double s0 = -0.0, s1 = -0.0, s2 = -0.0, s3 = -0.0;
  for_members<NC>(n, pq, r, [&](unsigned long long mk, const double (&v)[4]) {
    masked_add4(mk, s0, s1, s2, s3, v[0], v[1], v[2], v[3]);
  });
  const double oon = 1.0 / (double)(act ? cnt : 1);
  const double sm0 = s0 * oon, sm1 = s1 * oon, dm0 = s2 * oon, dm1 = s3 * oon;
  const bool lazy = (cnt + 4) < 20;
  const double scale = lazy ? oon : 1.0;  // 1.0 * x == x
  const double a0 = lazy ? -0.0 : 0.0;
  double a00 = a0, a01 = a0, a10 = a0, a11 = a0;  // a(di, sj)
  if (__any(act && lazy)) {
    for_members<NC>(n, pq, r, [&](unsigned long long mk, const double (&v)[4]) {
      const double e0 = v[0] - sm0, e1 = v[1] - sm1;
      const double d0 = scale * (v[2] - dm0), d1 = scale * (v[3] - dm1);
      masked_add4(mk, a00, a01, a10, a11, d0 * e0, d0 * e1, d1 * e0, d1 * e1);
    });
  } else {  // every item in the GEMM form: scale is 1.0 and 1.0 * x == x
    for_members<NC>(n, pq, r, [&](unsigned long long mk, const double (&v)[4]) {
      const double e0 = v[0] - sm0, e1 = v[1] - sm1;
      const double d0 = v[2] - dm0, d1 = v[3] - dm1;
      masked_add4(mk, a00, a01, a10, a11, d0 * e0, d0 * e1, d1 * e0, d1 * e1);
    });
  }
  if (act) {
    // column-major sigma S(di, sj)
    const double S[4] = {lazy ? a00 : a00 * oon, lazy ? a10 : a10 * oon,
                         lazy ? a01 : a01 * oon, lazy ? a11 : a11 * oon};
    const double sm[2] = {sm0, sm1}, dm[2] = {dm0, dm1};
    double R[4], t[2], g;
    umeyama_finish(S, sm, dm, R, t, &g);
    galign = g < galign ? g : galign;
    double* o = out + 6 * k;
    o[0] = R[0]; o[1] = R[1]; o[2] = R[2]; o[3] = R[3]; o[4] = t[0]; o[5] = t[1];
  }
}

template <int NC>
#ifndef ACL_ALIGN_OCC
#define ACL_ALIGN_OCC 1  // min waves per SIMD align_kernel is built for (1: the compiler's choice)
#endif
__global__ void __launch_bounds__(64, ACL_ALIGN_OCC) align_kernel(const SolveParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const AlignLayout L = make_align_layout(n);
  const int b = P.b0 + blockIdx.x;
  const int lane = threadIdx.x;
  double* pq = reinterpret_cast<double*>(smem + L.pq);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adjF);
  unsigned char* items = smem + L.items;
  unsigned char* itm = smem + L.itm;
  unsigned long long* seen = reinterpret_cast<unsigned long long*>(smem + L.seen);
  int* misc = reinterpret_cast<int*>(smem + L.misc);
  const int f_in = P.fidx[b];
  if (f_in < 0 || f_in >= P.F) return;  // BAD_INPUT: the auction kernel reads nothing
  const int f = f_in;
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  const double* gp = P.p + (size_t)f * n * 3;
  const uint64_t* ga = P.adj + (size_t)f * n * NC;
  if (lane < 2) seen[lane] = 0ull;
  if (lane == 0) misc[0] = 0;
  for (int k = lane; k < 4 * (n + 8); k += 64) pq[k] = 0.0;
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  for (int j = lane; j < n; j += 64) {
    pq[4 * j] = gp[3 * j];
    pq[4 * j + 1] = gp[3 * j + 1];
  }
  for (int k = lane; k < 2 * n; k += 64) {
    const int i = k >> 1, w = k & 1;
    unsigned long long x = 0ull;
    if (w < NC) {
      x = ga[(size_t)i * NC + w];
      if (w == NC - 1) x &= lastmask;
    }
    adjF[k] = x;
  }
  // the permutation check and q in formation order: qf[P_in[v]] = q[v]
  for (int v = lane; v < n; v += 64) {
    const unsigned pv = P.P_in[(size_t)b * n + v];
    if (pv >= (unsigned)n) {
      misc[0] = 1;
    } else {
      const unsigned long long bit = 1ull << (pv & 63);
      if (atomicOr(&seen[pv >> 6], bit) & bit) misc[0] = 1;
      const double* qv = P.q + ((size_t)b * n + v) * 3;
      pq[4 * pv + 2] = qv[0];
      pq[4 * pv + 3] = qv[1];
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (misc[0]) return;  // not a permutation: BAD_INPUT (wave-uniform)
  const int nitems = align_worklist<NC>(n, adjF, items, itm, lane);
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  unsigned char* wsa = P.ws + P.W.align + (size_t)b * P.W.align_stride;
  double* gout = reinterpret_cast<double*>(wsa);
  double galign = 1.0;
  for (int k0 = 0; k0 < nitems; k0 += 64) align_chunk<NC>(n, pq, adjF, items, nitems, k0, lane, gout, galign);
  // the swarm's smallest alignment gap, the item of every row, the count
  const unsigned long long gb =
      ~wave_max_u64(~(unsigned long long)__double_as_longlong(galign));  // wave minimum
  unsigned char* gitm = wsa + (size_t)n * 48;
  for (int i = lane; i < n; i += 64) gitm[i] = itm[i];
  if (lane == 0) {
    *reinterpret_cast<unsigned long long*>(wsa + (size_t)n * 48 + a16(n)) = gb;
    *reinterpret_cast<int*>(wsa + (size_t)n * 48 + a16(n) + 8) = nitems;
  }
}

// FUSE: phase 5, the control law of a swarm whose vehicles all adopted one
// assignment, runs in this workgroup right after its auction (see below);
// GM: the fused phase also reports the gate margin.
// A/B knobs: the control phase's wave issue priority (s_setprio 0-3), and
// the CBAA phase's (set at the kernel's start, lowered again for control)
#ifndef ACL_CTL_PRIO
#define ACL_CTL_PRIO 0
#endif
#ifndef ACL_CBAA_PRIO
#define ACL_CBAA_PRIO 0
#endif
#ifndef ACL_AUCTION_OCC_SMALL
#define ACL_AUCTION_OCC_SMALL 6  // waves per SIMD the 128-thread (n <= 32) instantiation is built for
#endif
template <int NC, int kAB, bool FUSE, bool GM, bool MG>
__global__ void __launch_bounds__(kAB, kAB == 128 ? ACL_AUCTION_OCC_SMALL : 6)
    auction_kernel(const SolveParams P) {
  constexpr int kAW = kAB / 64;  // waves per swarm
  constexpr int kCW = kAW < ACL_CBAA_WAVES ? kAW : ACL_CBAA_WAVES;  // CBAA round waves
  static_assert((kCW & (kCW - 1)) == 0, "ACL_CBAA_WAVES: a power of two");
  // the CBAA rounds' decision-margin work (MG false: skip_margin)
  constexpr bool kMarg = MG && !ACL_AUCTION_NO_MARGIN;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const ALayout L = make_alayout(n);
  const int TS = L.TS;
  const int b = P.b0 + blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // n <= 64 (kAB <= 256): the alignment stays in this workgroup (an extra
  // launch costs the launch-bound small configurations more than it saves)
  constexpr bool kInlineAlign = kAB <= 256;
  float* C = reinterpret_cast<float*>(smem + L.C);
  double* pq = reinterpret_cast<double*>(smem + L.pq);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adjF);
  unsigned char* items = smem + L.items;
  double* p = reinterpret_cast<double*>(smem + L.p);
  double* qf = reinterpret_cast<double*>(smem + L.qf);
  double* out = reinterpret_cast<double*>(smem + L.out);
  unsigned char* T = smem + L.T;
  unsigned long long* vadj = reinterpret_cast<unsigned long long*>(smem + L.vadj);
  unsigned char* Pin = smem + L.Pin;
  unsigned char* Ptin = smem + L.Ptin;
  unsigned char* itm = smem + L.itm;
  unsigned char* validv = smem + L.valid;
  unsigned long long* H = reinterpret_cast<unsigned long long*>(smem + L.H);
  int* misc = reinterpret_cast<int*>(smem + L.misc);
  unsigned long long* margw = reinterpret_cast<unsigned long long*>(misc + M_MARG);
  unsigned long long* W1 = reinterpret_cast<unsigned long long*>(smem + L.W1);
  // [n] u32 column maxima (ACL_CBAA_COLMAX): overlays vadj, dead once every
  // thread has its neighbourhood masks in registers (the price-phase barrier)
  unsigned* cmax = reinterpret_cast<unsigned*>(smem + L.vadj);

  // a formation index out of range is a bad input like a bad P_in (nothing
  // of the formation table is read for it)
  const int f_in = P.fidx[b];
  const bool fbad = f_in < 0 || f_in >= P.F;
  const int f = fbad ? 0 : f_in;
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  // the vehicles hold their own assignments (acl_solve_args_t::P_rows)
  const bool rowsm = P.P_rows != nullptr && P.P_rows_on[b] != 0;  // workgroup-uniform
  MarginPair mp;
  margin_init(mp);
  stamp_phase(P, b, tid, 0);
  stamp_rt(P, b, tid, kStampRt0);

  // ---------------- phase 0: load ------------------------------------------
  // Every global read of the phase is issued up front (one HBM round trip,
  // not three): thread v < n (n <= kAB) holds P_in[v] and q[v] in registers
  // until the permutation check can run.
  const bool hv = tid < n;
  bool pbad = false;  // a formation coordinate is not finite (phase 2's fast path)
  unsigned pvr = 0u;
  double qx = 0.0, qy = 0.0, qz = 0.0;
  if (hv) {
    pvr = P.P_in[(size_t)b * n + tid];
    const double* qv = P.q + ((size_t)b * n + tid) * 3;
    qx = qv[0]; qy = qv[1]; qz = qv[2];
  }
  {
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += kAB) {
      const double x = gp[k];
      pbad |= !__builtin_isfinite(x);
      p[k] = x;
      const int j = k / 3, comp = k - 3 * j;
      if (kInlineAlign && comp < 2) pq[4 * j + comp] = x;  // pq[j] = {p_j.xy, qf_j.xy}
    }
    const uint64_t* ga = P.adj + (size_t)f * n * NC;
    for (int k = tid; k < 2 * n; k += kAB) {
      const int i = k >> 1, w = k & 1;
      unsigned long long x = 0ull;
      if (w < NC) {
        x = ga[(size_t)i * NC + w];
        if (w == NC - 1) x &= lastmask;
      }
      adjF[k] = x;
    }
    if (tid < 16) {
      misc[tid] = 0;
      H[tid] = 0ull;
    }
    if (tid < n) W1[tid] = 0ull;
  }
  // the alignment launch's results (align_kernel: every work item's (R, t),
  // the item of every formation row, the swarm's smallest alignment gap) in
  // the same round trip: all 6n doubles of the item region are read (items
  // past the count are never used), so no read waits for the item count
  unsigned long long agap = 0ull;
#ifndef ACL_ALIGN_PREFETCH
#define ACL_ALIGN_PREFETCH 1
#endif
  if (ACL_ALIGN_PREFETCH && !kInlineAlign && !rowsm) {
    const unsigned char* wsa = P.ws + P.W.align + (size_t)b * P.W.align_stride;
    const double* gout = reinterpret_cast<const double*>(wsa);
    for (int k = tid; k < 6 * n; k += kAB) out[k] = gout[k];
    for (int i = tid; i < n; i += kAB) itm[i] = wsa[(size_t)n * 48 + i];
    if (tid == 0) agap = *reinterpret_cast<const unsigned long long*>(wsa + (size_t)n * 48 + a16(n));
  }
  __syncthreads();
  if (tid == 0) {
    misc[M_AGREE] = 1;
    if (fbad) misc[M_BAD] = 1;
    *margw = (unsigned long long)__double_as_longlong(1.0);
  }
  if (__any(pbad) && lane == 0) misc[M_PINF] = 1;
  if (hv) {
    // the permutation check; q in formation order: qf[P_in[v]] = q[v]
    const int v = tid;
    const unsigned pv = pvr;
    Pin[v] = (unsigned char)pv;
    if (pv >= (unsigned)n) {
      misc[M_BAD] = 1;
    } else {
      const unsigned long long bit = 1ull << (pv & 63);
      if (atomicOr(&H[8 + (pv >> 6)], bit) & bit) misc[M_BAD] = 1;  // not a permutation
      Ptin[pv] = (unsigned char)v;
      qf[3 * pv] = qx; qf[3 * pv + 1] = qy; qf[3 * pv + 2] = qz;
      if (kInlineAlign) {
        pq[4 * pv + 2] = qx;
        pq[4 * pv + 3] = qy;
      }
    }
  }
  __syncthreads();
  // (M_BAD is final here: the own-row checks below report into M_ROWBAD, so
  // no wave's entry test sees another wave's write and the barrier inside
  // stays workgroup-uniform)
  if (rowsm && !misc[M_BAD]) {
    // each vehicle's own row: checked, its neighbourhood mask and its
    // alignment (thread v; align_own_row), the alignment at out[Pin[v]] with
    // itm the identity, so the price phase reads it as a row's item
    double galign = 1.0;
    if (hv) {
      const int v = tid, i = Pin[v];
      const uint16_t* row = P.P_rows + ((size_t)b * n + v) * n;
      unsigned long long nbm[2];
      const bool ok = align_own_row<2>(
          n, NC, v, i, adjF + 2 * i, p, [&](int j) { return (int)row[j]; },
          [&](int u, double& x, double& y) {
            x = qf[3 * Pin[u]];
            y = qf[3 * Pin[u] + 1];
          },
          nbm, out + 6 * i, galign);
      if (!ok) misc[M_ROWBAD] = 1;
      vadj[2 * v] = nbm[0];
      vadj[2 * v + 1] = nbm[1];
    }
    for (int i = tid; i < n; i += kAB) itm[i] = (unsigned char)i;
    block_min_gap(margw, galign);
    __syncthreads();
  }
  if (misc[M_BAD] | misc[M_ROWBAD]) {
    // P_in is not a permutation (or fidx is out of range): nothing is solved
    for (int v = tid; v < n; v += kAB) {
      P.P_out[(size_t)b * n + v] = P.P_in[(size_t)b * n + v];
      if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = 0;
    }
    for (int k = tid; k < 3 * n; k += kAB) {
      if (P.u) P.u[(size_t)b * n * 3 + k] = 0.0;
      if (P.u_safe) P.u_safe[(size_t)b * n * 3 + k] = 0.0;
    }
    if (P.who)
      for (int k = tid; k < n * n; k += kAB) P.who[(size_t)b * n * n + k] = 0xFFFF;
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
  // closed neighbourhoods in vehicle space (bidIterComplete, auctioneer.cpp:
  // 419-437): u ~ v iff u == v or adj(P[v], P[u]) (rows: built above)
  if (!rowsm) {
    int pu[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) pu[c] = (lane + 64 * c < n) ? Pin[lane + 64 * c] : 0;
    for (int v = wave; v < n; v += kAW) {
      const int i = Pin[v];
      const unsigned long long r0 = adjF[2 * i], r1 = adjF[2 * i + 1];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int u = lane + 64 * c;
        const bool okl = u < n;
        const bool e = okl && (u == v || (((pu[c] < 64 ? r0 : r1) >> (pu[c] & 63)) & 1ull));
        const unsigned long long me = __ballot(e);
        if (lane == 0) vadj[2 * v + c] = me;
      }
      if (NC == 1 && lane == 0) vadj[2 * v + 1] = 0ull;
    }
  }
  if (kInlineAlign && wave == 0 && !rowsm) {
    const int ni = align_worklist<NC>(n, adjF, items, itm, lane);
    if (lane == 0) misc[A_NITEMS] = ni;
  }
  __syncthreads();
  stamp_phase(P, b, tid, 1);
  ACL_AUCTION_STOP_AT(1);

  // ---------------- phase 1: alignment (align_kernel's results) -------------
  // Auctioneer::alignFormation per distinct neighbourhood (auctioneer.cpp:
  // 347-415) ran in align_kernel: read back the items' (R, t), the item of
  // every formation row and the swarm's smallest alignment gap
  if (rowsm) {
    // (the own-row alignments are in out already)
  } else if constexpr (kInlineAlign) {
    const int nitems = misc[A_NITEMS];
    double galign = 1.0;
    if (wave * 64 < nitems) align_chunk<NC>(n, pq, adjF, items, nitems, wave * 64, lane, out, galign);
    // the alignments' gaps go into the swarm margin now: the CBAA rounds
    // prune their margin work against it (below)
    block_min_gap(margw, galign);
  } else if (ACL_ALIGN_PREFETCH) {
    // (out and itm were filled in phase 0)
    if (tid == 0) atomicMin(margw, agap);
  } else {
    const unsigned char* wsa = P.ws + P.W.align + (size_t)b * P.W.align_stride;
    const int nitems = *reinterpret_cast<const int*>(wsa + (size_t)n * 48 + a16(n) + 8);
    const double* gout = reinterpret_cast<const double*>(wsa);
    for (int k = tid; k < 6 * nitems; k += kAB) out[k] = gout[k];
    for (int i = tid; i < n; i += kAB) itm[i] = wsa[(size_t)n * 48 + i];
    if (tid == 0)
      atomicMin(margw, *reinterpret_cast<const unsigned long long*>(wsa + (size_t)n * 48 + a16(n)));
  }
  __syncthreads();
  stamp_phase(P, b, tid, 2);
  ACL_AUCTION_STOP_AT(2);
  if (P.align_Rt)
    for (int k = tid; k < 6 * n; k += kAB) {
      const int v = k / 6;
      P.align_Rt[(size_t)b * n * 6 + k] = out[6 * itm[Pin[v]] + (k - 6 * v)];
    }

  // ---------------- phase 2: prices and the START bids ---------------------
  // A thread per (vehicle v, task class j0): v = tid % n, tasks j = j0, j0 +
  // per, ... ascending. The thread keeps v's alignment and q in registers and
  // tracks, over its tasks, the START select (start, auctioneer.cpp:105 ->
  // selectTaskAssignment :517-542 on the all-`none` table: the first task of
  // the largest price > 0) and the runner-up price, so the START bids need no
  // pass over the price matrix: the per-vehicle winner is one LDS atomic max
  // over the `per` threads' (price, task) words (ties to the lowest task),
  // the runner-up a second one over what each thread saw besides the winner.
  // (The select's decision margin is its closest eligible loser: the
  // runner-up -- a tie is a runner-up equal to the winner.)
  unsigned* W2 = reinterpret_cast<unsigned*>(C + n * n);  // the `none` row, borrowed
  const int per = kAB / n;
  const int pv = tid % n, j0 = tid / n;
  const bool pact = j0 < per;
  float pbest = 0.0f, psec = 0.0f;
  int pbj = -1;
  {
    int nonfin = 0;
    // The aligned point is Eigen's 3x3 [R 0; 0 1] times p plus [t; 0]. With
    // every coordinate of p finite, the terms 0 * p are signed zeros: they
    // can change only the sign of a zero component of the aligned point, and
    // every component enters the price squared, so dropping them leaves the
    // price bit-identical (a non-finite p keeps the full expression: 0 * inf
    // is NaN).
    const bool pfin = misc[M_PINF] == 0;  // workgroup-uniform
    const int ip = Pin[pv];
    const double* o = out + 6 * itm[ip];
    const double* qv = qf + 3 * ip;
    const double o0 = o[0], o1 = o[1], o2 = o[2], o3 = o[3], o4 = o[4], o5 = o[5];
    const double q0 = qv[0], q1 = qv[1], q2 = qv[2];
    float* Crow = C + pv * n;
    for (int j = j0; pact && j < n; j += per) {
      const double px = p[3 * j], py = p[3 * j + 1], pz = p[3 * j + 2];
      double dx, dy, dz;
      if (pfin) {
        dx = q0 - ((o0 * px + o1 * py) + o4);
        dy = q1 - ((o2 * px + o3 * py) + o5);
        dz = q2 - pz;
      } else {
        const double ax = ((o0 * px + o1 * py) + 0.0 * pz) + o4;
        const double ay = ((o2 * px + o3 * py) + 0.0 * pz) + o5;
        const double az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0;
        dx = q0 - ax; dy = q1 - ay; dz = q2 - az;
      }
      const float c = acl_price((dx * dx + dy * dy) + dz * dz);  // bit-exact, see common.h
      Crow[j] = c;
      nonfin |= (c != c);
      // strict > from max = 0 (NaN never wins, never becomes the runner-up)
      const bool gt = c > pbest;
      psec = gt ? pbest : (c > psec ? c : psec);
      pbj = gt ? j : pbj;
      pbest = gt ? c : pbest;
    }
    if (pact && pbj >= 0)
      atomicMax(&W1[pv], ((unsigned long long)__float_as_uint(pbest) << 8) |
                             (unsigned long long)(255 - pbj));
    if (__any(nonfin) && lane == 0) misc[M_NONFIN] = 1;
    for (int jj = tid; jj < n; jj += kAB) W2[jj] = 0u;  // (the `none` row: zeros again below)
  }
  // per-lane neighbourhood masks of this lane's vehicles (lane + 64 c)
  unsigned long long vm[NC][NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int v = lane + 64 * c;
#pragma unroll
    for (int w = 0; w < NC; ++w) vm[c][w] = (v < n) ? vadj[2 * v + w] : 0ull;
  }
  __syncthreads();  // region A (p, qf, out) is dead from here: T overlays it
  const bool nonfinite = misc[M_NONFIN] != 0;
  stamp_phase(P, b, tid, 3);
  ACL_AUCTION_STOP_AT(3);

  // ---------------- START bids ----------------------------------------------
  unsigned long long* dmask = H;      // [2 parities][2 words]
  unsigned long long* obm = H + 4;    // [2][2]
  {
    // every table row `none` (reset, auctioneer.cpp:448-465); each thread's
    // runner-up candidate: its best unless that is the winner, else its second
    const unsigned fill = (unsigned)n * 0x01010101u;
    unsigned* T32 = reinterpret_cast<unsigned*>(T);
    for (int k = tid; k < n * (TS / 4); k += kAB) T32[k] = fill;
    if (ACL_CBAA_COLMAX)
      for (int jj = tid; jj < n; jj += kAB) cmax[jj] = 1u;  // the `none` key
    if (pact && pbj >= 0) {
      const int js = 255 - (int)(W1[pv] & 255ull);
      const float cand = pbj == js ? psec : pbest;
      if (cand > 0.0f) atomicMax(&W2[pv], __float_as_uint(cand));
    }
  }
  __syncthreads();
  if (tid < n) {
    const int v = tid;
    const unsigned long long w = W1[v];
    const unsigned sec = W2[v];
    W2[v] = 0u;  // the `none` row's price 0 again
    if (w) {
      const int js = 255 - (int)(w & 255ull);
      T[v * TS + js] = (unsigned char)v;
      atomicOr(&dmask[2 + (js >> 6)], 1ull << (js & 63));
      if (ACL_CBAA_COLMAX) atomicMax(&cmax[js], (unsigned)(w >> 8) + 1u);
      // the select's decision gaps (wave_select's terms on a fresh row): the
      // winner against its price 0 (gap 1), every eligible loser against the
      // winner -- the closest is the runner-up
      if (MG && sec) margin_track(mp, __uint_as_float((unsigned)(w >> 8)), __uint_as_float(sec));
    }
  }
  // the START selects' gaps, published for round 1's walk bound
  if (MG && !ACL_AUCTION_NO_PUBLISH) publish_gap_ub(margw, mp, 1.0f, 0.0f);
  __syncthreads();
  ACL_AUCTION_STOP_AT(4);

  // ---------------- phase 3: CBAA -------------------------------------------
  if (ACL_CBAA_PRIO) __builtin_amdgcn_s_setprio(ACL_CBAA_PRIO);
  bool okv[NC];
  unsigned long long okm[NC];
  unsigned okk[NC];  // key mask: all ones for real vehicles, 0 past n
  int rowa[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    okv[c] = lane + 64 * c < n;
    okm[c] = __ballot(okv[c]);
    okk[c] = okv[c] ? 0xFFFFFFFFu : 0u;
    rowa[c] = (okv[c] ? lane + 64 * c : 0) * TS;
  }
  // the wave's uniform margin pair over the level-resolved evaluations
  float uhi = 1.0f, ulo = 0.0f;
  int eff = 0;
  // per-lane flags (FL_*) published once per wave and phase instead of
  // atomics per column and per re-select: FL_OB << c = vehicle lane + 64 c
  // outbid, FL_DIRTY << w = column 64 w + lane dirty next round, FL_CH = a
  // column changed this round
  // (wave-uniform 64-bit masks instead, with the outbid and dirty terms on
  // the scalar unit, spilled ~60 scalar registers to VGPR lanes: 360 more
  // vector instructions in the loop)
  unsigned fl = 0u;
  bool evald = false;  // the wave evaluated a column or a select since it last published
  SecProf sp;
  sp.start();
  const int max_rounds = 2 * n;  // cbaa_max_iter_ = n * diameter (:50-51)
  for (int r = 1; r <= max_rounds; ++r) {
    const int par = r & 1, npar = par ^ 1;
    // the swarm's smallest gap published so far (alignments, and every
    // wave's evaluations up to the last round): an evaluation whose gap is
    // bounded below by it cannot lower the margin, so its runner-up walk is
    // skipped (margin_gap is monotone in the pair's ratio)
    // this wave's dirty columns: every 8th set bit in rank order
    const bool cw = wave < kCW;  // this wave takes round work (wave-uniform)
    unsigned long long mine[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) mine[c] = 0ull;
    if (cw) {
      int base = 0;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const unsigned long long D = uni_u64(dmask[2 * par + c]);
        const int rk = base + (int)__builtin_amdgcn_mbcnt_hi(
                                  (unsigned)(D >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)D, 0u));
        mine[c] = __ballot(((D >> lane) & 1ull) && (rk & (kCW - 1)) == wave);
        base += __popcll(D);
      }
    }
    unsigned long long anymine = 0ull;
#pragma unroll
    for (int c = 0; c < NC; ++c) anymine |= mine[c];
    if (anymine) evald = true;
    if (!ACL_CBAA_LAZY || anymine) {
    const double Gpub = __longlong_as_double((long long)*margw);
    // the walk bound: a column's exact runner-up walk can lower the margin
    // only if some resolving level's successor is within Gw of it, Gw = min
    // (the published gap, the wave's own running gap); Gwf its float bound
    // for the conservative f32 tests (at least Gw (1 + 2^-20)), refreshed after walks
    double Gw = fmin(Gpub, margin_gap_pair(uhi, ulo));
    float Gwf = (float)(Gw * (1.0 + 0x1p-20));
    // 1 - Gw (1 + 2^-20) as a float one ulp below its rounding (a lower
    // bound), 0 when not positive: the successor test's factor (below)
    auto gfac = [](double gw) {
      const double x = 1.0 - gw * (1.0 + 0x1p-20);
      return x > 0.0 ? __uint_as_float(__float_as_uint((float)x) - 1u) : 0.0f;
    };
    float Gfacf = gfac(Gw);
    {
      // one loop over both words (the column body is emitted once)
      unsigned long long mm = mine[0], m1 = NC > 1 ? mine[NC - 1] : 0ull;
      int jb = 0;
      for (;;) {
        if (!mm) {
          if (!m1) break;
          mm = m1;
          m1 = 0ull;
          jb = 64;
        }
        const int j = jb + __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        // one wave per dirty column, lanes = vehicles
        int wu[NC], nw[NC];
        unsigned key[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          // every lane reads (rows clamped, who <= n): no exec masking
          wu[c] = T[rowa[c] + j];
          key[c] = entry_key(C, n, wu[c], j) & okk[c];
          nw[c] = wu[c];
        }
        // level 0: the column's highest price key, its holders and `who`
        const unsigned M0 = ACL_CBAA_COLMAX
                                ? (unsigned)__builtin_amdgcn_readfirstlane((int)cmax[j])
                                : level_key<NC>(key, 0xFFFFFFFFu);
        unsigned long long h[NC];
        int cum = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          h[c] = __ballot(key[c] == M0);
          cum += __popcll(h[c]);
        }
        int wk = first_who<NC>(h, wu);
        unsigned long long tie = 0ull;
#pragma unroll
        for (int c = 0; c < NC; ++c) tie |= h[c] & __ballot(wu[c] != wk);
        if (ACL_AUCTION_PROF) sp.cols++;
#ifdef ACL_CAL_VALU
        // calibration builds: 20 independent VALU (or SALU) instructions per column
        { int dmy; asm volatile(".rept 20\n\tv_mov_b32 %0, 0\n\t.endr" : "=v"(dmy)); }
#endif
#ifdef ACL_CAL_SALU
        { int dmy; asm volatile(".rept 20\n\ts_mov_b32 %0, 0\n\t.endr" : "=s"(dmy)); }
#endif
        // (no fast exit for a column holding one (price, who) everywhere: the
        // uniform-column rule below keeps such columns out of the dirty set,
        // so the test cost more than it saved; the levels resolve it exactly)
        sp.mark(PS_L0);
        // winners, level by level. Per-vehicle state as lane masks: U = not
        // yet resolved, Nd = exact scan. Each resolving level's successor
        // bounds the decision gap of the vehicles it resolved (their
        // runner-up is that level or a lower one).
        unsigned long long U[NC], Nd[NC];
        unsigned k1[NC];  // a vehicle's winning level key (0: tie / scan)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          U[c] = okm[c];
          Nd[c] = 0ull;
          k1[c] = 0u;
        }
        unsigned Mk = M0, kres = 0u;  // kres: the last level that resolved a vehicle
        // the runner-up walk is needed: a resolving level's successor within
        // Gw (its vehicles' decision gaps are at least that level pair's)
        bool walk = false;
        if (nonfinite) {  // NaN prices: the exact scan for every vehicle
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            Nd[c] = U[c];
            U[c] = 0ull;
          }
        } else {
#pragma unroll 1
          for (int k = 0;;) {
            if (tie) {
              // a level held under two `who`s (equal prices): the exact scan
              // for every vehicle not resolved above it (rare; the bound of
              // the last resolving level was taken against this level)
#pragma unroll
              for (int c = 0; c < NC; ++c) {
                Nd[c] = U[c];
                U[c] = 0ull;
              }
              kres = 0u;
              break;
            }
            unsigned long long hitm[NC];
            level_hits<NC>(U, h, vm, hitm);
            unsigned long long left = 0ull, res = 0ull;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              const bool hit = lanebit(hitm[c]);
              nw[c] = hit ? wk : nw[c];
              k1[c] = hit ? Mk : k1[c];
              U[c] &= ~hitm[c];
              left |= U[c];
              res |= hitm[c];
            }
            kres = res ? Mk : 0u;
            if (!left || ++k == kAL) break;
            // the next level
            Mk = level_key<NC>(key, Mk);
            if (kMarg) {
              // gap(P(kres), P(Mk)) <= Gw, tested conservatively in f32
              // (kres == 0: a NaN pair, no effect; Mk == 0: lo = NaN, no effect)
              const float hk = __uint_as_float(kres - 1u), lk = __uint_as_float(Mk - 1u);
              walk |= hk - lk <= Gwf * hk;
            }
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              h[c] = __ballot(key[c] == Mk);
              cum += __popcll(h[c]);
            }
            wk = first_who<NC>(h, wu);
            tie = 0ull;
#pragma unroll
            for (int c = 0; c < NC; ++c) tie |= h[c] & __ballot(wu[c] != wk);
          }
        }
        sp.mark(PS_LV);
        if (kMarg && !walk && kres != 0u && cum < n) {
          // the last resolving level's successor (the highest key below
          // kres) within Gw: an entry with a key in [low, kres), low the key
          // of a lower bound of P(kres) (1 - Gw (1 + 2^-20)): the f32 product
          // with the factor one ulp low, then one more ulp lower, so no
          // successor within Gw is missed
          const float lowf = __uint_as_float(kres - 1u) * Gfacf;
          const unsigned lb = __float_as_uint(lowf);
          const unsigned lowk = lb > 1u ? lb : 1u;  // (bits - 1) + 1
          unsigned long long any = 0ull;
#pragma unroll
          for (int c = 0; c < NC; ++c) any |= __ballot(key[c] >= lowk && key[c] < kres);
          walk = any != 0ull;
        }
        // the exact runner-ups only where a level pair could lower the
        // wave's running minimum or the published one (an evaluation skipped
        // here has gaps >= its level pairs' > Gw, so the minimum is unchanged)
        walk = walk && kMarg;
        sp.mark(PS_MB);
        if (walk) {
          runner_up_walk<NC>(n, key, k1, Nd, vm, uhi, ulo);
          Gw = fmin(Gpub, margin_gap_pair(uhi, ulo));
          Gwf = (float)(Gw * (1.0 + 0x1p-20));
          Gfacf = gfac(Gw);
          if (ACL_AUCTION_PROF) sp.walks++;
          sp.mark(PS_WALK);
        }
        // the exact ordered scan (ascending vehid, strict >) for ties, NaN
        // prices and vehicles the levels did not resolve; the runner-up is the
        // best price of another `who` (entries of one `who` share its price)
        unsigned long long scan = 0ull;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          Nd[c] |= U[c];
          scan |= Nd[c];
        }
        if (scan) {
          if (ACL_AUCTION_PROF) sp.scans++;
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            if (lanebit(Nd[c])) {
              float bp = 0.0f, p2 = 0.0f;
              int bw = n;
              bool first = true, have2 = false;
#pragma unroll
              for (int w2 = 0; w2 < NC; ++w2) {
                unsigned long long m2 = vm[c][w2];
                while (m2) {
                  const int u = 64 * w2 + __ffsll((long long)m2) - 1;
                  m2 &= m2 - 1;
                  const int wx = T[u * TS + j];
                  const float px = C[__umul24(wx, n) + j];
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
        sp.mark(PS_SCAN);
        // the scan read the column: rewrite it only now
        __builtin_amdgcn_wave_barrier();
        unsigned long long ch = 0ull, mixed = 0ull;
        const int nw0 = __builtin_amdgcn_readfirstlane(nw[0]);  // vehicle 0's new entry
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          // (lanes past n store to a dummy row: no branch, see margin_track_sel)
          smem[okv[c] ? L.T + rowa[c] + j : L.dummy + lane] = (unsigned char)nw[c];
          const int u = lane + 64 * c;
          fl |= (vflag(okv[c]) & vflag(wu[c] == u) & vflag(nw[c] != u)) << c;
          ch |= __ballot(nw[c] != wu[c]);
          mixed |= __ballot(okv[c] && nw[c] != nw0);
        }
        // A column left holding one `who` everywhere is a fixed point (every
        // neighbourhood sees one (price, who)) with no runner-up: it is not
        // dirty next round unless a re-select writes it (which marks it).
        // The change itself still counts for eff_rounds.
        if (ch) {
          fl |= 1u << FL_CH;
          if (mixed || nonfinite) fl |= vflag(lane == (j & 63)) << (FL_DIRTY + (j >> 6));
        }
        sp.mark(PS_WB);
      }
    }
    }  // (a wave with no dirty column)
#pragma unroll
    for (int c = 0; c < NC; ++c) {  // publish the outbid vehicles
      if (!cw) break;
      const unsigned long long ob = __ballot((fl >> c) & 1u);
      if (ob && lane == 0) atomicOr(&obm[2 * par + c], ob);
    }
    if (MG && !ACL_AUCTION_NO_PUBLISH && (!ACL_CBAA_LAZY || evald) && r <= ACL_PUBLISH_ROUNDS) {
      // publish this wave's smallest gap so far (its lanes' select and scan
      // evaluations, its walks' pair) for the next round's pruning: an upper
      // bound is enough there (gap_ub); only after a round in which the wave
      // evaluated something (its pairs are unchanged otherwise)
      publish_gap_ub(margw, mp, uhi, ulo);
      evald = false;
    }
    sp.mark(PS_WB);
    __syncthreads();
    sp.mark(PS_BAR);
    // outbid vehicles re-select on their updated rows (auctioneer.cpp:224)
    {
      if (tid == 0) {
        dmask[2 * par] = 0ull;  // consumed; becomes round r+2's mask
        dmask[2 * par + 1] = 0ull;
        obm[2 * npar] = 0ull;   // round r+1's outbid mask
        obm[2 * npar + 1] = 0ull;
        misc[A_RCH + npar] = 0;  // round r+1's change flag (round r-1's was read)
      }
      int base = 0;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (!cw) break;
        const unsigned long long O = uni_u64(obm[2 * par + c]);
        const int rk = base + (int)__builtin_amdgcn_mbcnt_hi(
                                  (unsigned)(O >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)O, 0u));
        unsigned long long mv = __ballot(((O >> lane) & 1ull) && (rk & (kCW - 1)) == wave);
        base += __popcll(O);
        while (mv) {
          const int v = 64 * c + __ffsll((long long)mv) - 1;
          mv &= mv - 1;
          const int task = wave_select<NC, MG>(n, TS, v, lane, C, T, false, mp, &sp.selx);
          if (ACL_AUCTION_PROF) sp.sels++;
          evald = true;
          smem[(task >= 0 && lane == 0) ? L.T + v * TS + task : L.dummy + lane] = (unsigned char)v;
          if (ACL_CBAA_COLMAX && task >= 0 && lane == 0)
            atomicMax(&cmax[task], __float_as_uint(C[v * n + task]) + 1u);
          fl |= (vflag(task >= 0) & vflag(lane == (task & 63))) << (FL_DIRTY + (task >> 6));
        }
      }
    }
    if (cw) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {  // publish next round's dirty columns
        const unsigned long long dm = __ballot((fl >> (FL_DIRTY + c)) & 1u);
        if (dm && lane == 0) atomicOr(&dmask[2 * npar + c], dm);
      }
      if (__any((fl >> FL_CH) & 1u) && lane == 0) misc[A_RCH + par] = 1;
    }
    fl = 0u;
    __syncthreads();
    sp.mark(PS_SEL);
    // a re-select always changes an entry; columns that changed but became
    // uniform are not in the next mask (above)
    const bool next = (dmask[2 * npar] | dmask[2 * npar + 1]) != 0ull;
    if (next || misc[A_RCH + par]) eff = r;
    // no dirty column and no re-select: round r+1 changes nothing, so round
    // r's table is the fixed point every later round repeats (SURVEY App.
    // A.5): the outcome of all 2N rounds. early_exit = 0 still iterates the
    // remaining (empty) rounds, the reference's literal schedule.
    if (!next && P.early_exit) break;
  }
  sp.flush(P, b, lane);
  stamp_phase(P, b, tid, 4);
  ACL_AUCTION_STOP_AT(5);
  // FUSE: the control phase's global reads now, so that adoption and the
  // hand-off hide their latency (pair_fused.h, fused_prefetch). P.ctl through
  // the kernel-argument segment, loaded where it is used (pair_fused.h): P is
  // this kernel's only argument, at offset 0
  FusedPre fpre;
#ifndef ACL_FUSED_PREFETCH
#define ACL_FUSED_PREFETCH 0
#endif
  if constexpr (FUSE && ACL_FUSED_PREFETCH) {
    KCtlParams* pc = (KCtlParams*)((const __attribute__((address_space(4))) char*)
                                       __builtin_amdgcn_kernarg_segment_ptr() +
                                   offsetof(SolveParams, ctl));
    asm volatile("" : "+s"(pc));
    fused_prefetch(*pc, b, f, tid, fpre);
  }
  if (MG) {  // swarm margin: every lane's pair and the wave's level pair (the
             // alignments' gaps are in already)
    margin_track(mp, uhi, ulo);
    block_min_gap(margw, margin_gap(mp));
  }

  // ---------------- phase 4: adoption ---------------------------------------
  // do all vehicles hold vehicle 0's table? (rows compared as dwords; the
  // padding bytes of a row are `none` in every row)
  {
    const unsigned* T32 = reinterpret_cast<const unsigned*>(T);
    const int rw = TS / 4;  // <= 32 dwords per row (n <= 128)
    bool diff = false;
    // a wave per row, lanes over its dwords (no division by rw)
    const unsigned r0 = lane < rw ? T32[lane] : 0u;
    for (int v = wave; v < n; v += kAW) diff |= lane < rw && T32[v * rw + lane] != r0;
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
    for (int c = 0; c < NC; ++c) {
      const int jj = lane + 64 * c;
      if (jj < n) {
        const int w = row[jj];
        if (w >= n) bad = true;
        else lo[w >> 5] |= 1u << (w & 31);
      }
    }
    int cnt = 0;
#pragma unroll
    for (int q4 = 0; q4 < 2 * NC; ++q4) cnt += __popc(wave_or_u32(lo[q4]));
    return !__any(bad) && cnt == n;
  };
  if (allagree) {
    // one table: its validity is every vehicle's; vehicle T[0][j] adopts j
    const bool valid0 = row_valid(T);  // every wave checks row 0 (no barrier)
    if (tid == 0 && !valid0) misc[M_NINV] = n;
    for (int jj = tid; jj < n; jj += kAB) {
      const int v = valid0 ? T[jj] : Ptin[jj];
      P.P_out[(size_t)b * n + v] = (uint16_t)jj;
      validv[v] = valid0;
      if (jj != Pin[v]) misc[M_CHANGED] = 1;
    }
  } else {
    for (int v = wave; v < n; v += kAW) {
      const unsigned char* row = T + v * TS;
      bool ismine[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int jj = lane + 64 * c;
        ismine[c] = (jj < n) && (row[jj] == v);
      }
      int mine = -1;
#pragma unroll
      for (int c = NC - 1; c >= 0; --c) {
        const unsigned long long mm = __ballot(ismine[c]);
        if (mm) mine = 64 * c + __ffsll((long long)mm) - 1;
      }
      const bool valid = row_valid(row) && mine >= 0;
      const int adopted = valid ? mine : Pin[v];
      if (lane == 0) {
        validv[v] = valid;
        if (!valid) atomicAdd(&misc[M_NINV], 1);
        if (adopted != Pin[v]) misc[M_CHANGED] = 1;
        P.P_out[(size_t)b * n + v] = (uint16_t)adopted;
      }
    }
  }
  if (P.who) {
    for (int k = tid; k < n * n; k += kAB) {
      const int v = k / n, jj = k - v * n;
      const int w = T[v * TS + jj];
      P.who[(size_t)b * n * n + k] = (w >= n) ? (uint16_t)0xFFFF : (uint16_t)w;
    }
  }
  __syncthreads();
  stamp_phase(P, b, tid, 5);

  // ---------------- hand-off to the control kernels --------------------------
  // Each vehicle's adopted inverse assignment (formation point -> vehicle):
  // one shared row when every vehicle adopts the same one (all tables valid
  // and identical, or none valid), else one row per vehicle.
  const int ninv = misc[M_NINV];
  const bool allvalid = ninv == 0;
  // (own rows: a vehicle without a valid table keeps its own row, so only an
  // agreed valid table is one row for all)
  const bool uniform = (allvalid && misc[M_AGREE]) || (ninv == n && !rowsm);
  // this thread's entry of the shared row (fused control phase)
  const int ptv = (uniform && tid < n) ? (allvalid ? T[tid] : Ptin[tid]) : 0;
  {
    uint16_t* wsPt = reinterpret_cast<uint16_t*>(P.ws + P.W.pt) + (size_t)b * n;
    if (tid == 0) P.ws[P.W.mode + b] = uniform ? 0 : 1;
    if (uniform) {
      for (int jj = tid; jj < n; jj += kAB) wsPt[jj] = allvalid ? T[jj] : Ptin[jj];
    } else {
      uint16_t* rows = reinterpret_cast<uint16_t*>(P.ws + P.W.rows) + (size_t)b * n * n;
      for (int k = tid; k < n * n; k += kAB) {
        const int v = k / n, jj = k - v * n;
        rows[k] = validv[v] ? T[v * TS + jj]
                  : rowsm ? P.P_rows[(size_t)b * n * n + k] : Ptin[jj];
      }
      for (int v = tid; v < n; v += kAB) P.ws[P.W.vvalid + (size_t)b * n + v] = validv[v];
    }
    if (tid == 0) {
      acl_swarm_status_t st = {};
      uint32_t fl = 0;
      if (allvalid) fl |= ACL_SWARM_VALID;
      if (misc[M_AGREE]) fl |= ACL_SWARM_AGREE;
      if (misc[M_CHANGED]) fl |= ACL_SWARM_CHANGED;
      if (nonfinite) fl |= ACL_SWARM_NONFINITE;
      // (MG false: acl_solve_args_t::skip_margin -- not tracked, -1)
      const double g = !MG ? -1.0 : nonfinite ? 0.0 : __longlong_as_double((long long)*margw);
      if (MG && g < ACL_FRAGILE_MARGIN) fl |= ACL_SWARM_FRAGILE;
      st.flags = fl;
      st.eff_rounds = (uint16_t)eff;
      st.rounds = (uint16_t)(2 * n);
      st.n_invalid = (uint16_t)ninv;
      st.margin = (float)g;
      P.status[b] = st;
    }
  }
  stamp_phase(P, b, tid, 6);

  // ---------------- phase 5: control (FUSE) ---------------------------------
  // DistCntrl::compute (distcntrl.cpp:46-102), saturation and the first
  // collision test of a swarm whose vehicles all adopted one assignment, by
  // this workgroup's waves once its own auction is done: the swarm's gain
  // stream (the call's HBM bytes) overlaps the auctions of the co-resident
  // swarms (scalar/LDS-issue bound) instead of following all of them in a
  // second launch. LDS: every auction table is dead after the barrier; the
  // pair layout starts at 0. Swarms with per-vehicle rows (mode 1) are left
  // to gain_kernel (launch_control which = 2).
  if constexpr (FUSE) {
    if (!uniform) return;  // workgroup-uniform
#ifdef ACL_EXP_SKIP_GAIN
    return;  // diagnostic builds: the fused kernel without its control phase
#endif
    __syncthreads();       // T, C and the hand-off reads are done
    const FusedLayout GL = make_fused_layout(n, kAW);
    if (tid < n) reinterpret_cast<uint16_t*>(smem + GL.Pt)[tid] = (uint16_t)ptv;
    // P.ctl through the kernel-argument segment, loaded where it is used
    // (pair_fused.h): P is this kernel's only argument, at offset 0
    KCtlParams* pc = (KCtlParams*)((const __attribute__((address_space(4))) char*)
                                       __builtin_amdgcn_kernarg_segment_ptr() +
                                   offsetof(SolveParams, ctl));
    asm volatile("" : "+s"(pc));
    if (!ACL_FUSED_PREFETCH) fused_prefetch(*pc, b, f, tid, fpre);
    if (ACL_CTL_PRIO || ACL_CBAA_PRIO) __builtin_amdgcn_s_setprio(ACL_CTL_PRIO);
    pair_gain_fused<kAW, GM>(pc, b, f, smem, tid, kAB, fpre);
    stamp_phase(P, b, tid, 7);  // diagnostic: end of the control phase
  }
  stamp_rt(P, b, tid, kStampRt1);
}

// test hook: acl_price (fast path) and the IEEE expression for m squared
// distances (tests/test_gpu_prices.py)
__global__ void price_sweep_kernel(const double* x, float* fast, float* ieee, int m) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) {
    fast[i] = acl_price(x[i]);
    ieee[i] = (float)(1.0 / (sqrt(x[i]) + 1e-8));
  }
}

// the dynamic LDS of the auction kernel, fused or not
static int auction_lds(int n, bool fuse) {
  const int a = make_alayout(n).total;
  if (!fuse) return a;
  const int kAW = n <= 32 ? 2 : (n <= 64 ? 4 : 8);
  const int g = make_fused_layout(n, kAW).total;
  return a > g ? a : g;
}

template <bool FUSE, bool GM, bool MG>
static hipError_t launch_auction_t(const SolveParams& P, int nb, hipStream_t stream) {
  static PerDeviceOnce once;
  const hipError_t ea = once.run([] {
    for (const void* k : {(const void*)auction_kernel<1, 128, FUSE, GM, MG>,
                          (const void*)auction_kernel<1, 256, FUSE, GM, MG>,
                          (const void*)auction_kernel<2, 512, FUSE, GM, MG>}) {
      const hipError_t e =
          hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  });
  if (ea != hipSuccess) return ea;
  // phase 1 (the alignment) as its own launch, one wave per swarm
  // (n <= 64: inside the auction workgroup)
  if (P.n > 64)
    hipLaunchKernelGGL((align_kernel<2>), dim3(nb), dim3(64), make_align_layout(P.n).total, stream,
                       P);
  const int lds = auction_lds(P.n, FUSE);
  // (64 threads for n <= 32 measured no faster at C2: 0.091 vs 0.088 ms)
  if (P.n <= 32)
    hipLaunchKernelGGL((auction_kernel<1, 128, FUSE, GM, MG>), dim3(nb), dim3(128), lds, stream, P);
  else if (P.n <= 64)
    hipLaunchKernelGGL((auction_kernel<1, 256, FUSE, GM, MG>), dim3(nb), dim3(256), lds, stream, P);
  else
    hipLaunchKernelGGL((auction_kernel<2, 512, FUSE, GM, MG>), dim3(nb), dim3(512), lds, stream, P);
  return hipGetLastError();
}

// fuse: run the control phase in the auction's workgroups (P.ctl filled;
// 5-plane gain records, n <= 128)
// skip_margin: the decision margin is not tracked (status margin -1)
hipError_t launch_auction(const SolveParams& P, int nb, hipStream_t stream, bool fuse) {
  const bool mg = !P.skip_margin;
  if (!fuse)
    return mg ? launch_auction_t<false, false, true>(P, nb, stream)
              : launch_auction_t<false, false, false>(P, nb, stream);
  if (P.ctl.gate_margin)
    return mg ? launch_auction_t<true, true, true>(P, nb, stream)
              : launch_auction_t<true, true, false>(P, nb, stream);
  return mg ? launch_auction_t<true, false, true>(P, nb, stream)
            : launch_auction_t<true, false, false>(P, nb, stream);
}

}  // namespace acl_amd

extern "C" int acl_internal_price_sweep(const double* x, float* fast, float* ieee, int m) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(acl_amd::price_sweep_kernel, dim3((m + 255) / 256), dim3(256), 0, 0, x, fast,
                     ieee, m);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
