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

#include "../../include/aclswarm_amd.h"
#include "umeyama_dev.h"

namespace acl_amd {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kMaxN = 128;  // two 64-bit words per bitmask row, u8 indices
constexpr double kPi = 3.14159265358979323846;

struct Layout {
  // byte offsets into the dynamic LDS block (all 16-byte aligned)
  int q, p, qf, out, adjF, vadj, H, C, T0, T1, Pin, Ptin, cao, myi, valid, rowptr, misc;
  int total;
};

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

constexpr int kLevels = 3;  // price levels tracked per dirty column

__host__ __device__ inline Layout make_layout(int n) {
  Layout L;
  int o = 0;
  L.q = o;      o = align16(o + n * 3 * 8);
  L.p = o;      o = align16(o + n * 3 * 8);
  L.qf = o;     o = align16(o + n * 2 * 8);   // q_xy in formation space
  L.out = o;    o = align16(o + n * 6 * 8);   // R,t per vehicle; later u, u_safe
  L.adjF = o;   o = align16(o + n * 2 * 8);
  L.vadj = o;   o = align16(o + n * 2 * 8);
  L.H = o;      o = align16(o + 64 + n);      // CBAA masks + per-column buffer index
  L.C = o;
  {
    const int csz = (n + 1) * n * 4;
    const int ca = kWaves * 4 * n * 9;         // collision-avoidance scratch
    o = align16(o + (csz > ca ? csz : ca));
  }
  L.T0 = o;     o = align16(o + n * n);
  L.T1 = o;     o = align16(o + n * n);
  L.Pin = o;    o = align16(o + n);
  L.Ptin = o;   o = align16(o + n);
  L.cao = o;    o = align16(o + n);
  L.myi = o;    o = align16(o + n);
  L.valid = o;  o = align16(o + n);
  L.rowptr = o; o = align16(o + (n + 1) * 4);
  L.misc = o;   o = align16(o + 64);
  L.total = o;
  return L;
}

struct SolveParams {
  int n, B, F;
  const double* p;
  const uint64_t* adj;
  const double* gains;
  const int64_t* gain_off;
  const int32_t* fidx;
  const double* q;
  const double* vel;
  const uint16_t* P_in;
  uint16_t* P_out;
  acl_swarm_status_t* status;
  double* u;
  double* u_safe;
  uint8_t* ca_flag;
  uint16_t* who;
  acl_cntrl_gains_t g;
  acl_safety_params_t s;
  int early_exit;
  int do_control;
  unsigned long long* stamps;  // diagnostic: [B][16] s_memtime at phase ends (NULL = off)
};

// misc int slots
enum { M_BAD = 0, M_NONFIN = 1, M_CHG0 = 2, M_NINV = 5, M_AGREE = 6, M_CHANGED = 7, M_NCA = 8 };

// Wave64 reductions on DPP (VALU lane shuffles, no LDS round trip):
// quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, 8 give every lane its row's
// result; row_bcast15 / row_bcast31 fold rows 0-3 into lane 63.
// Callers must have all 64 lanes active.
#define ACL_DPP_STEP(x, op, ctrl, rmask)                                                   \
  x = op(x, __builtin_amdgcn_update_dpp(x, x, ctrl, rmask, 0xF, false))

__device__ __forceinline__ unsigned umax32(unsigned a, int b) { return a > (unsigned)b ? a : (unsigned)b; }

__device__ __forceinline__ unsigned wave_max_u32(unsigned ux) {
  int x = (int)ux;
#define ACL_UMAX(a, b) (int)umax32((unsigned)(a), (b))
  ACL_DPP_STEP(x, ACL_UMAX, 0xB1, 0xF);
  ACL_DPP_STEP(x, ACL_UMAX, 0x4E, 0xF);
  ACL_DPP_STEP(x, ACL_UMAX, 0x124, 0xF);
  ACL_DPP_STEP(x, ACL_UMAX, 0x128, 0xF);
  ACL_DPP_STEP(x, ACL_UMAX, 0x142, 0xA);
  ACL_DPP_STEP(x, ACL_UMAX, 0x143, 0xC);
#undef ACL_UMAX
  return (unsigned)__builtin_amdgcn_readlane(x, 63);
}

__device__ __forceinline__ float wave_max_f32(float fx) {
  int x = __float_as_int(fx);
#define ACL_FMAX(a, b) __float_as_int(fmaxf(__int_as_float(a), __int_as_float(b)))
  ACL_DPP_STEP(x, ACL_FMAX, 0xB1, 0xF);
  ACL_DPP_STEP(x, ACL_FMAX, 0x4E, 0xF);
  ACL_DPP_STEP(x, ACL_FMAX, 0x124, 0xF);
  ACL_DPP_STEP(x, ACL_FMAX, 0x128, 0xF);
  ACL_DPP_STEP(x, ACL_FMAX, 0x142, 0xA);
  ACL_DPP_STEP(x, ACL_FMAX, 0x143, 0xC);
#undef ACL_FMAX
  return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long x) {
  const unsigned hi = (unsigned)(x >> 32), lo = (unsigned)x;
  const unsigned mh = wave_max_u32(hi);
  const unsigned ml = wave_max_u32(hi == mh ? lo : 0u);
  return ((unsigned long long)mh << 32) | ml;
}

// DPP move of a double; lanes outside RMASK read 0 (the sum's identity).
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_f64_z(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u, CTRL, RMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, RMASK, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Sum over the wave, result in every lane (tree order: the control law's
// parity is tolerance-based, 1e-5 relative).
__device__ __forceinline__ double wave_sum(double x) {
  x += dpp_f64_z<0xB1, 0xF>(x);
  x += dpp_f64_z<0x4E, 0xF>(x);
  x += dpp_f64_z<0x124, 0xF>(x);
  x += dpp_f64_z<0x128, 0xF>(x);
  x += dpp_f64_z<0x142, 0xA>(x);
  x += dpp_f64_z<0x143, 0xC>(x);
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)u, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(u >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ double wrap_to_pi(double a) {  // utils.h:275-280
  if (a > kPi) return a - 2 * kPi;
  if (a < -kPi) return a + 2 * kPi;
  return a;
}

__device__ __forceinline__ void stamp(const SolveParams& P, int b, int tid, int k) {
  if (P.stamps && tid == 0) P.stamps[(size_t)b * 16 + k] = __builtin_amdgcn_s_memtime();
}

// selectTaskAssignment (auctioneer.cpp:517-542) for vehicle v as a wave
// argmax: the first task j maximizing C[v][j] among tasks with
// C[v][j] > price_j (price_j = C[who_j][j]); nw[c] is this lane's entry for
// task lane+64c. Returns the selected task (wave-uniform) or -1.
__device__ __forceinline__ int wave_select(int n, int v, int lane, const float* C,
                                           const int (&nw)[2]) {
  unsigned long long key = 0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int j = lane + 64 * c;
    if (j < n) {
      const float cv = C[v * n + j];
      const float pr = C[nw[c] * n + j];
      if (cv > 0.0f && cv > pr)
        key = max(key, ((unsigned long long)__float_as_uint(cv) << 32) |
                           (unsigned long long)(0xFFFFFFFFu - (unsigned)j));
    }
  }
  key = wave_max_u64(key);
  if (key == 0) return -1;
  return (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull));
}

__global__ void __launch_bounds__(kBlock) solve_kernel(const SolveParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const Layout L = make_layout(n);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;

  double* q = reinterpret_cast<double*>(smem + L.q);
  double* p = reinterpret_cast<double*>(smem + L.p);
  double* qf = reinterpret_cast<double*>(smem + L.qf);
  double* out = reinterpret_cast<double*>(smem + L.out);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adjF);
  unsigned long long* vadj = reinterpret_cast<unsigned long long*>(smem + L.vadj);
  unsigned long long* H = reinterpret_cast<unsigned long long*>(smem + L.H);
  float* C = reinterpret_cast<float*>(smem + L.C);
  // the two table buffers; indexed by offset so every access stays an LDS
  // (addrspace 3) access -- a runtime-selected pointer would become flat
  unsigned char* const T0 = smem + L.T0;
  const int Tstr = L.T1 - L.T0;
  unsigned char* Pin = smem + L.Pin;
  unsigned char* Ptin = smem + L.Ptin;
  unsigned char* cao = smem + L.cao;
  unsigned char* myi = smem + L.myi;
  unsigned char* validv = smem + L.valid;
  int* rowptr = reinterpret_cast<int*>(smem + L.rowptr);
  int* misc = reinterpret_cast<int*>(smem + L.misc);

  const int f = P.fidx[b];
  const int W = 2;
  const int gw = (n + 63) >> 6;  // words per row in the global table
  const unsigned long long lastmask =
      (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  stamp(P, b, tid, 0);

  // ---------------- phase 0: load -----------------------------------------
  {
    const double* gq = P.q + (size_t)b * n * 3;
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += kBlock) {
      q[k] = gq[k];
      p[k] = gp[k];
    }
    const uint64_t* ga = P.adj + (size_t)f * n * gw;
    for (int k = tid; k < n * W; k += kBlock) {
      const int i = k >> 1, w = k & 1;
      unsigned long long x = 0;
      if (w < gw) {
        x = ga[(size_t)i * gw + w];
        if (w == gw - 1) x &= lastmask;
      }
      adjF[k] = x;
    }
    if (tid < 16) misc[tid] = 0;
    if (tid == 0) misc[M_AGREE] = 1;
    if (tid < 2) H[tid] = 0ull;  // "seen" mask for the permutation check
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
  // rows of the formation CSR (edge e of row i in row-major order); the
  // diagonal is an edge of the control law if adjmat(i,i) != 0 (distcntrl.cpp:62)
  if (tid == 0) {
    int acc = 0;
    for (int i = 0; i < n; ++i) {
      rowptr[i] = acc;
      acc += __popcll(adjF[2 * i]) + __popcll(adjF[2 * i + 1]);
    }
    rowptr[n] = acc;
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
    if (tid == 0) {
      acl_swarm_status_t st = {};
      st.flags = ACL_SWARM_BAD_INPUT;
      st.rounds = (uint16_t)(2 * n);
      P.status[b] = st;
    }
    return;
  }

  // q in formation space: qf[j] = q[Pt[j]] (xy only; the alignment is 2-D)
  for (int j = tid; j < n; j += kBlock) {
    const int vj = Ptin[j];
    qf[2 * j] = q[3 * vj];
    qf[2 * j + 1] = q[3 * vj + 1];
  }
  // vehicle-space closed neighbourhoods: u ~ v iff u == v or adj(P[v], P[u])
  // (bidIterComplete, auctioneer.cpp:419-437). Lane = v, uniform loop over u.
  for (int v = tid; v < ((n + 63) & ~63); v += kBlock) {
    const int i = (v < n) ? Pin[v] : 0;
    const unsigned long long a0 = adjF[2 * i], a1 = adjF[2 * i + 1];
    unsigned long long m0 = 0, m1 = 0;
    for (int u = 0; u < n; ++u) {
      const int pu = Pin[u];
      const bool e = (u == v) || (((pu < 64 ? a0 : a1) >> (pu & 63)) & 1ull);
      if (u < 64) m0 |= (unsigned long long)e << u;
      else m1 |= (unsigned long long)e << (u - 64);
    }
    if (v < n) {
      vadj[2 * v] = m0;
      vadj[2 * v + 1] = m1;
    }
  }
  __syncthreads();
  stamp(P, b, tid, 1);

  // ---------------- phase 1: alignment (one thread per vehicle) ----------
  // Uniform loop over formation points j (broadcast LDS reads), predicated
  // on "j in my closed neighbourhood": the sums stay sequential in
  // ascending j, exactly as Eigen's rowwise().sum() / GEMM accumulate.
  for (int v = tid; v < ((n + 63) & ~63); v += kBlock) {
    const bool act = v < n;
    const int i = act ? Pin[v] : 0;
    unsigned long long r0 = adjF[2 * i], r1 = adjF[2 * i + 1];
    if (i < 64) r0 |= 1ull << i; else r1 |= 1ull << (i - 64);
    const int k = __popcll(r0) + __popcll(r1);
    double ssx = 0, ssy = 0, sdx = 0, sdy = 0;
    bool first = true;
    for (int j = 0; j < n; ++j) {
      const bool in = ((j < 64 ? r0 : r1) >> (j & 63)) & 1ull;
      const double px = p[3 * j], py = p[3 * j + 1], qx = qf[2 * j], qy = qf[2 * j + 1];
      if (in) {
        if (first) { ssx = px; ssy = py; sdx = qx; sdy = qy; first = false; }
        else { ssx = ssx + px; ssy = ssy + py; sdx = sdx + qx; sdy = sdy + qy; }
      }
    }
    const double oon = 1.0 / (double)k;
    const double sm[2] = {ssx * oon, ssy * oon};
    const double dm[2] = {sdx * oon, sdy * oon};
    // sigma = one_over_n * dst_demean * src_demean^T: lazy product (scaled
    // lhs) when k + 4 < 20, GEMM (alpha after the sum) otherwise
    const bool lazy = (k + 4) < 20;
    double a00 = 0, a01 = 0, a10 = 0, a11 = 0;  // a_ij = sum dst_i * src_j
    first = true;
    for (int j = 0; j < n; ++j) {
      const bool in = ((j < 64 ? r0 : r1) >> (j & 63)) & 1ull;
      const double s0 = p[3 * j] - sm[0], s1 = p[3 * j + 1] - sm[1];
      double d0 = qf[2 * j] - dm[0], d1 = qf[2 * j + 1] - dm[1];
      if (lazy) {
        d0 = oon * d0;
        d1 = oon * d1;
      }
      if (in) {
        if (lazy && first) {
          a00 = d0 * s0; a01 = d0 * s1; a10 = d1 * s0; a11 = d1 * s1;
        } else {
          a00 = a00 + d0 * s0; a01 = a01 + d0 * s1;
          a10 = a10 + d1 * s0; a11 = a11 + d1 * s1;
        }
        first = false;
      }
    }
    double S[4];  // column-major sigma
    if (lazy) { S[0] = a00; S[1] = a10; S[2] = a01; S[3] = a11; }
    else { S[0] = a00 * oon; S[1] = a10 * oon; S[2] = a01 * oon; S[3] = a11 * oon; }
    double R[4], t[2];
    umeyama_finish(S, sm, dm, R, t);
    if (act) {
      double* o = out + 6 * v;
      o[0] = R[0]; o[1] = R[1]; o[2] = R[2]; o[3] = R[3]; o[4] = t[0]; o[5] = t[1];
    }
  }
  __syncthreads();
  stamp(P, b, tid, 2);

  // ---------------- phase 2: prices ---------------------------------------
  {
    int nonfin = 0;
    for (int k = tid; k < n * n; k += kBlock) {
      const int v = k / n, j = k - v * n;
      const double* o = out + 6 * v;
      const double px = p[3 * j], py = p[3 * j + 1], pz = p[3 * j + 2];
      const double ax = ((o[0] * px + o[1] * py) + 0.0 * pz) + o[4];
      const double ay = ((o[2] * px + o[3] * py) + 0.0 * pz) + o[5];
      const double az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0;
      const double dx = q[3 * v] - ax, dy = q[3 * v + 1] - ay, dz = q[3 * v + 2] - az;
      const double nrm = sqrt((dx * dx + dy * dy) + dz * dz);
      const float c = (float)(1.0 / (nrm + 1e-8));
      C[k] = c;
      nonfin |= (c != c);
    }
    for (int j = tid; j < n; j += kBlock) C[n * n + j] = 0.0f;  // row `none`
    // initial tables: every entry unassigned (reset, auctioneer.cpp:448-465)
    for (int k = tid; k < n * n; k += kBlock) T0[k] = (unsigned char)n;
    if (__any(nonfin) && lane == 0) misc[M_NONFIN] = 1;
  }
  __syncthreads();
  const bool nonfinite = misc[M_NONFIN] != 0;
  stamp(P, b, tid, 3);

  // ---------------- phase 3: CBAA ------------------------------------------
  // CBAA state in the (now free) level region: dirty-column masks by round
  // parity, outbid-vehicle masks by round parity, per-column buffer index.
  unsigned long long* dmask = H;      // [2][2]
  unsigned long long* obm = H + 4;    // [2][2]
  unsigned char* colbuf = reinterpret_cast<unsigned char*>(H + 8);  // [n]
  if (tid < 8) H[tid] = 0ull;
  for (int jj = tid; jj < n; jj += kBlock) colbuf[jj] = 0;
  __syncthreads();
  // round 0: START bid = select from the zero table (start, auctioneer.cpp:105);
  // every column that received a bid is dirty for round 1
  for (int v = wave; v < n; v += kWaves) {
    int nw[2] = {n, n};
    const int task = wave_select(n, v, lane, C, nw);
    if (task >= 0 && lane == 0) {
      T0[v * n + task] = (unsigned char)v;
      atomicOr(&dmask[2 * 1 + (task >> 6)], 1ull << (task & 63));
    }
  }
  __syncthreads();

  int eff = 0;
  const int max_rounds = 2 * n;  // cbaa_max_iter_ = n * diameter (:50-51)
  unsigned long long sub[4] = {0, 0, 0, 0};
  unsigned long long tprev = P.stamps ? __builtin_amdgcn_s_memtime() : 0;
  auto substamp = [&](int k) {
    if (P.stamps) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      sub[k] += t - tprev;
      tprev = t;
    }
  };
  for (int r = 1; r <= max_rounds; ++r) {
    const int par = r & 1, npar = par ^ 1;
    const unsigned long long D0 = dmask[2 * par], D1 = dmask[2 * par + 1];
    if (P.stamps) sub[2] += __popcll(D0) + __popcll(D1);
    // A+B) One wave per dirty column j. A column none of whose entries changed
    // last round is a fixed point of updateTaskAssignment (it reads only
    // that column, and a select always changes the entry it writes), so only
    // dirty columns are recomputed. Lanes = vehicles.
    {
      int idx = 0;
      for (int w = 0; w < 2; ++w) {
        unsigned long long m = w ? D1 : D0;
        while (m) {
          const int j = 64 * w + __ffsll((long long)m) - 1;
          m &= m - 1;
          if ((idx++ & (kWaves - 1)) != wave) continue;
          const int cb = colbuf[j];
          const unsigned char* Tc = T0 + cb * Tstr;
          unsigned char* Tn = T0 + (cb ^ 1) * Tstr;
          int wu[2];
          float pu[2];
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int u = lane + 64 * c;
            wu[c] = n;
            pu[c] = -1.0f;
            if (u < n) {
              wu[c] = Tc[u * n + j];
              pu[c] = C[wu[c] * n + j];
            }
          }
          // A) the top kLevels distinct prices of the column, their holder
          //    masks, `who` and tie flag (wave max + ballots)
          float cap = __builtin_inff();
          unsigned long long Lh0[kLevels], Lh1[kLevels];
          int Lw[kLevels];
          bool Lt[kLevels];
#pragma unroll
          for (int k = 0; k < kLevels; ++k) {
            const float x0 = pu[0] < cap ? pu[0] : -1.0f;
            const float x1 = pu[1] < cap ? pu[1] : -1.0f;
            const float Pk = wave_max_f32(fmaxf(x0, x1));
            const bool e0 = pu[0] == Pk, e1 = pu[1] == Pk;
            const unsigned long long m0 = __ballot(e0), m1 = __ballot(e1);
            const int wk = m0 ? __builtin_amdgcn_readlane(wu[0], __ffsll((long long)m0) - 1)
                              : __builtin_amdgcn_readlane(wu[1], m1 ? __ffsll((long long)m1) - 1 : 0);
            const bool tk = (__ballot(e0 && wu[0] != wk) | __ballot(e1 && wu[1] != wk)) != 0ull;
            const bool empty = !(Pk >= 0.0f);
            Lh0[k] = empty ? 0ull : m0;
            Lh1[k] = empty ? 0ull : m1;
            Lw[k] = wk;
            Lt[k] = tk || nonfinite;
            cap = Pk;
          }
          // B) per vehicle v: the `who` of the highest level one of v's
          //    closed neighbours holds, unless that level is tied;
          //    otherwise the exact ordered scan (ascending vehid, strict >)
          bool ob[2], ch[2];
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int v = lane + 64 * c;
            ob[c] = ch[c] = false;
            if (v < n) {
              const unsigned long long vm0 = vadj[2 * v], vm1 = vadj[2 * v + 1];
              const int old = wu[c];
              int nw = n;
              bool decided = false, need = false;
#pragma unroll
              for (int k = 0; k < kLevels; ++k) {
                if (!decided && (((Lh0[k] & vm0) | (Lh1[k] & vm1)) != 0ull)) {
                  decided = true;
                  if (Lt[k]) need = true;
                  else nw = Lw[k];
                }
              }
              if (!decided) need = true;
              if (need) {
                float bp = 0.0f;
                int bw = n;
                bool first = true;
#pragma unroll
                for (int w2 = 0; w2 < 2; ++w2) {
                  unsigned long long mm = w2 ? vm1 : vm0;
                  while (mm) {
                    const int u = 64 * w2 + __ffsll((long long)mm) - 1;
                    mm &= mm - 1;
                    const int wx = Tc[u * n + j];
                    const float px = C[wx * n + j];
                    if (first) { bp = px; bw = wx; first = false; }
                    else if (px > bp) { bp = px; bw = wx; }
                  }
                }
                nw = bw;
              }
              Tn[v * n + j] = (unsigned char)nw;
              ob[c] = (old == v) && (nw != v);  // outbid (auctioneer.cpp:502)
              ch[c] = nw != old;
            }
          }
          const unsigned long long ob0 = __ballot(ob[0]), ob1 = __ballot(ob[1]);
          const bool anych = __any(ch[0] || ch[1]);
          if (lane == 0) {
            if (ob0) atomicOr(&obm[2 * par], ob0);
            if (ob1) atomicOr(&obm[2 * par + 1], ob1);
            if (anych) atomicOr(&dmask[2 * npar + (j >> 6)], 1ull << (j & 63));
            colbuf[j] = (unsigned char)(cb ^ 1);
          }
        }
      }
    }
    __syncthreads();
    substamp(0);
    // outbid vehicles re-select on their updated rows (auctioneer.cpp:224)
    {
      if (tid == 0) {
        dmask[2 * par] = 0ull;        // consumed; becomes round r+2's mask
        dmask[2 * par + 1] = 0ull;
        obm[2 * npar] = 0ull;         // round r+1's outbid mask
        obm[2 * npar + 1] = 0ull;
      }
      const unsigned long long O0 = obm[2 * par], O1 = obm[2 * par + 1];
      if (P.stamps) sub[3] += __popcll(O0) + __popcll(O1);
      int idx = 0;
      for (int w = 0; w < 2; ++w) {
        unsigned long long m = w ? O1 : O0;
        while (m) {
          const int v = 64 * w + __ffsll((long long)m) - 1;
          m &= m - 1;
          if ((idx++ & (kWaves - 1)) != wave) continue;
          int nw[2];
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int jj = lane + 64 * c;
            nw[c] = (jj < n) ? T0[colbuf[jj] * Tstr + v * n + jj] : n;
          }
          const int task = wave_select(n, v, lane, C, nw);
          if (task >= 0 && lane == 0) {
            T0[colbuf[task] * Tstr + v * n + task] = (unsigned char)v;
            atomicOr(&dmask[2 * npar + (task >> 6)], 1ull << (task & 63));
          }
        }
      }
    }
    __syncthreads();
    substamp(1);
    const bool changed = (dmask[2 * npar] | dmask[2 * npar + 1]) != 0ull;
    if (changed) eff = r;
    else if (P.early_exit) break;  // fixed point
  }
  // consolidate the per-column buffers into T[0]
  for (int k = tid; k < n * n; k += kBlock) {
    const int jj = k % n;
    if (colbuf[jj]) T0[k] = T0[Tstr + k];
  }
  __syncthreads();
  stamp(P, b, tid, 4);
  if (P.stamps && tid == 0)
    for (int k = 0; k < 4; ++k) P.stamps[(size_t)b * 16 + 8 + k] = sub[k];

  // ---------------- phase 4: adoption --------------------------------------
  const unsigned char* Tf = T0;
  for (int v = tid; v < n; v += kBlock) {
    const unsigned char* row = Tf + v * n;
    unsigned long long s0 = 0, s1 = 0;
    bool valid = true, agree = true;
    int mine = -1;
    for (int j = 0; j < n; ++j) {
      const int w = row[j];
      if (w >= n) { valid = false; continue; }
      const unsigned long long bit = 1ull << (w & 63);
      unsigned long long& s = (w < 64) ? s0 : s1;
      if (s & bit) valid = false;
      s |= bit;
      if (w == v && mine < 0) mine = j;
    }
    for (int j = 0; j < n && agree; ++j) agree = (row[j] == Tf[j]);
    if (!valid || mine < 0) {
      valid = false;
      mine = Pin[v];
    }
    validv[v] = valid;
    myi[v] = (unsigned char)mine;
    if (!valid) atomicAdd(&misc[M_NINV], 1);
    if (!agree) misc[M_AGREE] = 0;
    if (mine != Pin[v]) misc[M_CHANGED] = 1;
    P.P_out[(size_t)b * n + v] = (uint16_t)mine;
  }
  if (P.who) {
    for (int k = tid; k < n * n; k += kBlock) {
      const int w = Tf[k];
      P.who[(size_t)b * n * n + k] = (w >= n) ? (uint16_t)0xFFFF : (uint16_t)w;
    }
  }
  __syncthreads();
  stamp(P, b, tid, 5);

  // ---------------- phase 5: control + safety -----------------------------
  if (P.do_control) {
    double* uo = out;           // [n][3] u
    double* uso = out + 3 * n;  // [n][3] u_safe
    const int E = rowptr[n];
    const double* G = P.gains + 9 * P.gain_off[f];
    const acl_cntrl_gains_t g = P.g;
    const acl_safety_params_t sp = P.s;
    double* caA = reinterpret_cast<double*>(C) + wave * (4 * n);               // angles
    signed char* caS = reinterpret_cast<signed char*>(C) + kWaves * 4 * n * 8 + wave * 4 * n;
    // the 3x3 blocks of the vehicle's formation row: lane = column j (two
    // chunks of 64), coalesced across lanes in each of the 9 planes
    auto load_row = [&](int v, double (&A)[2][9], bool (&has)[2]) {
      const int i = myi[v];
      int ebase = rowptr[i];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const unsigned long long rowbits = adjF[2 * i + c];
        has[c] = (rowbits >> lane) & 1ull;
        const int e = ebase + __popcll(rowbits & ((1ull << lane) - 1ull));
        ebase += __popcll(rowbits);
#pragma unroll
        for (int k = 0; k < 9; ++k)
          A[c][k] = has[c] ? __builtin_nontemporal_load(G + (size_t)k * E + e) : 0.0;
      }
    };
    double Acur[2][9], Anx[2][9];
    bool hcur[2], hnx[2];
    if (wave < n) load_row(wave, Acur, hcur);
    for (int v = wave; v < n; v += kWaves) {
      // prefetch the next vehicle's gain blocks while this one computes
      if (v + kWaves < n) load_row(v + kWaves, Anx, hnx);
      const int i = myi[v];
      const unsigned char* Ptv = validv[v] ? (Tf + v * n) : Ptin;
      const double* gv = P.vel + ((size_t)b * n + v) * 3;
      const double vel0 = gv[0], vel1 = gv[1], vel2 = gv[2];
      const double qv0 = q[3 * v], qv1 = q[3 * v + 1], qv2 = q[3 * v + 2];
      const double pix = p[3 * i], piy = p[3 * i + 1], piz = p[3 * i + 2];
      const double Ni = pix * pix + piy * piy, Nzi = piz * piz;
      double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = lane + 64 * c;
        if (hcur[c]) {
          const double* A = Acur[c];
          const int u = Ptv[j];
          const double q0 = q[3 * u] - qv0, q1 = q[3 * u + 1] - qv1, q2 = q[3 * u + 2] - qv2;
          const double pjx = p[3 * j], pjy = p[3 * j + 1], pjz = p[3 * j + 2];
          const double Nj = pjx * pjx + pjy * pjy, Nzj = pjz * pjz;
          const double dxy = sqrt((Ni + Nj) - 2.0 * (pix * pjx + piy * pjy));
          const double dz = sqrt((Nzi + Nzj) - 2.0 * (piz * pjz));
          const double e_xy = sqrt(q0 * q0 + q1 * q1) - dxy;
          const double e_z = sqrt(q2 * q2) - dz;
          double Fxy = 0.0, Fz = 0.0;
          if (fabs(e_xy) > g.e_xy_thr) Fxy = g.K1_xy * atan(g.K2_xy * e_xy);
          if (fabs(e_z) > g.e_z_thr) Fz = g.K1_z * atan(g.K2_z * e_z);
          const double up0 = ((A[0] * q0 + A[1] * q1) + A[2] * q2) + Fxy * q0;
          const double up1 = ((A[3] * q0 + A[4] * q1) + A[5] * q2) + Fxy * q1;
          const double up2 = ((A[6] * q0 + A[7] * q1) + A[8] * q2) + Fz * q2;
          acc0 += g.kp * up0 + g.kd * (-vel0);
          acc1 += g.kp * up1 + g.kd * (-vel1);
          acc2 += g.kp * up2 + g.kd * (-vel2);
        }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        hcur[c] = hnx[c];
#pragma unroll
        for (int k = 0; k < 9; ++k) Acur[c][k] = Anx[c][k];
      }
      double cmd0 = wave_sum(acc0), cmd1 = wave_sum(acc1), cmd2 = wave_sum(acc2);
      if (lane == 0) {
        uo[3 * v] = cmd0; uo[3 * v + 1] = cmd1; uo[3 * v + 2] = cmd2;
      }
      // Safety::cmdinCb saturation (safety.cpp:185-196)
      {
        const double velxy = sqrt(cmd0 * cmd0 + cmd1 * cmd1);
        if (velxy > sp.max_vel_xy) {
          cmd0 = cmd0 / velxy * sp.max_vel_xy;
          cmd1 = cmd1 / velxy * sp.max_vel_xy;
        }
        const double velz = fabs(cmd2);
        if (velz > sp.max_vel_z) cmd2 = cmd2 / velz * sp.max_vel_z;
      }
      // Safety::collisionAvoidance (safety.cpp:412-541)
      bool modified = false;
      {
        bool cand[2];
        double dxv[2], dyv[2], dv[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int j = lane + 64 * c;
          cand[c] = false;
          if (j < n && j != v) {
            dxv[c] = q[3 * j] - qv0;
            dyv[c] = q[3 * j + 1] - qv1;
            dv[c] = sqrt(dxv[c] * dxv[c] + dyv[c] * dyv[c]);
            cand[c] = !(dv[c] > sp.d_avoid_thresh);
          }
        }
        const unsigned long long m0 = __ballot(cand[0]), m1 = __ballot(cand[1]);
        if (m0 | m1) {
          bool wrapped = false;
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            if (cand[c]) {
              const int slot = 4 * (__popcll((c ? m1 : m0) & ((1ull << lane) - 1ull)) +
                                    (c ? __popcll(m0) : 0));
              const double theta = atan2(dyv[c], dxv[c]);
              const double x = sp.r_keep_out / dv[c];
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
          }
          const bool didWrap = __any(wrapped);
          const int nslot = 4 * (__popcll(m0) + __popcll(m1));
          __builtin_amdgcn_wave_barrier();
          asm volatile("" ::: "memory");
          if (lane == 0) {
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
        uso[3 * v] = cmd0; uso[3 * v + 1] = cmd1; uso[3 * v + 2] = cmd2;
        cao[v] = modified;
        if (modified) atomicAdd(&misc[M_NCA], 1);
      }
    }
    __syncthreads();
    for (int k = tid; k < 3 * n; k += kBlock) {
      if (P.u) P.u[(size_t)b * n * 3 + k] = uo[k];
      if (P.u_safe) P.u_safe[(size_t)b * n * 3 + k] = uso[k];
    }
    if (P.ca_flag)
      for (int v = tid; v < n; v += kBlock) P.ca_flag[(size_t)b * n + v] = cao[v];
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

extern "C" int32_t acl_max_vehicles(void) { return acl_amd::kMaxN; }

// Diagnostic hook (not part of the public ABI): when set, the next solves
// record s_memtime at the end of each phase into stamps[B][8].
static unsigned long long* g_stamps = nullptr;
extern "C" void acl_internal_set_stamps(unsigned long long* stamps) { g_stamps = stamps; }

extern "C" acl_status_t acl_solve_batch(const acl_formations_t* F, const acl_solve_args_t* a,
                                        void* stream) {
  using namespace acl_amd;
  if (!F || !a) return acl__set_error("acl_solve_batch: null argument");
  const int n = F->n;
  if (n < 1 || n > kMaxN) return acl__set_error("acl_solve_batch: n out of range [1, 128]");
  if (a->B < 0) return acl__set_error("acl_solve_batch: B < 0");
  if (a->B == 0) return ACL_OK;
  if (!F->p || !F->adj || !a->fidx || !a->q || !a->P_in || !a->P_out || !a->status)
    return acl__set_error("acl_solve_batch: required pointer is NULL");
  if (a->do_control && (!F->gains || !F->gain_off || !a->vel))
    return acl__set_error("acl_solve_batch: do_control needs gains, gain_off and vel");
  SolveParams P;
  P.n = n; P.B = a->B; P.F = F->n_formations;
  P.p = F->p; P.adj = F->adj; P.gains = F->gains; P.gain_off = F->gain_off;
  P.fidx = a->fidx; P.q = a->q; P.vel = a->vel; P.P_in = a->P_in; P.P_out = a->P_out;
  P.status = a->status; P.u = a->u; P.u_safe = a->u_safe; P.ca_flag = a->ca_flag;
  P.who = a->who; P.g = a->cntrl; P.s = a->safety;
  P.early_exit = a->early_exit; P.do_control = a->do_control;
  P.stamps = g_stamps;
  const Layout L = make_layout(n);
  static int configured = 0;
  if (!configured) {
    if (hipFuncSetAttribute((const void*)solve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return acl__set_error("hipFuncSetAttribute failed");
    configured = 1;
  }
  hipLaunchKernelGGL(solve_kernel, dim3(a->B), dim3(kBlock), L.total, (hipStream_t)stream, P);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  return ACL_OK;
}
