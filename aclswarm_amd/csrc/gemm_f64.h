// gemm_f64.h -- batched fp64 GEMM on CDNA4 matrix cores (v_mfma_f64_16x16x4_f64).
//
// D = alpha * op(A) * op(B) + beta * C, column-major, one descriptor per
// batch entry (dims, leading dimensions, pointers and an optional skip flag
// live in device memory, so a setup kernel may fill them and converged
// problems drop out without a host round trip).
//
// Placement: a 1-D grid whose block b works on job (b % 8) + 8 k -- blocks
// b and b + 8 share an XCD (blocks are dealt round-robin over the 8 XCDs), so
// every tile of one job runs on one XCD and its operand panels are re-read
// from that XCD's L2 instead of being fetched by all eight.
// Symmetric jobs (SYM: D symmetric in exact arithmetic, square) compute only
// the tiles on and above the diagonal and store each off-diagonal one twice;
// in a diagonal tile (default kernel) only the 15 of 25 16 x 16 blocks on and
// above the block diagonal are computed, the others stored as their mirrors
// (C5: 6 025 -> 6 400 formations/s, profiles/r5_ab_c5diag/).
//
// Tiling (default): an 80 x 80 output tile per 256-thread workgroup, one wave
// per SIMD, 25 MFMA 16x16 blocks split evenly over the four waves
// (gemm80w4_f64_kernel); alternatives 64 x 64 / 32 x 32 (four waves in a 2 x 2
// arrangement) and the 80 tile on five waves. K staged through LDS in steps of
// 16, double-buffered, one barrier per step: untransposed jobs the host
// marks eligible by LDS-DMA (global_load_lds, no staging registers: four
// waves per SIMD), the others through a register prefetch (three).
// The MFMA is issued with the operands swapped (it computes the tile of D^T),
// so the accumulator's lane index runs along D's rows and every epilogue
// load/store is a contiguous 128-byte column segment.
#pragma once

#include <type_traits>

#include <hip/hip_runtime.h>
#include <stdlib.h>

namespace acl_amd {

struct GemmJob {
  const double* A;
  const double* B;
  const double* C;  // read when beta != 0 (may alias D)
  double* D;
  int m, n, k;
  int lda, ldb, ldc, ldd;
  double alpha, beta;
  const int* skip;  // job skipped when non-NULL and *skip != 0
  double* err2;     // non-NULL (default kernel only): += |D - I|_F^2 of the stored D
  // operand transform (default kernel only): operands in tmask (bit 0 A,
  // bit 1 B, bit 2 C) are read as (x - [diagonal] tdiag) * (1 / *tnrm) --
  // the Newton-Schulz start Z0 = (W - eps I) / nrm formed while staging
  // instead of a pass that writes it
  const double* tnrm = nullptr;
  double tdiag = 0.0;
  int tmask = 0;
  // trace partials (default kernel only): a diagonal tile (bi == bj) stores
  // the sum of its diagonal at trp[bi] (fixed-order sums: deterministic)
  double* trp = nullptr;
  // scaled Newton-Schulz update (default kernel only): with nsp set, the
  // product D = alpha Z Y + beta Z (Y = Z^2) is taken for a Z -- alpha *= a^3,
  // beta *= a -- with a = sqrt(m / tr Y) capped at nscap, tr Y = the nsn
  // partials at nsp summed in order; a = 1 when *nserr < nstol (the part's
  // last update) or the ratio is not a number
  const double* nsp = nullptr;
  const double* nserr = nullptr;
  int nsn = 0;
  double nscap = 0.0, nstol = 0.0;
  // gate (default kernel only): the job runs only while glo <= *gerr < ghi
  const double* gerr = nullptr;
  double glo = 0.0, ghi = 0.0;
  // alternative operand (default kernel only, with nserr): while
  // qlo <= *nserr < qhi the product reads B = qB (untransformed) and takes
  // alpha = qalpha, beta = qbeta, unscaled (the quintic final update)
  const double* qB = nullptr;
  double qlo = 0.0, qhi = 0.0, qalpha = 0.0, qbeta = 0.0;
};

typedef double f64x4 __attribute__((ext_vector_type(4)));

// 16 zero bytes: the source of the LDS-DMA lanes outside an operand
__device__ __attribute__((aligned(16))) double g_gemm_zero16[2];

template <int W>
struct GemmWave {  // a wave index as a type (per-wave specialised code)
  static constexpr int value = W;
};

constexpr int kGemmKStep = 16;
#ifndef ACL_GEMM_WSPEC
#define ACL_GEMM_WSPEC 1  // the 80-tile kernel's K loop specialised per wave
#endif
#ifndef ACL_GEMM_OPF
#define ACL_GEMM_OPF 1  // LDS operands read one k4 step ahead
#endif
#ifndef ACL_GEMM_DMA
#define ACL_GEMM_DMA 1  // untransposed products staged by LDS-DMA where the host allows
#endif
#ifndef ACL_GEMM_DMA_WAVES
#define ACL_GEMM_DMA_WAVES 3  // the 80-tile kernel's occupancy bound (waves per SIMD)
#endif
#ifndef ACL_GEMM_EDGE
#define ACL_GEMM_EDGE 1  // an edge tile skips its 16-blocks outside the matrix
#endif
#ifndef ACL_GEMM_TILE_DEFAULT
#define ACL_GEMM_TILE_DEFAULT 80  // the four-wave 80 tile
#endif

// op(A)[i][kk]: TA ? A[kk + i*lda] : A[i + kk*lda]
// op(B)[kk][j]: TB ? B[j + kk*ldb] : B[kk + j*ldb]
// TW = MFMA 16x16 tiles per wave per dimension: TW = 2 -> 64 x 64 output
// tile per workgroup, TW = 1 -> 32 x 32 (less padding on the ADMM's 392- and
// 196-sized products, but one accumulator per wave).
template <bool TA, bool TB, int TW, bool SYM>
__global__ void __launch_bounds__(256) gemm_f64_kernel(const GemmJob* __restrict__ jobs, int njobs,
                                                          int tm, int tiles,
                                                          unsigned long long* flops) {
  constexpr int TILE = 32 * TW;
  constexpr int EPT = TILE / 16;  // operand elements each thread stages per K step
  const int blk = blockIdx.x;
  const int slot = blk >> 3;
  const int job = (blk & 7) + 8 * (slot / tiles);
  if (job >= njobs) return;
  int t = slot % tiles, bi, bj;
  if (SYM) {  // upper-triangle tile t: row blocks bi <= bj
    bj = 0;
    while (t > bj) { t -= bj + 1; ++bj; }
    bi = t;
  } else {
    bi = t % tm;
    bj = t / tm;
  }
  const GemmJob J = jobs[job];
  if (J.skip && *J.skip) return;
  const int m0 = bi * TILE, n0 = bj * TILE;
  if (m0 >= J.m || n0 >= J.n) return;
  if (flops && threadIdx.x == 0)  // algorithmic flops of this tile (diagnostics)
    atomicAdd(flops, 2ull * (unsigned long long)min(TILE, J.m - m0) *
                         (unsigned long long)min(TILE, J.n - n0) * (unsigned long long)J.k);
  constexpr int PAD = TILE + 16;  // LDS row stride in doubles (bank shift)
  __shared__ double As[2][kGemmKStep][PAD];
  __shared__ double Bs[2][kGemmKStep][PAD];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  double ra[EPT], rb[EPT];
  auto a_idx = [&](int r, int& i, int& kk) {
    if (!TA) { i = tid % TILE; kk = tid / TILE + (256 / TILE) * r; }
    else     { kk = tid & 15; i = (tid >> 4) + 16 * r; }
  };
  auto b_idx = [&](int r, int& j, int& kb) {
    if (TB) { j = tid % TILE; kb = tid / TILE + (256 / TILE) * r; }
    else    { kb = tid & 15; j = (tid >> 4) + 16 * r; }
  };
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < EPT; ++r) {
      int i, kk;
      a_idx(r, i, kk);
      const int gi = m0 + i, gk = k0 + kk;
      ra[r] = (gi < J.m && gk < J.k)
                  ? (TA ? J.A[gk + (size_t)gi * J.lda] : J.A[gi + (size_t)gk * J.lda])
                  : 0.0;
      int j, kb;
      b_idx(r, j, kb);
      const int gj = n0 + j, gkb = k0 + kb;
      rb[r] = (gj < J.n && gkb < J.k)
                  ? (TB ? J.B[gj + (size_t)gkb * J.ldb] : J.B[gkb + (size_t)gj * J.ldb])
                  : 0.0;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int r = 0; r < EPT; ++r) {
      int i, kk;
      a_idx(r, i, kk);
      As[buf][kk][i] = ra[r];
      int j, kb;
      b_idx(r, j, kb);
      Bs[buf][kb][j] = rb[r];
    }
  };

  f64x4 acc[TW][TW];
#pragma unroll
  for (int a = 0; a < TW; ++a)
#pragma unroll
    for (int b = 0; b < TW; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};

  const int nk = (J.k + kGemmKStep - 1) / kGemmKStep;
  if (nk > 0) {
    load(0);
    store(0);
    __syncthreads();
  }
  for (int kb = 0; kb < nk; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nk) load((kb + 1) * kGemmKStep);
#pragma unroll
    for (int k4 = 0; k4 < kGemmKStep; k4 += 4) {
      const int kr = k4 + (lane >> 4);
      double av[TW], bv[TW];
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        av[t] = As[cur][kr][wm * 16 * TW + t * 16 + (lane & 15)];
        bv[t] = Bs[cur][kr][wn * 16 * TW + t * 16 + (lane & 15)];
      }
#pragma unroll
      for (int a = 0; a < TW; ++a)
#pragma unroll
        for (int b = 0; b < TW; ++b)
          // swapped operands: the MFMA tile is D^T, lane&15 runs along D's rows
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(bv[b], av[a], acc[a][b], 0, 0, 0);
    }
    if (kb + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  const double alpha = J.alpha, beta = J.beta;
#pragma unroll
  for (int a = 0; a < TW; ++a)
#pragma unroll
    for (int b = 0; b < TW; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = m0 + wm * 16 * TW + a * 16 + (lane & 15);
        const int gj = n0 + wn * 16 * TW + b * 16 + (lane >> 4) + 4 * r;
        if (gi < J.m && gj < J.n) {
          double v = alpha * acc[a][b][r];
          if (beta != 0.0) v += beta * J.C[gi + (size_t)gj * J.ldc];
          J.D[gi + (size_t)gj * J.ldd] = v;
          if (SYM && bi != bj) J.D[gj + (size_t)gi * J.ldd] = v;
        }
      }
}

// 80 x 80 output tile per 320-thread workgroup (five waves, wave w owns the
// 16-row block strip w: one A operand and five B operands per MFMA step).
// 80 = 5 x 16 fits the ADMM's 392-sized products with 2% padding (64-tiles
// pad them to 448: 23% of the MFMA work on zeros).
template <bool TA, bool TB, bool SYM>
__global__ void __launch_bounds__(320) gemm80_f64_kernel(const GemmJob* __restrict__ jobs, int njobs,
                                                           int tm, int tiles,
                                                           unsigned long long* flops) {
  constexpr int TILE = 80, NB = 5, EPT = 4;  // 2 x 80 x 16 operands / 320 threads = 4 + 4
  const int blk = blockIdx.x;
  const int slot = blk >> 3;
  const int job = (blk & 7) + 8 * (slot / tiles);
  if (job >= njobs) return;
  int t = slot % tiles, bi, bj;
  if (SYM) {
    bj = 0;
    while (t > bj) { t -= bj + 1; ++bj; }
    bi = t;
  } else {
    bi = t % tm;
    bj = t / tm;
  }
  const GemmJob J = jobs[job];
  if (J.skip && *J.skip) return;
  const int m0 = bi * TILE, n0 = bj * TILE;
  if (m0 >= J.m || n0 >= J.n) return;
  if (flops && threadIdx.x == 0)
    atomicAdd(flops, 2ull * (unsigned long long)min(TILE, J.m - m0) *
                         (unsigned long long)min(TILE, J.n - n0) * (unsigned long long)J.k);
  // LDS images, conflict-free for the MFMA operand reads (ds_read_b64 lane
  // groups 0-31 / 32-63, bank = dword mod 64) and the staging stores
  // (ds_write_b64 groups of 16 contiguous lanes, bank = dword mod 32):
  // an operand contiguous along i (j) in memory is staged k-major, rows of
  // 80 doubles (two k rows of 16 doubles land on disjoint bank halves); one
  // contiguous along k is staged i-major, rows of 18 doubles (16 i x 2 k in
  // a read group cover all 64 banks once), so 16 lanes store one row.
  constexpr bool AT = TA, BT = !TB;  // staged i-major (k contiguous in memory)
  constexpr int KM = TILE, IM = 18;  // row strides (doubles)
  constexpr int SZ = TILE * IM;      // >= kGemmKStep * KM
  __shared__ double Ash[2][SZ];
  __shared__ double Bsh[2][SZ];
  auto a_at = [&](int buf, int kk, int i) -> double& {
    return AT ? Ash[buf][i * IM + kk] : Ash[buf][kk * KM + i];
  };
  auto b_at = [&](int buf, int kk, int j) -> double& {
    return BT ? Bsh[buf][j * IM + kk] : Bsh[buf][kk * KM + j];
  };
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  double ra[EPT], rb[EPT];
  // staging maps: the contiguous dimension along the threads
  auto a_idx = [&](int r, int& i, int& kk) {
    if (!TA) { i = tid % TILE; kk = tid / TILE + 4 * r; }
    else     { kk = tid & 15; i = (tid >> 4) + 20 * r; }
  };
  auto b_idx = [&](int r, int& j, int& kb) {
    if (TB) { j = tid % TILE; kb = tid / TILE + 4 * r; }
    else    { kb = tid & 15; j = (tid >> 4) + 20 * r; }
  };
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < EPT; ++r) {
      int i, kk;
      a_idx(r, i, kk);
      const int gi = m0 + i, gk = k0 + kk;
      ra[r] = (gi < J.m && gk < J.k)
                  ? (TA ? J.A[gk + (size_t)gi * J.lda] : J.A[gi + (size_t)gk * J.lda])
                  : 0.0;
      int j, kb;
      b_idx(r, j, kb);
      const int gj = n0 + j, gkb = k0 + kb;
      rb[r] = (gj < J.n && gkb < J.k)
                  ? (TB ? J.B[gj + (size_t)gkb * J.ldb] : J.B[gkb + (size_t)gj * J.ldb])
                  : 0.0;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int r = 0; r < EPT; ++r) {
      int i, kk;
      a_idx(r, i, kk);
      a_at(buf, kk, i) = ra[r];
      int j, kb;
      b_idx(r, j, kb);
      b_at(buf, kb, j) = rb[r];
    }
  };
  f64x4 acc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = f64x4{0.0, 0.0, 0.0, 0.0};
  const int nk = (J.k + kGemmKStep - 1) / kGemmKStep;
  if (nk > 0) {
    load(0);
    store(0);
    __syncthreads();
  }
  for (int kb = 0; kb < nk; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nk) load((kb + 1) * kGemmKStep);
#pragma unroll
    for (int k4 = 0; k4 < kGemmKStep; k4 += 4) {
      const int kr = k4 + (lane >> 4);
      const double av = a_at(cur, kr, wave * 16 + (lane & 15));
      double bv[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) bv[b] = b_at(cur, kr, b * 16 + (lane & 15));
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(bv[b], av, acc[b], 0, 0, 0);
    }
    if (kb + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }
  const double alpha = J.alpha, beta = J.beta;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = m0 + wave * 16 + (lane & 15);
      const int gj = n0 + b * 16 + (lane >> 4) + 4 * r;
      if (gi < J.m && gj < J.n) {
        double v = alpha * acc[b][r];
        if (beta != 0.0) v += beta * J.C[gi + (size_t)gj * J.ldc];
        J.D[gi + (size_t)gj * J.ldd] = v;
        if (SYM && bi != bj) J.D[gj + (size_t)gi * J.ldd] = v;
      }
    }
}

// The 80 x 80 tile with four waves (256 threads), one per SIMD: five waves
// put two of a workgroup's MFMA streams on one SIMD. Wave w owns row strip w
// (five blocks), block (4, w) of strip 4, and block (4, 4) for the k rows of
// its own k4 step (k4 = w in every K step of 16): 25 MFMAs per wave per K
// step. The four partial (4, 4) accumulators are summed through LDS in wave
// order after the K loop.
template <bool TA, bool TB, bool SYM, bool DMA = false>
__global__ void __launch_bounds__(256, ACL_GEMM_DMA_WAVES) gemm80w4_f64_kernel(
    const GemmJob* __restrict__ jobs, int njobs, int tm, int tiles, unsigned long long* flops) {
  static_assert(!DMA || (!TA && !TB), "LDS-DMA staging: A and B untransposed only");
  constexpr int TILE = 80, NB = 5, EPT = 5;  // 80 x 16 operands / 256 threads = 5
  const int blk = blockIdx.x;
  const int slot = blk >> 3;
  const int job = (blk & 7) + 8 * (slot / tiles);
  if (job >= njobs) return;
  int t = slot % tiles, bi, bj;
  if (SYM) {
    bj = 0;
    while (t > bj) { t -= bj + 1; ++bj; }
    bi = t;
  } else {
    bi = t % tm;
    bj = t / tm;
  }
  GemmJob J = jobs[job];
  if (J.skip && *J.skip) return;
  if (J.gerr) {
    const double ge = *J.gerr;
    if (!(ge >= J.glo && ge < J.ghi)) return;
  }
  bool quint = false;
  if (J.qB) {
    const double qe = *J.nserr;
    if (qe >= J.qlo && qe < J.qhi) {
      quint = true;
      J.B = J.qB;
      J.tmask &= ~2;
    }
  }
  const int m0 = bi * TILE, n0 = bj * TILE;
  if (m0 >= J.m || n0 >= J.n) return;
  // a diagonal tile of a symmetric product: only the 15 blocks on and above
  // the block diagonal are computed (diag_blocks below), each one off the
  // diagonal stored twice
  const bool dtile = SYM && bi == bj;
  // an edge tile (ACL_GEMM_EDGE): only its row / column blocks inside the
  // matrix run their MFMAs (the others would multiply zero-filled operands
  // into outputs that are never stored); workgroup-uniform, so the K loops
  // are instantiated for edge and interior tiles apart
  const int mbk = min(5, (J.m - m0 + 15) >> 4), nbk = min(5, (J.n - n0 + 15) >> 4);
  const bool edge = ACL_GEMM_EDGE && (mbk < 5 || nbk < 5);
  if (flops && threadIdx.x == 0) {
    unsigned long long mn = 0;
    if (dtile) {
      for (int r = 0; r < NB; ++r)
        for (int c = r; c < NB; ++c)
          mn += (unsigned long long)max(0, min(16, J.m - m0 - 16 * r)) *
                (unsigned long long)max(0, min(16, J.n - n0 - 16 * c));
    } else {
      mn = (unsigned long long)min(TILE, J.m - m0) * (unsigned long long)min(TILE, J.n - n0);
    }
    atomicAdd(flops, 2ull * mn * (unsigned long long)J.k);
  }
  constexpr bool AT = TA, BT = !TB;  // staged i-major (k contiguous in memory)
  constexpr int KM = TILE, IM = 18;
  // DMA: dense images, A k-major [16][80], B as [80 columns][8 k-pairs] with
  // the pair slot xor-swizzled by the column, (kp ^ ((j >> 1) & 7)): the MFMA
  // reads (16 columns x 2 k of one pair per half-wave) hit 64 distinct banks
  constexpr int SZ = DMA ? TILE * kGemmKStep : TILE * IM;
  __shared__ __attribute__((aligned(16))) double Ash[2][SZ];
  __shared__ __attribute__((aligned(16))) double Bsh[2][SZ];
  auto a_at = [&](int buf, int kk, int i) -> double& {
    return AT ? Ash[buf][i * IM + kk] : Ash[buf][kk * KM + i];
  };
  auto b_at = [&](int buf, int kk, int j) -> double& {
    if constexpr (DMA) return Bsh[buf][2 * (j * 8 + ((kk >> 1) ^ ((j >> 1) & 7))) + (kk & 1)];
    return BT ? Bsh[buf][j * IM + kk] : Bsh[buf][kk * KM + j];
  };
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  double ra[EPT], rb[EPT];
  auto a_idx = [&](int r, int& i, int& kk) {
    const int e = tid + 256 * r;
    if (!TA) { i = e % TILE; kk = e / TILE; }
    else     { kk = e & 15; i = e >> 4; }
  };
  auto b_idx = [&](int r, int& j, int& kb) {
    const int e = tid + 256 * r;
    if (TB) { j = e % TILE; kb = e / TILE; }
    else    { kb = e & 15; j = e >> 4; }
  };
  const int tmask = J.tmask;
  const double tinv = tmask ? 1.0 / *J.tnrm : 1.0, tdiag = J.tdiag;
  // Operand staging. The loads go through global (address space 1) pointers,
  // unconditionally from clamped offsets: a flat load would count in lgkmcnt
  // too, so the LDS-read waits before the MFMAs would also wait for the next
  // K step's operands; bounds (zero fill) and the operand transform are
  // applied when the registers are written to LDS, after this step's MFMAs,
  // so nothing waits for the loads before then.
  typedef const __attribute__((address_space(1))) double gdouble;
  gdouble* const gA = (gdouble*)J.A;
  gdouble* const gB = (gdouble*)J.B;
  // elements r0 .. r1 - 1 of this thread's share (the K loop may stage a
  // step in two parts: fewer registers held across the MFMAs)
  auto load_part = [&](int k0, int r0, int r1) {
#pragma unroll
    for (int r = r0; r < r1; ++r) {
      int i, kk;
      a_idx(r, i, kk);
      const int gi = m0 + i, gk = k0 + kk;
      const bool ina = gi < J.m && gk < J.k;
      const size_t oa = ina ? (TA ? gk + (size_t)gi * J.lda : gi + (size_t)gk * J.lda) : 0;
      ra[r - r0] = gA[oa];
      int j, kb;
      b_idx(r, j, kb);
      const int gj = n0 + j, gkb = k0 + kb;
      const bool inb = gj < J.n && gkb < J.k;
      const size_t ob = inb ? (TB ? gj + (size_t)gkb * J.ldb : gkb + (size_t)gj * J.ldb) : 0;
      rb[r - r0] = gB[ob];
    }
  };
  auto store_part = [&](int buf, int k0, int r0, int r1) {
#pragma unroll
    for (int r = r0; r < r1; ++r) {
      int i, kk;
      a_idx(r, i, kk);
      const int gi = m0 + i, gk = k0 + kk;
      double va = (gi < J.m && gk < J.k) ? ra[r - r0] : 0.0;
      if ((tmask & 1) && gi < J.m && gk < J.k) va = (va - (gi == gk ? tdiag : 0.0)) * tinv;
      a_at(buf, kk, i) = va;
      int j, kb;
      b_idx(r, j, kb);
      const int gj = n0 + j, gkb = k0 + kb;
      double vb = (gj < J.n && gkb < J.k) ? rb[r - r0] : 0.0;
      if ((tmask & 2) && gj < J.n && gkb < J.k) vb = (vb - (gj == gkb ? tdiag : 0.0)) * tinv;
      b_at(buf, kb, j) = vb;
    }
  };
  auto load = [&](int k0) { load_part(k0, 0, EPT); };
  auto store = [&](int buf, int k0) { store_part(buf, k0, 0, EPT); };
  // LDS-DMA staging (DMA): a K step's operands are 20 pieces of 1 KiB (A:
  // 10 x 64 lanes x one pair of rows of one k; B: 10 x 64 lanes x one k-pair
  // of one column), wave w issuing pieces w + 4t, t < 5, as global_load_lds
  // (16 bytes per lane straight into LDS: no registers, no VALU beyond the
  // addresses). A lane outside the matrix (rows >= m, columns >= n, k >= K)
  // reads a 16-byte zero block instead. The loads are inline asm: the
  // compiler would otherwise wait for them before every LDS read (it cannot
  // tell the buffers apart); the K loop waits for them itself, before the
  // barrier that publishes a step's buffer.
  unsigned doff[5];
  int dkk[5];
  if constexpr (DMA) {
    const int wv = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int q = wv + 4 * t;
      if (q < 10) {
        const int u = q * 64 + lane, k = u / 40, row = m0 + 2 * (u % 40);
        doff[t] = (unsigned)(row + k * J.lda) * 8u;
        dkk[t] = row < J.m ? k : (1 << 28);
      } else {
        const int P = (q - 10) * 64 + lane, j = P >> 3, kp = (P & 7) ^ ((j >> 1) & 7);
        const int col = n0 + j;
        doff[t] = (unsigned)(2 * kp + col * J.ldb) * 8u;
        dkk[t] = col < J.n ? 2 * kp : (1 << 28);
      }
    }
  }
  auto dma = [&](int buf, int k0) {
    if constexpr (DMA) {
      const int wv = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const int q = wv + 4 * t;
        const bool isA = q < 10;  // wave-uniform
        const char* base = (const char*)(isA ? J.A : J.B);
        const unsigned step = isA ? (unsigned)(k0 * J.lda) * 8u : (unsigned)k0 * 8u;
        const void* src = k0 + dkk[t] < J.k ? (const void*)(base + doff[t] + step)
                                            : (const void*)g_gemm_zero16;
        const double* dst = isA ? &Ash[buf][q * 128] : &Bsh[buf][(q - 10) * 128];
        const unsigned lds = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) double*)dst;
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(lds)
            : "memory");
      }
    }
  };
  // the DMA K loop's wait: this wave's pieces have landed in LDS; for a job
  // with an operand transform (tmask: the Newton-Schulz start) each lane then
  // applies it to its own landed 16 bytes, as store_part does to a staged
  // element (the same expression: the same bits), before the barrier that
  // publishes the buffer
  auto dma_wait = [&](int buf, int k0) {
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tmask & 3) {  // workgroup-uniform
        const int wv = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const int q = wv + 4 * t;
          const bool isA = q < 10;
          if (!(tmask & (isA ? 1 : 2)) || !(k0 + dkk[t] < J.k)) continue;
          double* e = (isA ? &Ash[buf][q * 128] : &Bsh[buf][(q - 10) * 128]) + 2 * lane;
          int gi0, gk0, di, dk;  // element 0's (row, k); element 1 steps by (di, dk)
          if (isA) {
            const int u = q * 64 + lane;
            gi0 = m0 + 2 * (u % 40); gk0 = k0 + u / 40; di = 1; dk = 0;
          } else {
            const int P = (q - 10) * 64 + lane, j = P >> 3;
            gi0 = n0 + j; gk0 = k0 + dkk[t]; di = 0; dk = 1;
          }
#pragma unroll
          for (int h = 0; h < 2; ++h)
            e[h] = (e[h] - (gi0 + h * di == gk0 + h * dk ? tdiag : 0.0)) * tinv;
        }
      }
    }
  };
  const int nk = (J.k + kGemmKStep - 1) / kGemmKStep;
  // alpha, beta of the epilogue (the scaled Newton-Schulz update, the
  // quintic band)
  auto scales = [&](double& alpha, double& beta) {
    alpha = J.alpha;
    beta = J.beta;
    if (quint) {
      alpha = J.qalpha;
      beta = J.qbeta;
    } else if (J.nsp && !(*J.nserr < J.nstol)) {
      double tr = 0.0;
      for (int b = 0; b < J.nsn; ++b) tr += J.nsp[b];
      const double a = sqrt((double)J.m / tr);
      if (a == a) {
        const double ac = a < J.nscap ? a : J.nscap;
        alpha *= ac * ac * ac;
        beta *= ac;
      }
    }
  };
  // one element of D: gi = m0 + 16 si + (lane & 15), gj = n0 + 16 cb +
  // (lane >> 4) + 4 r; mirrored when `mir`. e2 = |D - I|_F^2 of this lane's
  // stored elements (J.err2), tr = its diagonal elements (J.trp), in put order
  auto put_at = [&](int si, int cb, int r, double a, bool mir, double alpha, double beta,
                    double& e2, double& tr) {
    const int gi = m0 + si * 16 + (lane & 15);
    const int gj = n0 + cb * 16 + (lane >> 4) + 4 * r;
    if (gi < J.m && gj < J.n) {
      double v = alpha * a;
      if (beta != 0.0) {
        double c = J.C[gi + (size_t)gj * J.ldc];
        if (tmask & 4) c = (c - (gi == gj ? tdiag : 0.0)) * tinv;
        v += beta * c;
      }
      J.D[gi + (size_t)gj * J.ldd] = v;
      if (mir) J.D[gj + (size_t)gi * J.ldd] = v;
      const double d = v - (gi == gj ? 1.0 : 0.0);
      e2 += mir ? 2.0 * (d * d) : d * d;
      if (gi == gj) tr += v;
    }
  };
  auto finish = [&](double e2, double tr) {
    if (J.err2) {  // the Newton-Schulz error of Y = Z^2, fused (no pass over Y)
      for (int o = 32; o > 0; o >>= 1) e2 += __shfl_xor(e2, o, 64);
      if (lane == 0) atomicAdd(J.err2, e2);
    }
    if (J.trp && bi == bj) {  // workgroup-uniform; the B buffer is free after the K loop
      for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o, 64);
      double* tw = &Bsh[0][0];
      if (lane == 0) tw[wave] = tr;
      __syncthreads();
      if (tid == 0) J.trp[bi] = ((tw[0] + tw[1]) + tw[2]) + tw[3];
    }
  };
  if (dtile) {
    // Diagonal tile: blocks (r, c), r <= c, dealt 4 / 4 / 4 / 3 over the
    // waves (diag_blocks), each block's full K on one wave; the blocks below
    // the diagonal are the mirrors of the ones above it
    auto diag = [&](auto WC, auto EC) {
      constexpr int W = decltype(WC)::value;
      constexpr bool EDGE = decltype(EC)::value;
      constexpr int NQ = W == 3 ? 3 : 4;
      constexpr int RB[4][4] = {{0, 0, 0, 0}, {1, 1, 1, 1}, {2, 2, 2, 0}, {3, 3, 4, 4}};
      constexpr int CB[4][4] = {{0, 1, 2, 3}, {1, 2, 3, 4}, {2, 3, 4, 4}, {3, 4, 4, 4}};
      f64x4 dacc[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) dacc[q] = f64x4{0.0, 0.0, 0.0, 0.0};
      auto dstep = [&](int cur) {
#pragma unroll
        for (int k4 = 0; k4 < kGemmKStep; k4 += 4) {
          const int kr = k4 + (lane >> 4);
#pragma unroll
          for (int q = 0; q < NQ; ++q)
            if (!EDGE || (RB[W][q] < mbk && CB[W][q] < nbk))
              dacc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                  b_at(cur, kr, CB[W][q] * 16 + (lane & 15)),
                  a_at(cur, kr, RB[W][q] * 16 + (lane & 15)), dacc[q], 0, 0, 0);
        }
      };
      if constexpr (DMA) {
        if (nk > 0) dma(0, 0);
        for (int kb = 0; kb < nk; ++kb) {
          const int cur = kb & 1;
          dma_wait(cur, kb * kGemmKStep);
          __syncthreads();  // step kb's pieces landed; step kb - 1's buffer free
          if (kb + 1 < nk) dma(cur ^ 1, (kb + 1) * kGemmKStep);
          dstep(cur);
        }
        __syncthreads();
      } else {
        if (nk > 0) {
          load(0);
          store(0, 0);
          __syncthreads();
        }
        for (int kb = 0; kb < nk; ++kb) {
          const int cur = kb & 1;
          if (kb + 1 < nk) load((kb + 1) * kGemmKStep);
          dstep(cur);
          if (kb + 1 < nk) store(cur ^ 1, (kb + 1) * kGemmKStep);
          __syncthreads();
        }
      }
      double alpha, beta;
      scales(alpha, beta);
      double e2 = 0.0, tr = 0.0;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          put_at(RB[W][q], CB[W][q], r, dacc[q][r], RB[W][q] != CB[W][q], alpha, beta, e2, tr);
      finish(e2, tr);
    };
#define ACL_DIAG(W_) \
  (edge ? diag(GemmWave<W_>{}, std::true_type{}) : diag(GemmWave<W_>{}, std::false_type{}))
    switch (__builtin_amdgcn_readfirstlane(wave)) {
      case 0: ACL_DIAG(0); break;
      case 1: ACL_DIAG(1); break;
      case 2: ACL_DIAG(2); break;
      default: ACL_DIAG(3); break;
    }
#undef ACL_DIAG
    return;
  }
  f64x4 acc[NB], acc4w = f64x4{0.0, 0.0, 0.0, 0.0}, acc44 = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = f64x4{0.0, 0.0, 0.0, 0.0};
  // The K loop, specialised per wave (ACL_GEMM_WSPEC): block (4, w)'s B
  // operand and the k4 step of block (4, 4) are then compile-time choices
  // (no selects, no exec-masked MFMA); ACL_GEMM_OPF: each k4 step's LDS
  // operands are read one step ahead, while the previous step's MFMAs run.
  auto kloop = [&](auto WC, auto EC) {
    constexpr int WS = decltype(WC)::value;  // -1: the wave index at run time
    constexpr bool EDGE = decltype(EC)::value;
    const int w = WS >= 0 ? WS : wave;
    struct Ops {
      double av, a4, bv[NB];
    };
    auto rd = [&](int cur, int k4, Ops& o) {
      const int kr = k4 + (lane >> 4);
      o.av = a_at(cur, kr, w * 16 + (lane & 15));
      o.a4 = a_at(cur, kr, 4 * 16 + (lane & 15));
#pragma unroll
      for (int b = 0; b < NB; ++b) o.bv[b] = b_at(cur, kr, b * 16 + (lane & 15));
    };
    auto mm = [&](int k4, const Ops& o) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (!EDGE || (w < mbk && b < nbk))
          acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.bv[b], o.av, acc[b], 0, 0, 0);
      if constexpr (WS >= 0) {
        if (!EDGE || (4 < mbk && WS < nbk))
          acc4w = __builtin_amdgcn_mfma_f64_16x16x4f64(o.bv[WS], o.a4, acc4w, 0, 0, 0);
        if (k4 == 4 * WS && (!EDGE || (4 < mbk && 4 < nbk)))  // block (4, 4) on this wave's k4 step
          acc44 = __builtin_amdgcn_mfma_f64_16x16x4f64(o.bv[4], o.a4, acc44, 0, 0, 0);
      } else {
        // block (4, w): B column block w (a wave-uniform index: select, no
        // dynamic register indexing)
        double bw = o.bv[0];
#pragma unroll
        for (int b = 1; b < 4; ++b) bw = wave == b ? o.bv[b] : bw;
        acc4w = __builtin_amdgcn_mfma_f64_16x16x4f64(bw, o.a4, acc4w, 0, 0, 0);
        if (k4 == 4 * wave)  // block (4, 4) on this wave's k4 step
          acc44 = __builtin_amdgcn_mfma_f64_16x16x4f64(o.bv[4], o.a4, acc44, 0, 0, 0);
      }
    };
    if constexpr (DMA) {
      if (nk > 0) dma(0, 0);
      for (int kb = 0; kb < nk; ++kb) {
        const int cur = kb & 1;
        dma_wait(cur, kb * kGemmKStep);
        __syncthreads();  // step kb's pieces landed; step kb - 1's buffer free
        if (kb + 1 < nk) dma(cur ^ 1, (kb + 1) * kGemmKStep);
        Ops o0, o1;
        rd(cur, 0, o0);
        rd(cur, 4, o1);
        mm(0, o0);
        rd(cur, 8, o0);
        mm(4, o1);
        rd(cur, 12, o1);
        mm(8, o0);
        mm(12, o1);
      }
      __syncthreads();
      return;
    }
    if (nk > 0) {
      load(0);
      store(0, 0);
      __syncthreads();
    }
    for (int kb = 0; kb < nk; ++kb) {
      const int cur = kb & 1;
      if (!ACL_GEMM_OPF && kb + 1 < nk) load((kb + 1) * kGemmKStep);
      if constexpr (ACL_GEMM_OPF) {
        // the next step staged in two parts (3 + 2 elements per thread):
        // the first stored to the other buffer mid-step, the second loaded then
        const int kn = (kb + 1) * kGemmKStep;
        const bool more = kb + 1 < nk;
        if (more) load_part(kn, 0, 3);
        Ops o0, o1;
        rd(cur, 0, o0);
        rd(cur, 4, o1);
        mm(0, o0);
        rd(cur, 8, o0);
        mm(4, o1);
        if (more) {
          store_part(cur ^ 1, kn, 0, 3);
          load_part(kn, 3, EPT);
        }
        rd(cur, 12, o1);
        mm(8, o0);
        mm(12, o1);
        if (more) store_part(cur ^ 1, kn, 3, EPT);
        __syncthreads();
        continue;
      } else {
#pragma unroll
        for (int k4 = 0; k4 < kGemmKStep; k4 += 4) {
          Ops o;
          rd(cur, k4, o);
          mm(k4, o);
        }
      }
      if (kb + 1 < nk) store(cur ^ 1, (kb + 1) * kGemmKStep);
      __syncthreads();
    }
  };
#define ACL_KLOOP(W_) \
  (edge ? kloop(GemmWave<W_>{}, std::true_type{}) : kloop(GemmWave<W_>{}, std::false_type{}))
  if constexpr (ACL_GEMM_WSPEC) {
    switch (__builtin_amdgcn_readfirstlane(wave)) {
      case 0: ACL_KLOOP(0); break;
      case 1: ACL_KLOOP(1); break;
      case 2: ACL_KLOOP(2); break;
      default: ACL_KLOOP(3); break;
    }
  } else {
    ACL_KLOOP(-1);
  }
#undef ACL_KLOOP
  // (4, 4): the four partial sums through LDS (the A buffer is free), added in
  // wave order
  double* red = &Ash[0][0];
#pragma unroll
  for (int r = 0; r < 4; ++r) red[(wave * 4 + r) * 64 + lane] = acc44[r];
  __syncthreads();
  double alpha, beta;
  scales(alpha, beta);
  double e2 = 0.0, tr = 0.0;
  const bool mir = SYM && bi != bj;
  auto put = [&](int si, int cb, int r, double a) { put_at(si, cb, r, a, mir, alpha, beta, e2, tr); };
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) put(wave, b, r, acc[b][r]);
#pragma unroll
  for (int r = 0; r < 4; ++r) put(4, wave, r, acc4w[r]);
  if (wave == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double x = red[(0 * 4 + r) * 64 + lane];
      x += red[(1 * 4 + r) * 64 + lane];
      x += red[(2 * 4 + r) * 64 + lane];
      x += red[(3 * 4 + r) * 64 + lane];
      put(4, 4, r, x);
    }
  }
  finish(e2, tr);
}

// Output tile per workgroup (build-time ACL_GEMM_TILE_DEFAULT, diagnostic
// builds only): 80 (default: four waves, gemm80w4_f64_kernel), 85 (the 80
// tile on five waves, gemm80_f64_kernel), 64 or 32. Measured on C5 (N=100,
// F=1024): 80 on four waves 278 ms per batch, on five 325 ms, 64 338 ms.
// Round 1 (before the symmetric products): 64 548 ms, 32 684 ms (the
// 32-tile wave holds one accumulator: less padding, but dependent MFMAs).
constexpr int gemm_tile() { return ACL_GEMM_TILE_DEFAULT; }
static_assert(gemm_tile() == 32 || gemm_tile() == 64 || gemm_tile() == 80 || gemm_tile() == 85,
              "ACL_GEMM_TILE_DEFAULT");

// output tile edge of the configured kernel (the symmetric path mirrors the
// tiles off the diagonal: post-processing may rely on that)
constexpr int gemm_tile_size() { return gemm_tile() == 85 ? 80 : gemm_tile(); }

// Host launcher: `jobs` is a device array of `njobs` descriptors whose m, n
// are bounded by mmax, nmax. sym: every job's D is symmetric in exact
// arithmetic (and square): upper-triangle tiles only, mirrored.
inline hipError_t gemm_f64(bool ta, bool tb, const GemmJob* jobs, int njobs, int mmax, int nmax,
                           hipStream_t s, unsigned long long* flops = nullptr, bool sym = false,
                           bool dma = false) {
  if (njobs <= 0 || mmax <= 0 || nmax <= 0) return hipSuccess;
  const int TT = gemm_tile(), T = TT == 85 ? 80 : TT;
  const int tm = (mmax + T - 1) / T, tn = (nmax + T - 1) / T;
  if (sym && tm != tn) return hipErrorInvalidValue;
  const int tiles = sym ? tm * (tm + 1) / 2 : tm * tn;
  const dim3 grid(8 * ((njobs + 7) / 8) * tiles);
#define ACL_GEMM_LAUNCH2(TA_, TB_, SYM_)                                                   \
  do {                                                                                     \
    if (TT == 80 && ACL_GEMM_DMA && dma && !TA_ && !TB_)                                   \
      hipLaunchKernelGGL((gemm80w4_f64_kernel<false, false, SYM_, true>), grid, dim3(256), 0, s, \
                         jobs, njobs, tm, tiles, flops);                                   \
    else if (TT == 80)                                                                     \
      hipLaunchKernelGGL((gemm80w4_f64_kernel<TA_, TB_, SYM_>), grid, dim3(256), 0, s, jobs, \
                         njobs, tm, tiles, flops);                                         \
    else if (TT == 85)                                                                     \
      hipLaunchKernelGGL((gemm80_f64_kernel<TA_, TB_, SYM_>), grid, dim3(320), 0, s, jobs,  \
                         njobs, tm, tiles, flops);                                         \
    else if (T == 64)                                                                      \
      hipLaunchKernelGGL((gemm_f64_kernel<TA_, TB_, 2, SYM_>), grid, dim3(256), 0, s, jobs, \
                         njobs, tm, tiles, flops);                                         \
    else                                                                                   \
      hipLaunchKernelGGL((gemm_f64_kernel<TA_, TB_, 1, SYM_>), grid, dim3(256), 0, s, jobs, \
                         njobs, tm, tiles, flops);                                         \
  } while (0)
#define ACL_GEMM_LAUNCH(TA_, TB_)                       \
  do {                                                  \
    if (sym) ACL_GEMM_LAUNCH2(TA_, TB_, true);          \
    else ACL_GEMM_LAUNCH2(TA_, TB_, false);             \
  } while (0)
  if (!ta && !tb) ACL_GEMM_LAUNCH(false, false);
  else if (!ta && tb) ACL_GEMM_LAUNCH(false, true);
  else if (ta && !tb) ACL_GEMM_LAUNCH(true, false);
  else ACL_GEMM_LAUNCH(true, true);
#undef ACL_GEMM_LAUNCH
#undef ACL_GEMM_LAUNCH2
  return hipGetLastError();
}

}  // namespace acl_amd
