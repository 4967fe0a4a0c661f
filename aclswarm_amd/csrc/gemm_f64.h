// gemm_f64.h -- batched fp64 GEMM on CDNA4 matrix cores (v_mfma_f64_16x16x4_f64).
//
// D = alpha * op(A) * op(B) + beta * C, column-major, one descriptor per
// batch entry (dims, leading dimensions, pointers and an optional skip flag
// live in device memory, so a setup kernel may fill them and converged
// problems drop out without a host round trip).
//
// Tiling: 64 x 64 output tile per 256-thread workgroup, four waves in a 2 x 2
// arrangement, each wave 2 x 2 MFMA 16x16 tiles; K staged through LDS in
// steps of 16 with a register-prefetched double buffer (one barrier per step).
// The MFMA is issued with the operands swapped (it computes the tile of D^T),
// so the accumulator's lane index runs along D's rows and every epilogue
// load/store is a contiguous 128-byte column segment.
#pragma once

#include <hip/hip_runtime.h>

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
};

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kGemmTile = 64;
constexpr int kGemmKStep = 16;
constexpr int kGemmPad = 80;  // LDS row stride in doubles: 160 words = 32 banks shift

// op(A)[i][kk]: TA ? A[kk + i*lda] : A[i + kk*lda]
// op(B)[kk][j]: TB ? B[j + kk*ldb] : B[kk + j*ldb]
template <bool TA, bool TB>
__global__ void __launch_bounds__(256) gemm_f64_kernel(const GemmJob* __restrict__ jobs,
                                                          unsigned long long* flops) {
  const GemmJob J = jobs[blockIdx.z];
  if (J.skip && *J.skip) return;
  const int m0 = blockIdx.x * kGemmTile, n0 = blockIdx.y * kGemmTile;
  if (m0 >= J.m || n0 >= J.n) return;
  if (flops && threadIdx.x == 0)  // algorithmic flops of this tile (diagnostics)
    atomicAdd(flops, 2ull * (unsigned long long)min(kGemmTile, J.m - m0) *
                         (unsigned long long)min(kGemmTile, J.n - n0) * (unsigned long long)J.k);
  __shared__ double As[2][kGemmKStep][kGemmPad];
  __shared__ double Bs[2][kGemmKStep][kGemmPad];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  double ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int i, kk;
      if (!TA) { i = tid & 63; kk = (tid >> 6) + 4 * r; }
      else     { kk = tid & 15; i = (tid >> 4) + 16 * r; }
      const int gi = m0 + i, gk = k0 + kk;
      ra[r] = (gi < J.m && gk < J.k)
                  ? (TA ? J.A[gk + (size_t)gi * J.lda] : J.A[gi + (size_t)gk * J.lda])
                  : 0.0;
      int j, kb;
      if (TB) { j = tid & 63; kb = (tid >> 6) + 4 * r; }
      else    { kb = tid & 15; j = (tid >> 4) + 16 * r; }
      const int gj = n0 + j, gkb = k0 + kb;
      rb[r] = (gj < J.n && gkb < J.k)
                  ? (TB ? J.B[gj + (size_t)gkb * J.ldb] : J.B[gkb + (size_t)gj * J.ldb])
                  : 0.0;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      int i, kk;
      if (!TA) { i = tid & 63; kk = (tid >> 6) + 4 * r; }
      else     { kk = tid & 15; i = (tid >> 4) + 16 * r; }
      As[buf][kk][i] = ra[r];
      int j, kb;
      if (TB) { j = tid & 63; kb = (tid >> 6) + 4 * r; }
      else    { kb = tid & 15; j = (tid >> 4) + 16 * r; }
      Bs[buf][kb][j] = rb[r];
    }
  };

  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};

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
      double av[2], bv[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        av[t] = As[cur][kr][wm * 32 + t * 16 + (lane & 15)];
        bv[t] = Bs[cur][kr][wn * 32 + t * 16 + (lane & 15)];
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          // swapped operands: the MFMA tile is D^T, lane&15 runs along D's rows
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(bv[b], av[a], acc[a][b], 0, 0, 0);
    }
    if (kb + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  const double alpha = J.alpha, beta = J.beta;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = m0 + wm * 32 + a * 16 + (lane & 15);
        const int gj = n0 + wn * 32 + b * 16 + (lane >> 4) + 4 * r;
        if (gi < J.m && gj < J.n) {
          double v = alpha * acc[a][b][r];
          if (beta != 0.0) v += beta * J.C[gi + (size_t)gj * J.ldc];
          J.D[gi + (size_t)gj * J.ldd] = v;
        }
      }
}

// Host launcher: `jobs` is a device array of `njobs` descriptors whose m, n
// are bounded by mmax, nmax.
inline hipError_t gemm_f64(bool ta, bool tb, const GemmJob* jobs, int njobs, int mmax, int nmax,
                           hipStream_t s, unsigned long long* flops = nullptr) {
  if (njobs <= 0 || mmax <= 0 || nmax <= 0) return hipSuccess;
  const dim3 grid((mmax + kGemmTile - 1) / kGemmTile, (nmax + kGemmTile - 1) / kGemmTile, njobs);
  if (!ta && !tb) hipLaunchKernelGGL((gemm_f64_kernel<false, false>), grid, dim3(256), 0, s, jobs, flops);
  else if (!ta && tb) hipLaunchKernelGGL((gemm_f64_kernel<false, true>), grid, dim3(256), 0, s, jobs, flops);
  else if (ta && !tb) hipLaunchKernelGGL((gemm_f64_kernel<true, false>), grid, dim3(256), 0, s, jobs, flops);
  else hipLaunchKernelGGL((gemm_f64_kernel<true, true>), grid, dim3(256), 0, s, jobs, flops);
  return hipGetLastError();
}

}  // namespace acl_amd
