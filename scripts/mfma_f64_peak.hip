// fp64 MFMA throughput microbenchmark (no memory traffic): v_mfma_f64_16x16x4f64 chains,
// NACC independent accumulators per wave. Build: hipcc -O3 --offload-arch=gfx950
// scripts/mfma_f64_peak.hip -o mfma_f64_peak; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ void __launch_bounds__(256) k(double* out, int iters) {
  f64x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f64x4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int NACC>
void run(int blocks, int iters) {
  double* d; hipMalloc(&d, blocks * 256 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k<NACC><<<blocks, 256>>>(d, 10); hipDeviceSynchronize();
  hipEventRecord(e0); k<NACC><<<blocks, 256>>>(d, iters); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double flops = 2.0 * 16 * 16 * 4 * (double)NACC * iters * blocks * 4;
  printf("NACC=%d blocks=%d: %.3f ms, %.1f TF/s, cycles/MFMA/SIMD at 2.4GHz: %.1f\n", NACC, blocks, ms, flops / ms / 1e9,
         (ms * 1e-3 * 2.4e9) / ((double)NACC * iters * blocks * 4 / 1024.0));
  hipFree(d);
}
int main() {
  // short runs (the round-4 first measurement) under-read: the clock settles
  // over ~10 ms, and 3 waves per SIMD do not keep the pipe full
  run<8>(256 * 3, 1000); run<8>(256 * 3, 10000); run<8>(256 * 3, 20000);
  run<4>(256 * 6, 10000); run<8>(256 * 6, 10000); run<4>(256 * 8, 10000);
  run<2>(256 * 8, 20000); run<8>(256 * 3, 10000);
  return 0;
}
