// common.h -- device helpers shared by the auction and control kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace acl_amd {

constexpr double kPi = 3.14159265358979323846;

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

__device__ __forceinline__ unsigned wave_or_u32(unsigned ux) {
  int x = (int)ux;
#define ACL_UOR(a, b) ((a) | (b))
  ACL_DPP_STEP(x, ACL_UOR, 0xB1, 0xF);
  ACL_DPP_STEP(x, ACL_UOR, 0x4E, 0xF);
  ACL_DPP_STEP(x, ACL_UOR, 0x124, 0xF);
  ACL_DPP_STEP(x, ACL_UOR, 0x128, 0xF);
  ACL_DPP_STEP(x, ACL_UOR, 0x142, 0xA);
  ACL_DPP_STEP(x, ACL_UOR, 0x143, 0xC);
#undef ACL_UOR
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

}  // namespace acl_amd
