// control_params.h -- parameters of the control kernel (control.hip),
// filled by acl_solve_batch (solve.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/aclswarm_amd.h"

namespace acl_amd {

struct CtlParams {
  int n, B, b0;
  const double* p;
  const uint64_t* adj;
  const double* gains;
  const int64_t* gain_off;
  const int32_t* fidx;
  const double* q;
  const double* vel;
  const uint16_t* P_out;
  acl_swarm_status_t* status;
  double* u;        // DistCntrl output: the caller's u, or workspace scratch
  double* u_safe;
  uint8_t* ca_flag;
  const unsigned char* ws;
  acl_cntrl_gains_t g;
  acl_safety_params_t s;
};

// Control stage of chunk [P.b0, P.b0 + nb): which = 0 launches the gain
// kernel (DistCntrl::compute, the HBM stream), 1 the safety kernel
// (saturation + collision avoidance).
hipError_t launch_control(const CtlParams& P, int nb, int which, hipStream_t stream);

// Byte offset of the f64 u scratch inside the solve workspace.
__host__ __device__ inline size_t ws_u_offset(int n, int B) {
  return ((size_t)B * ((size_t)n + 1 + (size_t)n * n) + 255) & ~(size_t)255;
}

}  // namespace acl_amd
