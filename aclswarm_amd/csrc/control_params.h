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
  double* u;
  double* u_safe;
  uint8_t* ca_flag;
  const unsigned char* ws;
  acl_cntrl_gains_t g;
  acl_safety_params_t s;
};

hipError_t launch_control(const CtlParams& P, int nb, hipStream_t stream);

}  // namespace acl_amd
