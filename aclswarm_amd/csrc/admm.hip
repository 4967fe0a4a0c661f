// admm.hip -- batched ADMM formation-gain design (admm::Solver::solve,
// aclswarm/lib/admm/src/solver.cpp:28-79). Filled in by the ADMM milestone.
#include <hip/hip_runtime.h>
#include "../../include/aclswarm_amd.h"

extern "C" acl_status_t acl__set_error(const char* msg);

extern "C" acl_status_t acl_admm_solve_batch(int32_t F, int32_t n, const double* pts,
                                             const double* adj, double* gains, int32_t* iters,
                                             const acl_admm_params_t* params, void* stream) {
  (void)F; (void)n; (void)pts; (void)adj; (void)gains; (void)iters; (void)params; (void)stream;
  acl__set_error("acl_admm_solve_batch: not built yet");
  return ACL_ERR_UNSUPPORTED;
}
