// admm_ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// A C entry point over the reference's MATLAB-Coder ADMM gain design
// (aclswarm/lib/codegen_admm, compiled from the sources where they lie by
// oracle/Makefile `ref`, output oracle/_ref/libadmm_ref.so). Mirrors the
// reference wrapper ADMM::calculateFormationGains (aclswarm/src/admm.cpp:32-51):
// pts is the 3 x n column-major formation (p^T), adj the n x n adjacency as
// doubles, Aopt the 3n x 3n column-major gain matrix; |a| < 1e-10 is zeroed
// when `prune` is set (admm.cpp:50).
#include <cmath>
#include <cstring>

#include "ADMMGainDesign3D.h"
#include "ADMMGainDesign3D_emxAPI.h"
#include "ADMMGainDesign3D_initialize.h"
#include "ADMMGainDesign3D_terminate.h"
#include "svd.h"

// rt_InitInfAndNaN runs in ADMMGainDesign3D_initialize: until then rtInf and
// rtNaN are 0.0, and the codegen's finiteness checks misfire on zeros.
static void ensure_init() {
  static bool init = false;
  if (!init) {
    ADMMGainDesign3D_initialize();
    init = true;
  }
}

extern "C" int admm_ref_solve(int n, const double* pts, const double* adj, double* Aopt,
                              int prune) {
  ensure_init();
  emxArray_real_T* Qs = emxCreateWrapper_real_T(const_cast<double*>(pts), 3, n);
  emxArray_real_T* A = emxCreateWrapper_real_T(const_cast<double*>(adj), n, n);
  emxArray_real_T* out = nullptr;
  emxInitArray_real_T(&out, 2);
  ADMMGainDesign3D(Qs, A, out);
  int rc = 0;
  if (out->size[0] != 3 * n || out->size[1] != 3 * n) {
    rc = -1;
  } else {
    const size_t N = (size_t)9 * n * n;
    for (size_t k = 0; k < N; ++k) {
      const double a = out->data[k];
      Aopt[k] = (prune && !(1e-10 < std::fabs(a))) ? 0.0 : a;
    }
  }
  emxDestroyArray_real_T(out);
  emxDestroyArray_real_T(A);
  emxDestroyArray_real_T(Qs);
  return rc;
}

// U of the codegen's LINPACK-style svd (svd.cpp: `svd` for rows x 4 kernels,
// `c_svd` for rows x 1..2), for pinning the kernel-complement basis Q.
extern "C" int admm_ref_svd_u(int rows, int cols, const double* N, double* U) {
  ensure_init();
  emxArray_real_T* A = emxCreateWrapper_real_T(const_cast<double*>(N), rows, cols);
  emxArray_real_T* u = nullptr;
  emxArray_real_T* s = nullptr;
  emxInitArray_real_T(&u, 2);
  emxInitArray_real_T(&s, 2);
  if (cols == 4) {
    double V[16];
    svd(A, u, s, V);
  } else {
    double V[4];
    int vs[2];
    c_svd(A, u, s, V, vs);
  }
  if (u->size[0] != rows || u->size[1] != rows) return 100 * u->size[0] + u->size[1];
  std::memcpy(U, u->data, sizeof(double) * rows * rows);
  emxDestroyArray_real_T(s);
  emxDestroyArray_real_T(u);
  emxDestroyArray_real_T(A);
  return 0;
}
