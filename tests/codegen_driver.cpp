// codegen_driver.cpp -- drives the codegen-compatible ADMM entry points the
// way the reference's ADMM wrapper does (aclswarm/src/admm.cpp:13-48: one
// initialize, an emxInit'd 2-D result, wrappers around the caller's points
// and adjacency, the design, frees), built against include/codegen_admm/ --
// the header names admm.h includes (admm.h:16-20) -- and linked to
// libaclswarm_amd_codegen.so (over libaclswarm_amd.so). tests/test_gpu_codegen.py calls codegen_run through
// ctypes; tests/test_abi.py compiles it and checks the exported names.
#include <ADMMGainDesign3D.h>
#include <ADMMGainDesign3D_emxAPI.h>
#include <ADMMGainDesign3D_emxutil.h>
#include <ADMMGainDesign3D_initialize.h>
#include <ADMMGainDesign3D_terminate.h>

#include <cstring>
#include <vector>

// p: n x 3 row-major (PtsMat rows), adjmat: n x n 0/1 bytes. gains: 3n x 3n
// column-major out. Returns the result's rows (3n), or 0 with rows/cols of
// the (empty) result in dims when the design failed.
extern "C" int codegen_run(int n, const double* p, const unsigned char* adjmat, double* gains,
                           int* dims) {
  ADMMGainDesign3D_initialize();
  emxArray_real_T* Aopt = nullptr;
  emxInit_real_T(&Aopt, 2);
  // p.transpose() as a 3 x n column-major matrix, adjmat cast to double
  std::vector<double> pp((size_t)3 * n), a((size_t)n * n);
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < 3; ++r) pp[(size_t)r + 3 * i] = p[(size_t)3 * i + r];
  for (size_t k = 0; k < a.size(); ++k) a[k] = adjmat[k] ? 1.0 : 0.0;
  emxArray_real_T* Qs = emxCreateWrapper_real_T(pp.data(), 3, n);
  emxArray_real_T* adj = emxCreateWrapper_real_T(a.data(), n, n);
  ADMMGainDesign3D(Qs, adj, Aopt);
  emxFree_real_T(&adj);
  emxFree_real_T(&Qs);
  dims[0] = Aopt->size[0];
  dims[1] = Aopt->size[1];
  const int rows = Aopt->size[0];
  if (rows == 3 * n && Aopt->size[1] == 3 * n)
    std::memcpy(gains, Aopt->data, sizeof(double) * (size_t)rows * rows);
  emxFree_real_T(&Aopt);
  ADMMGainDesign3D_terminate();
  return rows == 3 * n ? rows : 0;
}

// a malformed call (Qs 2 x n): the result is empty, nothing is thrown
extern "C" int codegen_bad_call(int n) {
  emxArray_real_T* Aopt = emxCreate_real_T(1, 1);
  std::vector<double> pp((size_t)2 * n), a((size_t)n * n);
  emxArray_real_T* Qs = emxCreateWrapper_real_T(pp.data(), 2, n);
  emxArray_real_T* adj = emxCreateWrapper_real_T(a.data(), n, n);
  ADMMGainDesign3D(Qs, adj, Aopt);
  const int r = Aopt->size[0] + Aopt->size[1];
  emxDestroyArray_real_T(Qs);
  emxDestroyArray_real_T(adj);
  emxDestroyArray_real_T(Aopt);
  return r;
}
