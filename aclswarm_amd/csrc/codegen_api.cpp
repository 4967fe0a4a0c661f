// codegen_api.cpp -- the MATLAB-Coder entry points of the reference's ADMM
// gain design (include/aclswarm_amd_codegen.h) over acl_admm_solve_batch.
//
// The reference's ADMM wrapper (aclswarm/src/admm.cpp:13-48) drives the
// generated library through five calls: ADMMGainDesign3D_initialize, emxInit_
// real_T for the 3n x 3n result, emxCreateWrapper_real_T around its Eigen
// inputs, ADMMGainDesign3D, emxFree_real_T. These are the same functions with
// C++ linkage; the design itself is one formation of the batched solver
// (default parameters, LINPACK basis: the codegen's gains), synchronous on
// the default stream of the current device. Host code only, built into its
// own library (libaclswarm_amd_codegen.so, linked to libaclswarm_amd.so): the
// generic emx utility names stay out of the core library's exports.
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/aclswarm_amd.h"
#include "../../include/aclswarm_amd_codegen.h"

extern "C" acl_status_t acl__set_error(const char* msg);

namespace {

emxArray_real_T* emx_new(int numDimensions) {
  emxArray_real_T* a = static_cast<emxArray_real_T*>(std::malloc(sizeof(emxArray_real_T)));
  if (!a) return nullptr;
  const int nd = numDimensions > 0 ? numDimensions : 1;
  a->data = nullptr;
  a->size = static_cast<int*>(std::calloc((size_t)nd, sizeof(int)));
  a->allocatedSize = 0;
  a->numDimensions = numDimensions;
  a->canFreeData = true;
  return a;
}

size_t emx_numel(int numDimensions, const int* size) {
  size_t k = 1;
  for (int i = 0; i < numDimensions; ++i) k *= (size_t)(size[i] > 0 ? size[i] : 0);
  return k;
}

// Aopt as rows x cols, its data (re)allocated when it owns too little
bool emx_resize2(emxArray_real_T* a, int rows, int cols) {
  if (!a || !a->size || a->numDimensions < 2) return false;
  const size_t need = (size_t)rows * (size_t)cols;
  if (need > (size_t)a->allocatedSize || !a->data) {
    if (!a->canFreeData && a->data) return false;  // a wrapper cannot grow
    double* d = static_cast<double*>(std::malloc(need ? need * sizeof(double) : sizeof(double)));
    if (!d) return false;
    if (a->data && a->canFreeData) std::free(a->data);
    a->data = d;
    a->allocatedSize = (int)need;
    a->canFreeData = true;
  }
  a->size[0] = rows;
  a->size[1] = cols;
  for (int i = 2; i < a->numDimensions; ++i) a->size[i] = 1;
  return true;
}

void emx_empty(emxArray_real_T* a) {
  if (!a || !a->size) return;
  for (int i = 0; i < a->numDimensions; ++i) a->size[i] = 0;
}

}  // namespace

void ADMMGainDesign3D_initialize() {}
void ADMMGainDesign3D_terminate() {}

void emxInit_real_T(emxArray_real_T** pEmxArray, int numDimensions) {
  if (pEmxArray) *pEmxArray = emx_new(numDimensions);
}

void emxInitArray_real_T(emxArray_real_T** pEmxArray, int numDimensions) {
  emxInit_real_T(pEmxArray, numDimensions);
}

void emxFree_real_T(emxArray_real_T** pEmxArray) {
  if (!pEmxArray || !*pEmxArray) return;
  emxArray_real_T* a = *pEmxArray;
  if (a->data && a->canFreeData) std::free(a->data);
  std::free(a->size);
  std::free(a);
  *pEmxArray = nullptr;
}

void emxDestroyArray_real_T(emxArray_real_T* emxArray) { emxFree_real_T(&emxArray); }

emxArray_real_T* emxCreateND_real_T(int numDimensions, const int* size) {
  emxArray_real_T* a = emx_new(numDimensions);
  if (!a) return nullptr;
  for (int i = 0; i < numDimensions; ++i) a->size[i] = size[i];
  const size_t k = emx_numel(numDimensions, size);
  a->data = static_cast<double*>(std::calloc(k ? k : 1, sizeof(double)));
  a->allocatedSize = (int)k;
  return a;
}

emxArray_real_T* emxCreate_real_T(int rows, int cols) {
  const int sz[2] = {rows, cols};
  return emxCreateND_real_T(2, sz);
}

emxArray_real_T* emxCreateWrapperND_real_T(double* data, int numDimensions, const int* size) {
  emxArray_real_T* a = emx_new(numDimensions);
  if (!a) return nullptr;
  for (int i = 0; i < numDimensions; ++i) a->size[i] = size[i];
  a->data = data;
  a->allocatedSize = (int)emx_numel(numDimensions, size);
  a->canFreeData = false;
  return a;
}

emxArray_real_T* emxCreateWrapper_real_T(double* data, int rows, int cols) {
  const int sz[2] = {rows, cols};
  return emxCreateWrapperND_real_T(data, 2, sz);
}

void ADMMGainDesign3D(const emxArray_real_T* Qs, const emxArray_real_T* adj, emxArray_real_T* Aopt) {
  // the inputs of admm.cpp:34-40: Qs = p^T (3 x n), adj (n x n) as doubles
  if (!Qs || !adj || !Aopt || !Qs->data || !adj->data || Qs->numDimensions != 2 ||
      adj->numDimensions != 2 || Qs->size[0] != 3 || Qs->size[1] < 1 ||
      adj->size[0] != Qs->size[1] || adj->size[1] != Qs->size[1]) {
    acl__set_error("ADMMGainDesign3D: Qs must be 3 x n and adj n x n");
    emx_empty(Aopt);
    return;
  }
  const int n = Qs->size[1], N3 = 3 * n;
  if (!emx_resize2(Aopt, N3, N3)) {
    acl__set_error("ADMMGainDesign3D: cannot size Aopt to 3n x 3n");
    emx_empty(Aopt);
    return;
  }
  // [3][n] column-major points and [n][n] adjacency are the batched layouts
  // of one formation (acl_admm_solve_batch); the gains come back 3n x 3n
  // column-major, the GainMat Aopt holds
  const size_t bp = (size_t)3 * n * sizeof(double), ba = (size_t)n * n * sizeof(double),
               bg = (size_t)N3 * N3 * sizeof(double);
  void *dp = nullptr, *da = nullptr, *dg = nullptr, *di = nullptr;
  int32_t it[2] = {0, 0};
  acl_admm_params_t prm;
  acl_default_admm_params(&prm);
  prm.basis = ACL_ADMM_BASIS_LINPACK;
  const bool ok = acl_malloc(&dp, bp) == ACL_OK && acl_malloc(&da, ba) == ACL_OK &&
                  acl_malloc(&dg, bg) == ACL_OK && acl_malloc(&di, sizeof(it)) == ACL_OK &&
                  acl_memcpy_h2d(dp, Qs->data, bp, nullptr) == ACL_OK &&
                  acl_memcpy_h2d(da, adj->data, ba, nullptr) == ACL_OK &&
                  acl_admm_solve_batch(1, n, static_cast<const double*>(dp),
                                       static_cast<const double*>(da), static_cast<double*>(dg),
                                       static_cast<int32_t*>(di), &prm, nullptr) == ACL_OK &&
                  acl_memcpy_d2h(Aopt->data, dg, bg, nullptr) == ACL_OK &&
                  acl_memcpy_d2h(it, di, sizeof(it), nullptr) == ACL_OK &&
                  acl_stream_synchronize(nullptr) == ACL_OK;
  if (dp) acl_free(dp);
  if (da) acl_free(da);
  if (dg) acl_free(dg);
  if (di) acl_free(di);
  if (!ok) {
    emx_empty(Aopt);  // acl_last_error() holds the failing call's message
  } else if (it[0] < 0 || it[1] < 0) {
    // a PSD projection left unconverged (include/aclswarm_amd.h: negative
    // iters): the generated library has no error channel, so the design is
    // withheld (Aopt empty, as for the other failures) and the reason kept
    acl__set_error("ADMMGainDesign3D: a PSD projection did not converge (Jacobi fallback "
                   "exhausted); the gains are not reliable");
    emx_empty(Aopt);
  }
}
