/* aclswarm_amd_codegen.h -- the MATLAB-Coder entry points of the reference's
 * ADMM gain design, served by the batched GPU solver.
 *
 * The reference's ADMM wrapper (aclswarm/src/admm.cpp:13-48, class ADMM)
 * calls the generated library lib/codegen_admm (ADMMGainDesign3D.h:22-23,
 * ADMMGainDesign3D_emxAPI.h:22-28, ADMMGainDesign3D_emxutil.h:37,43,
 * ADMMGainDesign3D_initialize.h:22, ADMMGainDesign3D_terminate.h:22). Those
 * are C++ functions (the generated sources are .cpp, so the names carry C++
 * linkage) over MATLAB's emxArray_real_T. This header declares the same
 * functions with the same signatures and the same struct layout, so admm.cpp
 * compiles and links unchanged against libaclswarm_amd.so instead of the
 * generated library: point its include path at include/codegen_admm/ (the
 * five header names admm.h includes, each forwarding here) and link
 * aclswarm_amd instead of the codegen target.
 *
 * ADMMGainDesign3D(Qs, adj, Aopt): Qs 3 x n column-major points, adj n x n
 * column-major 0/1 (symmetric), Aopt resized to 3n x 3n and filled with the
 * gain matrix column-major -- acl_admm_solve_batch on one formation with
 * the default parameters (solver.h:18-31) and the LINPACK basis, i.e. the
 * codegen's gains, on the current HIP device, synchronously.
 * Errors (the generated code has none): Aopt becomes 0 x 0 and
 * acl_last_error() says why.
 */
#ifndef ACLSWARM_AMD_CODEGEN_H
#define ACLSWARM_AMD_CODEGEN_H

#ifndef __cplusplus
#error "the codegen entry points have C++ linkage, like the generated library"
#endif

/* MATLAB Coder's dynamic array of doubles (ADMMGainDesign3D_types.h:45-52) */
#ifndef struct_emxArray_real_T
#define struct_emxArray_real_T
struct emxArray_real_T {
  double* data;
  int* size;
  int allocatedSize;
  int numDimensions;
  bool canFreeData;
};
#endif
#ifndef typedef_emxArray_real_T
#define typedef_emxArray_real_T
typedef emxArray_real_T emxArray_real_T;
#endif

void ADMMGainDesign3D_initialize();
void ADMMGainDesign3D_terminate();
void ADMMGainDesign3D(const emxArray_real_T* Qs, const emxArray_real_T* adj, emxArray_real_T* Aopt);

/* emx utilities: an empty array of numDimensions (data NULL, sizes 0) ... */
void emxInit_real_T(emxArray_real_T** pEmxArray, int numDimensions);
void emxInitArray_real_T(emxArray_real_T** pEmxArray, int numDimensions);
/* ... freed with its data when it owns it (canFreeData), *pEmxArray = NULL */
void emxFree_real_T(emxArray_real_T** pEmxArray);
void emxDestroyArray_real_T(emxArray_real_T* emxArray);
/* owning arrays, zero-filled */
emxArray_real_T* emxCreate_real_T(int rows, int cols);
emxArray_real_T* emxCreateND_real_T(int numDimensions, const int* size);
/* wrappers of caller memory (never freed by the array) */
emxArray_real_T* emxCreateWrapper_real_T(double* data, int rows, int cols);
emxArray_real_T* emxCreateWrapperND_real_T(double* data, int numDimensions, const int* size);

#endif /* ACLSWARM_AMD_CODEGEN_H */
