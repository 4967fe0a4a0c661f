// api.cpp -- host side of the C ABI: defaults, error string, packing of the
// reference's Eigen layouts into the device layout, device-memory helpers.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>
#include <cstring>
#include <string>

#include "../../include/aclswarm_amd.h"

namespace {
thread_local std::string g_last_error;
}

extern "C" acl_status_t acl__set_error(const char* msg) {
  g_last_error = msg ? msg : "";
  return ACL_ERR_INVALID_ARG;
}

static acl_status_t hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return ACL_OK;
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return ACL_ERR_HIP;
}

extern "C" const char* acl_last_error(void) { return g_last_error.c_str(); }

extern "C" void acl_default_cntrl_gains(acl_cntrl_gains_t* g) {
  // aclswarm/launch/coordination.launch:32-39
  g->K1_xy = 0.1; g->K2_xy = 0.1; g->K1_z = 0.5; g->K2_z = 0.3;
  g->e_xy_thr = 0.3; g->e_z_thr = 0.1; g->kp = 1.5; g->kd = 0.5;
}

extern "C" void acl_default_safety_params(acl_safety_params_t* s) {
  // aclswarm/src/safety.cpp:49-52
  s->max_vel_xy = 0.5; s->max_vel_z = 0.3; s->d_avoid_thresh = 1.5; s->r_keep_out = 1.2;
}

extern "C" void acl_default_admm_params(acl_admm_params_t* a) {
  // aclswarm/lib/admm/include/admm/solver.h:18-31
  a->verbose = 0; a->thrSparseZero = 1e-8; a->thrPlanar = 1e-2; a->epsEig = 1e-5;
  a->mu = 1.0; a->thresh = 1e-4; a->threshTr = 0.10; a->maxItr = 10;
  a->basis = ACL_ADMM_BASIS_LINPACK;
}

extern "C" void acl_formations_init(acl_formations_t* F, int32_t n, int32_t n_formations) {
  if (!F) return;
  std::memset(F, 0, sizeof(*F));
  F->n = n;
  F->n_formations = n_formations;
  F->gain_planes = 9;
}

// ---- packing -------------------------------------------------------------

extern "C" int64_t acl_count_edges(int32_t n, const uint8_t* adj) {
  if (n < 1 || !adj) return -1;
  int64_t e = 0;
  for (int64_t k = 0; k < (int64_t)n * n; ++k) e += adj[k] != 0;
  return e;
}

extern "C" acl_status_t acl_pack_adjacency(int32_t n, const uint8_t* adj, uint64_t* out) {
  if (n < 1 || !adj || !out) return acl__set_error("acl_pack_adjacency: bad argument");
  const int W = (n + 63) / 64;
  std::memset(out, 0, sizeof(uint64_t) * (size_t)n * W);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      if (adj[(size_t)j * n + i])  // column-major AdjMat(i,j)
        out[(size_t)i * W + j / 64] |= 1ull << (j % 64);
  return ACL_OK;
}

namespace {
// (r, c) of the 5 stored entries of the record layout; the other four entries
// of every block are the structural zeros of admm::Solver::solve
constexpr int kPlanes5[5][2] = {{0, 0}, {0, 1}, {1, 0}, {1, 1}, {2, 2}};

bool is_pos_zero(double x) {
  uint64_t u;
  std::memcpy(&u, &x, 8);
  return u == 0;
}
}  // namespace

extern "C" int32_t acl_gain_planes(int32_t n, const uint8_t* adj, const double* gains) {
  if (n < 1 || !adj || !gains) return 9;
  const size_t ld = (size_t)3 * n;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (!adj[(size_t)j * n + i]) continue;
      const double* blk = gains + (3 * (size_t)j) * ld + 3 * (size_t)i;  // column-major
      // (0,2), (1,2), (2,0), (2,1)
      if (!is_pos_zero(blk[2 * ld + 0]) || !is_pos_zero(blk[2 * ld + 1]) ||
          !is_pos_zero(blk[0 * ld + 2]) || !is_pos_zero(blk[1 * ld + 2]))
        return 9;
    }
  return 5;
}

extern "C" acl_status_t acl_pack_gains_planes(int32_t n, const uint8_t* adj, const double* gains,
                                              int32_t planes, double* out) {
  if (n < 1 || !adj || !gains || !out || (planes != 9 && planes != 5))
    return acl__set_error("acl_pack_gains_planes: bad argument");
  if (planes == 5 && acl_gain_planes(n, adj, gains) != 5)
    return acl__set_error("acl_pack_gains_planes: a gain block has a nonzero (or -0.0) "
                          "entry outside the 5-entry structure");
  const int64_t E = acl_count_edges(n, adj);
  const size_t ld = (size_t)3 * n;  // column-major leading dimension
  int64_t e = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (!adj[(size_t)j * n + i]) continue;
      const double* blk = gains + (3 * (size_t)j) * ld + 3 * (size_t)i;
      if (planes == 9) {
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c) out[(size_t)(3 * r + c) * E + e] = blk[(size_t)c * ld + r];
      } else {  // one record of 5 doubles per edge
        for (int k = 0; k < 5; ++k)
          out[(size_t)5 * e + k] = blk[(size_t)kPlanes5[k][1] * ld + kPlanes5[k][0]];
      }
      ++e;
    }
  return ACL_OK;
}

extern "C" acl_status_t acl_pack_gains(int32_t n, const uint8_t* adj, const double* gains,
                                       double* out) {
  if (n < 1 || !adj || !gains || !out) return acl__set_error("acl_pack_gains: bad argument");
  return acl_pack_gains_planes(n, adj, gains, 9, out);
}

// ---- Auctioneer::logAssignment records (auctioneer.cpp:577-597) ----------

namespace {
// aligned = R p + t with the z row identity, in alignFormation's operation
// order (the same expression the price kernels evaluate)
void aligned_points(int n, const double* p, const double* Rt, double* out) {
  for (int j = 0; j < n; ++j) {
    const double px = p[3 * j], py = p[3 * j + 1], pz = p[3 * j + 2];
    out[3 * j] = ((Rt[0] * px + Rt[1] * py) + 0.0 * pz) + Rt[4];
    out[3 * j + 1] = ((Rt[2] * px + Rt[3] * py) + 0.0 * pz) + Rt[5];
    out[3 * j + 2] = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0;
  }
}
}  // namespace

extern "C" acl_status_t acl_write_assignment_log(const char* path, int32_t n, const double* q,
                                                 const uint8_t* adj, const uint16_t* lastP,
                                                 const double* p, const double* Rt,
                                                 const uint16_t* P) {
  if (!path || n < 1 || n > 255 || !q || !adj || !lastP || !p || !Rt || !P)
    return acl__set_error("acl_write_assignment_log: bad argument (n must be 1..255)");
  std::vector<double> al(3 * (size_t)n), col(3 * (size_t)n);
  aligned_points(n, p, Rt, al.data());
  FILE* f = std::fopen(path, "wb");
  if (!f) return acl__set_error("acl_write_assignment_log: cannot open file");
  auto colmajor = [&](const double* rm) {  // PtsMat is n x 3 column-major
    for (int c = 0; c < 3; ++c)
      for (int i = 0; i < n; ++i) col[(size_t)c * n + i] = rm[3 * i + c];
    std::fwrite(col.data(), sizeof(double), col.size(), f);
  };
  auto perm = [&](const uint16_t* x) {
    std::vector<uint8_t> b(n);
    for (int i = 0; i < n; ++i) b[i] = (uint8_t)x[i];
    std::fwrite(b.data(), 1, b.size(), f);
  };
  const uint8_t n8 = (uint8_t)n;
  std::fwrite(&n8, 1, 1, f);
  colmajor(q);
  std::fwrite(adj, 1, (size_t)n * n, f);
  perm(lastP);
  colmajor(p);
  colmajor(al.data());
  perm(P);
  const bool ok = std::ferror(f) == 0;
  std::fclose(f);
  return ok ? ACL_OK : acl__set_error("acl_write_assignment_log: write failed");
}

extern "C" acl_status_t acl_read_assignment_log(const char* path, int32_t* n_out, double* q,
                                                uint8_t* adj, uint16_t* lastP, double* p,
                                                double* aligned, uint16_t* P) {
  if (!path || !n_out) return acl__set_error("acl_read_assignment_log: bad argument");
  FILE* f = std::fopen(path, "rb");
  if (!f) return acl__set_error("acl_read_assignment_log: cannot open file");
  uint8_t n8 = 0;
  if (std::fread(&n8, 1, 1, f) != 1) {
    std::fclose(f);
    return acl__set_error("acl_read_assignment_log: truncated file");
  }
  const int n = n8;
  *n_out = n;
  if (!q || !adj || !lastP || !p || !aligned || !P) {
    std::fclose(f);
    return ACL_OK;  // size query
  }
  std::vector<double> col(3 * (size_t)n);
  bool ok = true;
  auto rowmajor = [&](double* rm) {
    ok = ok && std::fread(col.data(), sizeof(double), col.size(), f) == col.size();
    for (int c = 0; c < 3; ++c)
      for (int i = 0; i < n; ++i) rm[3 * i + c] = col[(size_t)c * n + i];
  };
  auto perm = [&](uint16_t* x) {
    std::vector<uint8_t> b(n);
    ok = ok && std::fread(b.data(), 1, b.size(), f) == b.size();
    for (int i = 0; i < n; ++i) x[i] = b[i];
  };
  rowmajor(q);
  ok = ok && std::fread(adj, 1, (size_t)n * n, f) == (size_t)n * n;
  perm(lastP);
  rowmajor(p);
  rowmajor(aligned);
  perm(P);
  std::fclose(f);
  return ok ? ACL_OK : acl__set_error("acl_read_assignment_log: truncated file");
}

// ---- device memory -------------------------------------------------------

extern "C" int32_t acl_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

extern "C" acl_status_t acl_set_device(int32_t d) { return hip_check(hipSetDevice(d), "hipSetDevice"); }

extern "C" acl_status_t acl_malloc(void** ptr, size_t bytes) {
  return hip_check(hipMalloc(ptr, bytes), "hipMalloc");
}

extern "C" acl_status_t acl_free(void* ptr) { return hip_check(hipFree(ptr), "hipFree"); }

extern "C" acl_status_t acl_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
  return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream),
                   "hipMemcpyAsync(H2D)");
}

extern "C" acl_status_t acl_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
  return hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream),
                   "hipMemcpyAsync(D2H)");
}

extern "C" acl_status_t acl_memset(void* dst, int value, size_t bytes, void* stream) {
  return hip_check(hipMemsetAsync(dst, value, bytes, (hipStream_t)stream), "hipMemsetAsync");
}

extern "C" acl_status_t acl_stream_synchronize(void* stream) {
  return hip_check(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
}

extern "C" int32_t acl_abi_version(void) { return ACL_ABI_VERSION; }
