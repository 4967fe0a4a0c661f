// hungarian.hip -- the centralized assignment comparator, batched:
// aclswarm/src/aclswarm/assignment.py:94-137 (find_optimal_assignment) for B
// swarms, one wavefront per swarm.
//
//   align (assignment.py:15-92): 2-D Arun of the formation onto the swarm in
//     the last assignment's order, as the closed-form proper rotation
//     (c, s) = (a, b) / |(a, b)|, a = H00 + H11, b = H10 - H01, H = Q P^T;
//   S[v][j] = ||q_v - paligned_j|| (scipy cdist: ((dx^2 + dy^2) + dz^2)^0.5);
//   P = linear_sum_assignment(S)[1]: SciPy's Crouse shortest augmenting
//     path, with its column order (reverse-initialised list, last entry
//     moved into the removed slot) and tie rule (equal reduced cost wins only
//     for an unassigned column) -- restated and pinned against scipy in
//     oracle/hungarian_oracle.c, which this kernel matches bit for bit.
//
// Layout on the wave. Lane l owns columns (formation points) j = l + 64 s and
// rows (vehicles) v = l + 64 s for slots s < S (n <= 64 S), all per-column
// state in registers: aligned point, dual v, shortest-path cost, path,
// row4col, and the column's position in SciPy's `remaining` list (-1 once
// scanned). One Dijkstra step = every lane prices its live columns against
// the wave-uniform row i (q_i broadcast from LDS), one fp64 DPP min, one u32
// DPP max over a packed (tie class, position, column) key, and a few
// readlanes. S is computed on the fly (no n x n matrix): ~2 fp64 distance
// evaluations per lane per step, so the kernel is VALU-bound; HBM traffic is
// the inputs and outputs only (q, P_last, P_cmp, p: ~5 KB per swarm at
// n = 100).
#include "common.h"

#include "../../include/aclswarm_amd.h"

extern "C" acl_status_t acl__set_error(const char* msg);

namespace acl_amd {

constexpr int kHungWaves = 4;  // swarms per workgroup (one per wave)

struct HungParams {
  int n, B, F;
  const double* p;
  const int32_t* fidx;
  const double* q;
  const uint16_t* P_last;
  const uint16_t* P_cmp;
  uint16_t* P_opt;
  double* cost;
  double* align_Rt;
  int32_t* status;
};

// per-wave LDS: q [n][3], p [n][3], spc gather [n] f64, Pt [n] u16
__host__ __device__ constexpr size_t hung_lds_per_wave(int n) {
  return (size_t)n * (3 + 3 + 1) * sizeof(double) + (((size_t)n * 2 + 15) & ~(size_t)15);
}

__device__ __forceinline__ double rl_f64(double x, int lane) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// slot register of wave-uniform index j (owner lane j & 63, slot j >> 6)
template <int S, typename T>
__device__ __forceinline__ T slot_sel(const T (&a)[S], int s) {
  T v = a[0];
#pragma unroll
  for (int k = 1; k < S; ++k) v = (s == k) ? a[k] : v;
  return v;
}
template <int S>
__device__ __forceinline__ int get_i(const int (&a)[S], int j) {
  return __builtin_amdgcn_readlane(slot_sel<S, int>(a, j >> 6), j & 63);
}
template <int S>
__device__ __forceinline__ double get_d(const double (&a)[S], int j) {
  return rl_f64(slot_sel<S, double>(a, j >> 6), j & 63);
}

// DPP move of a double with +inf (min's identity) where the pattern reads
// outside the row / where the row mask is off.
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_f64_inf(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u, CTRL, RMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0x7FF00000, (int)(u >> 32), CTRL, RMASK, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Minimum over the wave (no NaN inputs); the value, not its sign of zero,
// is what the caller uses (it compares with ==).
__device__ __forceinline__ double wave_min_f64(double x) {
  x = fmin(x, dpp_f64_inf<0xB1, 0xF>(x));
  x = fmin(x, dpp_f64_inf<0x4E, 0xF>(x));
  x = fmin(x, dpp_f64_inf<0x124, 0xF>(x));
  x = fmin(x, dpp_f64_inf<0x128, 0xF>(x));
  x = fmin(x, dpp_f64_inf<0x142, 0xA>(x));
  x = fmin(x, dpp_f64_inf<0x143, 0xC>(x));
  return rl_f64(x, 63);
}

__device__ __forceinline__ double dist3(double qx, double qy, double qz, double ax, double ay,
                                        double az) {
  const double dx = qx - ax, dy = qy - ay, dz = qz - az;
  return __builtin_sqrt((dx * dx + dy * dy) + dz * dz);  // cdist's order, no contraction
}

template <int S>
__global__ void __launch_bounds__(64 * kHungWaves) hungarian_kernel(const HungParams P) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const int n = P.n;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * kHungWaves + wave;
  if (b >= P.B) return;  // whole wave leaves; no workgroup barriers below
  unsigned char* base = lds_raw + (size_t)wave * hung_lds_per_wave(n);
  double* sq = reinterpret_cast<double*>(base);
  double* sp = sq + 3 * n;
  double* sgat = sp + 3 * n;
  uint16_t* sPt = reinterpret_cast<uint16_t*>(sgat + n);

  const int f = P.fidx[b];
  uint16_t* Popt = P.P_opt + (size_t)b * n;
  bool bad = f < 0 || f >= P.F;
  if (!bad) {
    const double* qb = P.q + (size_t)b * n * 3;
    const double* pf = P.p + (size_t)f * n * 3;
    for (int k = lane; k < 3 * n; k += 64) { sq[k] = qb[k]; sp[k] = pf[k]; }
    const uint16_t* Pl = P.P_last ? P.P_last + (size_t)b * n : nullptr;
    for (int v = lane; v < n; v += 64) sPt[v] = 0xFFFF;
    __builtin_amdgcn_wave_barrier();
    for (int v = lane; v < n; v += 64) {
      const int k = Pl ? Pl[v] : v;
      if (k < n) sPt[k] = (uint16_t)v;  // duplicates overwrite: caught below
    }
    __builtin_amdgcn_wave_barrier();
    bool mine_bad = false;
    for (int v = lane; v < n; v += 64) {
      const int k = Pl ? Pl[v] : v;
      mine_bad |= k >= n || sPt[k] != v;
    }
    bad = __builtin_amdgcn_ballot_w64(mine_bad) != 0;
  }
  if (bad) {
    for (int v = lane; v < n; v += 64) Popt[v] = 0xFFFF;
    if (lane == 0) {
      P.cost[2 * b] = __builtin_nan("");
      P.cost[2 * b + 1] = __builtin_nan("");
      P.status[b] = ACL_HUNG_BAD_INPUT;
    }
    return;
  }

  // ---- Arun (assignment.py:15-53) on qq[k] = q[Pt[k]]: lanes 0-3 run one
  // sequential sum each, in the oracle's order
  double sum = 0.0;
  if (lane < 4) {
    const int c = lane & 1;
    for (int k = 0; k < n; ++k) sum += lane < 2 ? sq[3 * sPt[k] + c] : sp[3 * k + c];
  }
  const double dn = (double)n;
  const double mqx = rl_f64(sum, 0) / dn, mqy = rl_f64(sum, 1) / dn;
  const double mpx = rl_f64(sum, 2) / dn, mpy = rl_f64(sum, 3) / dn;
  double h = 0.0;
  if (lane < 4) {
    const int cq = lane >> 1, cp = lane & 1;  // h00, h01, h10, h11
    const double mq = cq ? mqy : mqx, mp = cp ? mpy : mpx;
    for (int k = 0; k < n; ++k) h += (sq[3 * sPt[k] + cq] - mq) * (sp[3 * k + cp] - mp);
  }
  const double h00 = rl_f64(h, 0), h01 = rl_f64(h, 1), h10 = rl_f64(h, 2), h11 = rl_f64(h, 3);
  const double ra = h00 + h11, rb = h10 - h01;
  const double rr = __builtin_sqrt(ra * ra + rb * rb);
  double c = 1.0, s = 0.0;
  if (rr > 0.0) { c = ra / rr; s = rb / rr; }
  const double tx = mqx - (c * mpx - s * mpy);
  const double ty = mqy - (s * mpx + c * mpy);
  if (P.align_Rt && lane == 0) {
    double* o = P.align_Rt + 4 * (size_t)b;
    o[0] = c; o[1] = s; o[2] = tx; o[3] = ty;
  }

  // ---- per-lane column and row state
  double ax[S], ay[S], az[S], vv[S], spc[S], uu[S];
  int pos[S], path[S], r4c[S], c4r[S];
  unsigned SR = 0;  // bit s: row lane + 64 s is in SR
  bool nonfin = false;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const int j = lane + 64 * k;
    ax[k] = ay[k] = az[k] = 0.0;
    if (j < n) {
      const double px = sp[3 * j], py = sp[3 * j + 1];
      ax[k] = (c * px - s * py) + tx;
      ay[k] = (s * px + c * py) + ty;
      az[k] = sp[3 * j + 2];
      nonfin |= !__builtin_isfinite(ax[k]) || !__builtin_isfinite(ay[k]) ||
                !__builtin_isfinite(az[k]) || !__builtin_isfinite(sq[3 * j]) ||
                !__builtin_isfinite(sq[3 * j + 1]) || !__builtin_isfinite(sq[3 * j + 2]);
    }
    vv[k] = 0.0; uu[k] = 0.0; path[k] = -1; r4c[k] = -1; c4r[k] = -1;
  }
  // scipy rejects NaN / -inf costs: with every coordinate finite no cost is
  // NaN (overflow gives +inf, which is legal), otherwise scan all of S
  int status = 0;
  if (__builtin_amdgcn_ballot_w64(nonfin) != 0) {
    bool nan = false;
    for (int i = 0; i < n; ++i) {
      const double qx = sq[3 * i], qy = sq[3 * i + 1], qz = sq[3 * i + 2];
#pragma unroll
      for (int k = 0; k < S; ++k)
        if (lane + 64 * k < n) nan |= __builtin_isnan(dist3(qx, qy, qz, ax[k], ay[k], az[k]));
    }
    if (__builtin_amdgcn_ballot_w64(nan) != 0) status = ACL_HUNG_NONFINITE;
  }

  // ---- Crouse LSAP (see oracle/hungarian_oracle.c: orc_lsap)
  for (int cur = 0; cur < n && !status; ++cur) {
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int j = lane + 64 * k;
      pos[k] = j < n ? n - 1 - j : -1;  // remaining[it] = n - it - 1
      spc[k] = __builtin_inf();
    }
    SR = 0;
    int nrem = n;
    double minVal = 0.0;
    int i = cur, sink = -1;
    while (sink < 0) {
      if (lane == (i & 63)) SR |= 1u << (i >> 6);
      const double ui = get_d<S>(uu, i);
      const double qx = sq[3 * i], qy = sq[3 * i + 1], qz = sq[3 * i + 2];
      double lmin = __builtin_inf();
#pragma unroll
      for (int k = 0; k < S; ++k) {
        if (pos[k] >= 0) {
          const double r = ((minVal + dist3(qx, qy, qz, ax[k], ay[k], az[k])) - ui) - vv[k];
          if (r < spc[k]) { path[k] = i; spc[k] = r; }
          lmin = fmin(lmin, spc[k]);
        }
      }
      const double m = wave_min_f64(lmin);
      if (!(m < __builtin_inf())) { status = ACL_HUNG_NONFINITE; break; }  // infeasible
      // among columns at the minimum: the last unassigned one in list order
      // if any, else the first (the sequential scan's outcome)
      unsigned key = 0;
#pragma unroll
      for (int k = 0; k < S; ++k) {
        if (pos[k] >= 0 && spc[k] == m) {
          const unsigned cls = r4c[k] < 0 ? 512u + (unsigned)pos[k] : 511u - (unsigned)pos[k];
          const unsigned kk = (cls << 9) | (unsigned)(lane + 64 * k);
          key = kk > key ? kk : key;
        }
      }
      key = wave_max_u32(key);
      const int j = (int)(key & 511u);
      const unsigned cls = key >> 9;
      const int index = cls >= 512u ? (int)(cls - 512u) : (int)(511u - cls);
      minVal = get_d<S>(spc, j);  // == m
      const int rj = get_i<S>(r4c, j);
      if (rj < 0) sink = j; else i = rj;
      // remaining[index] = remaining[--nrem]
      --nrem;
#pragma unroll
      for (int k = 0; k < S; ++k) {
        if (lane + 64 * k == j) pos[k] = -1;
        else if (pos[k] == nrem) pos[k] = index;
      }
    }
    if (status) break;
    // ---- dual update: u[cur] += minVal; SR rows u[r] += minVal - spc[col4row[r]];
    // scanned columns v[j] -= minVal - spc[j]
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int j = lane + 64 * k;
      if (j < n) sgat[j] = spc[k];
      if (pos[k] < 0 && j < n) vv[k] -= minVal - spc[k];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const int r = lane + 64 * k;
      if (r == cur) uu[k] += minVal;
      else if ((SR >> k) & 1u) uu[k] += minVal - sgat[c4r[k]];
    }
    __builtin_amdgcn_wave_barrier();
    // ---- augment along path from the sink
    int j = sink;
    for (;;) {
      const int r = get_i<S>(path, j);
      if (lane == (j & 63)) {
#pragma unroll
        for (int k = 0; k < S; ++k) if (k == (j >> 6)) r4c[k] = r;
      }
      const int t = get_i<S>(c4r, r);
      if (lane == (r & 63)) {
#pragma unroll
        for (int k = 0; k < S; ++k) if (k == (r >> 6)) c4r[k] = j;
      }
      j = t;
      if (r == cur) break;
    }
  }

  // ---- outputs: P_opt, cost of P_opt and of P_cmp (sequential sums over v)
  if (status) {
    for (int v = lane; v < n; v += 64) Popt[v] = 0xFFFF;
    if (lane == 0) {
      P.cost[2 * b] = __builtin_nan("");
      P.cost[2 * b + 1] = __builtin_nan("");
      P.status[b] = status;
    }
    return;
  }
  const uint16_t* Pc = P.P_cmp ? P.P_cmp + (size_t)b * n : nullptr;
  // reuse LDS: sgat = S[v][P_opt[v]], spc-free region of sp is still p
  double* scmp = sq;  // q no longer needed after these reads: stage per row
  double dopt[S], dcmp[S];
  bool cmp_bad = false;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const int v = lane + 64 * k;
    dopt[k] = dcmp[k] = 0.0;
    if (v < n) {
      const double qx = sq[3 * v], qy = sq[3 * v + 1], qz = sq[3 * v + 2];
      const int jo = c4r[k];
      const double pxo = sp[3 * jo], pyo = sp[3 * jo + 1];
      dopt[k] = dist3(qx, qy, qz, (c * pxo - s * pyo) + tx, (s * pxo + c * pyo) + ty, sp[3 * jo + 2]);
      Popt[v] = (uint16_t)jo;
      if (Pc) {
        const int jc = Pc[v];
        if (jc >= n) { cmp_bad = true; }
        else {
          const double pxc = sp[3 * jc], pyc = sp[3 * jc + 1];
          dcmp[k] = dist3(qx, qy, qz, (c * pxc - s * pyc) + tx, (s * pxc + c * pyc) + ty,
                          sp[3 * jc + 2]);
        }
      }
    }
  }
  // P_cmp permutation check through Pt scratch
  if (Pc) {
    for (int v = lane; v < n; v += 64) sPt[v] = 0xFFFF;
    __builtin_amdgcn_wave_barrier();
    for (int v = lane; v < n; v += 64) if (Pc[v] < n) sPt[Pc[v]] = (uint16_t)v;
    __builtin_amdgcn_wave_barrier();
    for (int v = lane; v < n; v += 64) cmp_bad |= Pc[v] >= n || sPt[Pc[v]] != v;
    cmp_bad = __builtin_amdgcn_ballot_w64(cmp_bad) != 0;
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const int v = lane + 64 * k;
    if (v < n) { sgat[v] = dopt[k]; scmp[v] = dcmp[k]; }
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    double c0 = 0.0, c1 = 0.0;
    for (int v = 0; v < n; ++v) { c0 += sgat[v]; c1 += scmp[v]; }
    P.cost[2 * b] = c0;
    P.cost[2 * b + 1] = (Pc && !cmp_bad) ? c1 : __builtin_nan("");
    P.status[b] = (Pc && cmp_bad) ? ACL_HUNG_CMP_INVALID : 0;
  }
}

}  // namespace acl_amd

extern "C" acl_status_t acl_hungarian_batch(const acl_formations_t* F,
                                            const acl_hungarian_args_t* a, void* stream) {
  using namespace acl_amd;
  if (!F || !a) return acl__set_error("acl_hungarian_batch: null argument");
  const int n = F->n;
  if (n < 1 || n > 512) return acl__set_error("acl_hungarian_batch: n out of range [1, 512]");
  if (a->B < 0) return acl__set_error("acl_hungarian_batch: B < 0");
  if (a->B == 0) return ACL_OK;
  if (!F->p || F->n_formations < 1 || !a->fidx || !a->q || !a->P_opt || !a->cost || !a->status)
    return acl__set_error("acl_hungarian_batch: required pointer is NULL");
  HungParams P;
  P.n = n; P.B = a->B; P.F = F->n_formations;
  P.p = F->p; P.fidx = a->fidx; P.q = a->q; P.P_last = a->P_last; P.P_cmp = a->P_cmp;
  P.P_opt = a->P_opt; P.cost = a->cost; P.align_Rt = a->align_Rt; P.status = a->status;
  const size_t lds = hung_lds_per_wave(n) * kHungWaves;
  const int nb = (a->B + kHungWaves - 1) / kHungWaves;
  hipStream_t s = (hipStream_t)stream;
  if (n <= 128)
    hipLaunchKernelGGL(hungarian_kernel<2>, dim3(nb), dim3(64 * kHungWaves), lds, s, P);
  else if (n <= 256)
    hipLaunchKernelGGL(hungarian_kernel<4>, dim3(nb), dim3(64 * kHungWaves), lds, s, P);
  else
    hipLaunchKernelGGL(hungarian_kernel<8>, dim3(nb), dim3(64 * kHungWaves), lds, s, P);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  return ACL_OK;
}
