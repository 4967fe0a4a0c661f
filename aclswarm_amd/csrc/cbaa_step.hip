// cbaa_step.hip -- one vehicle's CBAA bid iteration, batched over V vehicles:
// the message-level protocol of the reference's per-vehicle Auctioneer, for
// vehicles that exchange their bids with neighbours round by round
// (auctioneer.cpp:124-160 enqueueBid/tick, :182-306 processBid) instead of
// running the whole consensus in one acl_solve_batch call. The facade's
// exchange mode (include/aclswarm_amd.hpp, Auctioneer::setBidExchange) calls
// it once per completed bid iteration; a simulator can batch the iterations
// of many vehicles into one launch.
//
// Per vehicle k (one wavefront; lane l owns tasks j = l + 64 s, s < 8):
//   start[k] = 1  reset (auctioneer.cpp:448-465: price 0, who -1), then the
//                 START bid: selectTaskAssignment (:517-542);
//   start[k] = 0  updateTaskAssignment (:469-513): for every task j the
//                 highest price among the candidates -- the vehicle's own
//                 table and its neighbours' bids of this iteration, in
//                 std::map order (ascending vehid), the first of equal prices
//                 kept (strict >) -- replaces its entry; outbid = some task it
//                 held now has another holder; then selectTaskAssignment if
//                 it was outbid.
// selectTaskAssignment's scan (max = 0, `price > max && price > bid.price[j]`
// in ascending j) takes the lowest task with the largest eligible price: one
// wave max over the eligible prices, then the lowest lane holding it.
// getPrice(q_k, paligned_j) (:546-549) is evaluated here from the vehicle's
// alignment (acl_solve_batch's align_Rt row: paligned = (R p + t, p.z),
// :400-414) in the reference's f64 operation order (this file is compiled
// with -ffp-contract=off), so the floats equal the batched auction's prices
// bit for bit.
#include "common.h"

#include "../../include/aclswarm_amd.h"

extern "C" acl_status_t acl__set_error(const char* msg);

namespace acl_amd {

struct StepParams {
  int n, V, K, F;
  const double* p;
  const int32_t* fidx;
  const int32_t* vehid;
  const double* q;
  const double* Rt;
  const uint8_t* start;
  float* price;
  int32_t* who;
  const int32_t* cand_off;
  const int32_t* cand_vehid;
  const float* cand_price;
  const int32_t* cand_who;
  int32_t* task;
  int32_t* flags;
};

constexpr int kStepWaves = 4;  // vehicles per workgroup (one per wave)

// getPrice of task j for a vehicle at (qx, qy, qz) with alignment o[6]:
// aligned = ((R p^T).colwise() + t)^T, R = [R2 0; 0 0 1] (auctioneer.cpp:
// 400-414), then (float)(1 / (||q - aligned|| + 1e-8)) with IEEE sqrt and
// division -- the oracle's orc_prices_rows expression term for term
__device__ __forceinline__ float step_price(const double* o, double qx, double qy, double qz,
                                            const double* pj) {
  const double px = pj[0], py = pj[1], pz = pj[2];
  const double ax = ((o[0] * px + o[1] * py) + 0.0 * pz) + o[4];
  const double ay = ((o[2] * px + o[3] * py) + 0.0 * pz) + o[5];
  const double az = ((0.0 * px + 0.0 * py) + 1.0 * pz) + 0.0;
  const double dx = qx - ax, dy = qy - ay, dz = qz - az;
  const double nrm = __builtin_sqrt((dx * dx + dy * dy) + dz * dz);
  return (float)(1.0 / (nrm + 1e-8));
}

template <int S>
__global__ void __launch_bounds__(64 * kStepWaves) cbaa_step_kernel(const StepParams P) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * kStepWaves + (int)(threadIdx.x >> 6);
  if (k >= P.V) return;  // wave-uniform
  const int n = P.n;
  const int v = P.vehid[k];
  const int f = P.fidx[k];
  const int c0 = P.cand_off[k], c1 = P.cand_off[k + 1];
  const bool st = P.start[k] != 0;
  // argument checks (wave-uniform): the vehicle, its formation, and the
  // candidates strictly ascending by vehid inside [0, n)
  bool bad = v < 0 || v >= n || f < 0 || f >= P.F ||
             (!st && (c0 < 0 || c1 <= c0 || c1 > P.K || !P.cand_vehid || !P.cand_price ||
                      !P.cand_who));
  if (!bad && !st) {
    for (int c = c0 + lane; c < c1; c += 64) {
      const int u = P.cand_vehid[c];
      if (u < 0 || u >= n || (c > c0 && P.cand_vehid[c - 1] >= u)) bad = true;
    }
    bad = __any(bad);
  }
  if (bad) {
    if (lane == 0) {
      P.task[k] = -1;
      P.flags[k] = ACL_CBAA_BAD_INPUT;
    }
    return;
  }
  float* pr = P.price + (size_t)k * n;
  int32_t* wh = P.who + (size_t)k * n;
  float own_p[S];
  int own_w[S];
  bool outbid = false;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int j = lane + 64 * s;
    own_p[s] = 0.0f;
    own_w[s] = -1;
    if (j < n && !st) {
      const int wmine = wh[j];
      // the first candidate, then strict > in ascending vehid (auctioneer.cpp:480-491)
      const float* cp = P.cand_price + (size_t)c0 * n + j;
      const int32_t* cw = P.cand_who + (size_t)c0 * n + j;
      float mp = cp[0];
      int mw = cw[0];
      for (int c = 1; c < c1 - c0; ++c) {
        const float x = cp[(size_t)c * n];
        if (x > mp) {
          mp = x;
          mw = cw[(size_t)c * n];
        }
      }
      // (:498) was I outbid on a task I held?
      if (wmine == v && mw != v) outbid = true;
      own_p[s] = mp;
      own_w[s] = mw;
    }
  }
  outbid = __any(outbid);
  int task = -1;
  unsigned best = 0u;  // float bits of the largest eligible price (> 0: ordered as u32)
  if (st || outbid) {
    // selectTaskAssignment (:517-542): the largest eligible price, lowest task
    const double* o = P.Rt + (size_t)k * 6;
    const double* q = P.q + (size_t)k * 3;
    const double qx = q[0], qy = q[1], qz = q[2];
    const double* pf = P.p + (size_t)f * n * 3;
    float c[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = lane + 64 * s;
      c[s] = 0.0f;
      if (j < n) {
        const float x = step_price(o, qx, qy, qz, pf + 3 * j);
        if (x > 0.0f && x > own_p[s]) {
          c[s] = x;
          const unsigned b = __float_as_uint(x);
          best = b > best ? b : best;
        }
      }
    }
    best = wave_max_u32(best);
    if (best != 0u) {
      // the lowest task holding it: each lane's lowest slot, then a wave minimum
      int jmin = 0x7FFFFFFF;
#pragma unroll
      for (int s = S - 1; s >= 0; --s) {
        const int j = lane + 64 * s;
        if (j < n && __float_as_uint(c[s]) == best) jmin = j;
      }
      for (int off = 32; off >= 1; off >>= 1) {
        const int o2 = __shfl_xor(jmin, off);
        jmin = o2 < jmin ? o2 : jmin;
      }
      task = jmin;
    }
  }
  // (:538-541) the bid on the selected task; the merged table elsewhere
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int j = lane + 64 * s;
    if (j < n) {
      const bool mine = j == task;
      pr[j] = mine ? __uint_as_float(best) : own_p[s];
      wh[j] = mine ? v : own_w[s];
    }
  }
  if (lane == 0) {
    P.task[k] = task;
    P.flags[k] = (outbid ? ACL_CBAA_OUTBID : 0) | (task >= 0 ? ACL_CBAA_SELECTED : 0);
  }
}

}  // namespace acl_amd

extern "C" acl_status_t acl_cbaa_step_batch(const acl_formations_t* F, const acl_cbaa_step_args_t* a,
                                            void* stream) {
  using namespace acl_amd;
  if (!F || !a) return acl__set_error("acl_cbaa_step_batch: null argument");
  const int n = F->n;
  if (n < 1 || n > 512) return acl__set_error("acl_cbaa_step_batch: n out of range [1, 512]");
  if (a->V < 0 || a->K < 0) return acl__set_error("acl_cbaa_step_batch: V < 0 or K < 0");
  if (a->V == 0) return ACL_OK;
  if (!F->p || F->n_formations < 1 || !a->fidx || !a->vehid || !a->q || !a->Rt || !a->start ||
      !a->price || !a->who || !a->cand_off || !a->task || !a->flags)
    return acl__set_error("acl_cbaa_step_batch: required pointer is NULL");
  StepParams P;
  P.n = n; P.V = a->V; P.K = a->K; P.F = F->n_formations; P.p = F->p;
  P.fidx = a->fidx; P.vehid = a->vehid; P.q = a->q; P.Rt = a->Rt; P.start = a->start;
  P.price = a->price; P.who = a->who; P.cand_off = a->cand_off; P.cand_vehid = a->cand_vehid;
  P.cand_price = a->cand_price; P.cand_who = a->cand_who; P.task = a->task; P.flags = a->flags;
  const int nb = (a->V + kStepWaves - 1) / kStepWaves;
  hipStream_t s = (hipStream_t)stream;
  if (n <= 64)
    hipLaunchKernelGGL(cbaa_step_kernel<1>, dim3(nb), dim3(64 * kStepWaves), 0, s, P);
  else if (n <= 128)
    hipLaunchKernelGGL(cbaa_step_kernel<2>, dim3(nb), dim3(64 * kStepWaves), 0, s, P);
  else if (n <= 256)
    hipLaunchKernelGGL(cbaa_step_kernel<4>, dim3(nb), dim3(64 * kStepWaves), 0, s, P);
  else
    hipLaunchKernelGGL(cbaa_step_kernel<8>, dim3(nb), dim3(64 * kStepWaves), 0, s, P);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  return ACL_OK;
}
