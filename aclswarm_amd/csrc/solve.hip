// solve.hip -- host entry points of the batched solve (C ABI).
//
// acl_solve_batch enqueues, stream-ordered, over all B swarms:
//   1. the alignment launch (n > 64): align_kernel<2> (auction.hip, one wave
//      per swarm) for 64 < n <= 128, align_wide_kernel (solve_wide.hip, one
//      1 024-thread workgroup per swarm) for n > 128; n <= 64 aligns inside
//      the auction workgroup;
//   2. the auction launch: auction_kernel (auction.hip, n <= 128, every CBAA
//      table in LDS) or solve_wide_kernel (solve_wide.hip, n <= 512, the
//      `who` table in the workspace). With 5-entry gain records and
//      do_control it is FUSED: a swarm whose vehicles all adopted one
//      assignment runs DistCntrl::compute (distcntrl.cpp:46-102), saturation
//      and the first collision test (safety.cpp:172-197, 412-430) in its own
//      workgroup after adoption (pair_fused.h for n <= 128, wide_control for
//      n > 128);
//   3. the gain launch (control.hip): the directed walk for the swarms the
//      fused phase did not take (per-vehicle assignments, 9-plane records,
//      or every swarm when not fused) -- an early exit for the others;
//   4. the collision-avoidance launch (control.hip: ca_pair_kernel for
//      n <= 128, ca_kernel above) over the vehicles step 2/3 listed
//      (Safety::collisionAvoidance, safety.cpp:412-541).
// acl_control_batch runs 3-4 for a given assignment (the pair kernel for
// uniform swarms); acl_tile_gains re-lays 5-entry records for it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "../../include/aclswarm_amd.h"
#include "common.h"
#include "control_params.h"

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" acl_status_t acl__set_error(const char* msg);

extern "C" int32_t acl_max_vehicles(void) { return acl_amd::kMaxNWide; }

// Diagnostic hook (not part of the public ABI): when set, the next solves
// record phase stamps into stamps[B][kStampStride] (control_params.h).
static unsigned long long* g_stamps = nullptr;
extern "C" void acl_internal_set_stamps(unsigned long long* stamps) { g_stamps = stamps; }

extern "C" size_t acl_solve_workspace_bytes(int32_t n, int32_t B) {
  if (n < 1 || B < 0) return 0;
  return acl_amd::ws_layout(n, B).total;
}

namespace {
// Diagnostic per-launch kernel timing (not part of the public ABI): events
// around each kernel launch, so bench.py can report every kernel's own time.
struct KTiming {
  bool on = false;
  int n[3] = {0, 0, 0};
  hipEvent_t ev[3][64][2] = {};
};
KTiming g_kt;

void kt_record(int kind, int which, hipStream_t s) {
  if (!g_kt.on) return;
  const int i = g_kt.n[kind];
  if (i >= 64) return;
  hipEvent_t& e = g_kt.ev[kind][i][which];
  if (!e) (void)hipEventCreate(&e);
  (void)hipEventRecord(e, s);
  if (which == 1) g_kt.n[kind] = i + 1;
}
}  // namespace

// enable != 0 starts a fresh timing window; 0 stops recording.
extern "C" void acl_internal_kernel_timing(int enable) {
  g_kt.on = enable != 0;
  if (enable) g_kt.n[0] = g_kt.n[1] = g_kt.n[2] = 0;
}

// Sums the recorded launches: ms[k]/count[k] for k = 0 auction kernel,
// 1 gain kernel, 2 collision-avoidance kernel. Synchronises on the events.
extern "C" int acl_internal_kernel_times(double* ms, int* count) {
  for (int k = 0; k < 3; ++k) {
    double t = 0.0;
    for (int i = 0; i < g_kt.n[k]; ++i) {
      float x = 0.f;
      if (hipEventSynchronize(g_kt.ev[k][i][1]) != hipSuccess ||
          hipEventElapsedTime(&x, g_kt.ev[k][i][0], g_kt.ev[k][i][1]) != hipSuccess)
        return -1;
      t += x;
    }
    ms[k] = t;
    count[k] = g_kt.n[k];
  }
  return 0;
}

namespace acl_amd {
// acl_swarm_stats: workgroups stride over the 16-byte records. Every count is
// reduced in the wave first (DPP sums; the histogram by one ballot
// per distinct bin of the wave into lane `bin`'s register), so the LDS
// accumulators take one atomic per wave and key instead of one per record
// (a 1 024-record workgroup's same-address LDS atomics had serialised: 27 us
// at C2). Up to kStatsSmall records run on one workgroup, which writes the
// output words itself (no zeroing memsets before it); larger batches use up
// to kStatsGrid workgroups and integer atomics into the zeroed output words
// (exact, order-free), extrema as u32 bit patterns (emax, and the complement
// of the smallest margin: non-negative floats order like their bits),
// converted by the last workgroup to finish (a done counter).
constexpr int kStatsThreads = 1024, kStatsHist = 64, kStatsKeys = 11, kStatsGrid = 64;
constexpr int kStatsSmall = 16384, kStatsPre = 4;

// (wave sums on DPP: common.h's ACL_WAVE_REDUCE, no LDS round trips)
__device__ __forceinline__ unsigned op_uadd(unsigned a, unsigned b) { return a + b; }

__device__ __forceinline__ unsigned wave_sum_u32(unsigned x) {
  ACL_WAVE_REDUCE(x, op_uadd);
  return (unsigned)__builtin_amdgcn_readlane((int)x, 63);
}

__global__ void __launch_bounds__(kStatsThreads) stats_kernel(const acl_swarm_status_t* st, int B,
                                                              long long* counters, double* ext) {
  // (grid > 1) the 16 bytes of ext serve as scratch until the last workgroup
  // writes them: [0] emax, [1] ~(smallest margin bits) (0 = +inf), [2]
  // workgroups done
  unsigned* scratch = reinterpret_cast<unsigned*>(ext);
  __shared__ unsigned long long cnt[kStatsKeys + kStatsHist];
  __shared__ unsigned emax, mmin;
  __shared__ bool last;
  const int tid = threadIdx.x, lane = tid & 63;
  for (int k = tid; k < kStatsKeys + kStatsHist; k += kStatsThreads) cnt[k] = 0ull;
  if (tid == 0) {
    emax = 0u;
    mmin = 0x7F800000u;  // +inf
  }
  __syncthreads();
  static_assert(kStatsHist == 64, "one histogram bin per lane");
  // per-lane counts in 32 bits: a lane takes at most B / (grid 1 024) records
  // (eff_rounds <= 1 024 each), a wave's sums stay below 2^32 for B < 2^31
  unsigned c[kStatsKeys] = {};
  unsigned hist = 0u;  // this lane's bin of the wave's histogram
  unsigned em = 0u, mm = 0x7F800000u;
  const int stride = gridDim.x * kStatsThreads;
  const uint32_t bits[7] = {ACL_SWARM_VALID, ACL_SWARM_AGREE, ACL_SWARM_CHANGED,
                            ACL_SWARM_NONFINITE, ACL_SWARM_BAD_INPUT, ACL_SWARM_CA_ACTIVE,
                            ACL_SWARM_FRAGILE};
  // one record per lane (ok: the lane has one); wave-uniform control
  auto take = [&](const acl_swarm_status_t& s, bool ok) {
    c[0] += ok ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 7; ++k) c[1 + k] += (s.flags & bits[k]) ? 1u : 0u;
    c[8] += s.n_invalid;
    c[9] += s.n_ca;
    c[10] += s.eff_rounds;
    // the histogram: lane h of the wave counts bin h (kStatsHist == 64), one
    // ballot per distinct bin of the wave (the bin read by readlane: no LDS
    // round trip); added to LDS once per wave below
    const unsigned bin = s.eff_rounds < kStatsHist - 1 ? s.eff_rounds : kStatsHist - 1;
    unsigned long long todo = __ballot(ok);
    while (todo) {
      const int leader = __ffsll((long long)todo) - 1;
      const unsigned lb = (unsigned)__builtin_amdgcn_readlane((int)bin, leader);
      const unsigned long long m = __ballot(bin == lb) & todo;
      hist += (unsigned)lane == lb ? (unsigned)__popcll(m) : 0u;
      todo &= ~m;
    }
    if (ok) {
      em = s.eff_rounds > em ? s.eff_rounds : em;
      const unsigned mb = __float_as_uint(s.margin);
      mm = mb < mm ? mb : mm;
    }
  };
  // kStatsPre records per lane are loaded before any is reduced (their HBM
  // latencies overlap: one round trip per kStatsPre strides, not per stride);
  // the loop bounds are wave-uniform: every lane of a wave iterates together
  for (int b1 = blockIdx.x * kStatsThreads + (tid & ~63); b1 < B; b1 += kStatsPre * stride) {
    acl_swarm_status_t sp[kStatsPre];
#pragma unroll
    for (int u = 0; u < kStatsPre; ++u) {
      const int b = b1 + u * stride + lane;
      sp[u] = acl_swarm_status_t{};
      if (b < B) sp[u] = st[b];
    }
#pragma unroll
    for (int u = 0; u < kStatsPre; ++u)
      if (b1 + u * stride < B) take(sp[u], b1 + u * stride + lane < B);
  }
  unsigned w[kStatsKeys];
#pragma unroll
  for (int k = 0; k < kStatsKeys; ++k) w[k] = wave_sum_u32(c[k]);
  // lane k < kStatsKeys adds key k (one LDS atomic instruction per wave)
  unsigned mine = 0u;
#pragma unroll
  for (int k = 0; k < kStatsKeys; ++k) mine = lane == k ? w[k] : mine;
  if (lane < kStatsKeys && mine) atomicAdd(&cnt[lane], (unsigned long long)mine);
  if (hist) atomicAdd(&cnt[kStatsKeys + lane], (unsigned long long)hist);
  em = wave_max_u32(em);
  mm = ~wave_max_u32(~mm);
  if (lane == 0) {
    atomicMax(&emax, em);
    atomicMin(&mmin, mm);
  }
  __syncthreads();
  if (gridDim.x == 1) {  // the whole batch: write the outputs (no memsets)
    for (int k = tid; k < kStatsKeys + kStatsHist; k += kStatsThreads)
      counters[k] = (long long)cnt[k];
    if (tid == 0) {
      ext[0] = B > 0 ? (double)emax : 0.0;
      ext[1] = B > 0 ? -(double)__uint_as_float(mmin) : -1.0;
    }
    return;
  }
  for (int k = tid; k < kStatsKeys + kStatsHist; k += kStatsThreads)
    if (cnt[k]) atomicAdd(reinterpret_cast<unsigned long long*>(counters + k), cnt[k]);
  if (tid == 0) {
    atomicMax(&scratch[0], emax);
    atomicMax(&scratch[1], ~mmin);
    __threadfence();
    last = atomicAdd(&scratch[2], 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last && tid == 0) {
    __threadfence();
    const unsigned e = atomicAdd(&scratch[0], 0u), m = ~atomicAdd(&scratch[1], 0u);
    ext[0] = B > 0 ? (double)e : 0.0;
    ext[1] = B > 0 ? -(double)__uint_as_float(m) : -1.0;
  }
}
}  // namespace acl_amd

extern "C" acl_status_t acl_swarm_stats(const acl_swarm_status_t* status, int32_t B,
                                        int64_t* counters, double* extrema, void* stream) {
  using namespace acl_amd;
  static_assert(kStatsKeys + kStatsHist == ACL_STATS_COUNTERS, "counter layout");
  if (B < 0) return acl__set_error("acl_swarm_stats: B < 0");
  if (!counters || !extrema || (B > 0 && !status))
    return acl__set_error("acl_swarm_stats: null argument");
  const hipStream_t s = (hipStream_t)stream;
  const int grid =
      B > kStatsSmall ? std::min(kStatsGrid, (B + kStatsThreads - 1) / kStatsThreads) : 1;
  if (grid > 1 &&
      (hipMemsetAsync(counters, 0, ACL_STATS_COUNTERS * sizeof(int64_t), s) != hipSuccess ||
       hipMemsetAsync(extrema, 0, 2 * sizeof(double), s) != hipSuccess))
    return acl__set_error("acl_swarm_stats: hipMemsetAsync failed");
  hipLaunchKernelGGL(stats_kernel, dim3(grid), dim3(kStatsThreads), 0, s, status, B,
                     (long long*)counters, extrema);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  return ACL_OK;
}

extern "C" acl_status_t acl_solve_batch(const acl_formations_t* F, const acl_solve_args_t* a,
                                        void* stream) {
  using namespace acl_amd;
  if (!F || !a) return acl__set_error("acl_solve_batch: null argument");
  const int n = F->n;
  if (n < 1 || n > kMaxNWide) return acl__set_error("acl_solve_batch: n out of range [1, 512]");
  if (a->B < 0) return acl__set_error("acl_solve_batch: B < 0");
  if (a->B == 0) return ACL_OK;
  if (!F->p || !F->adj || !a->fidx || !a->q || !a->P_in || !a->P_out || !a->status)
    return acl__set_error("acl_solve_batch: required pointer is NULL");
  if (F->n_formations < 1) return acl__set_error("acl_solve_batch: n_formations < 1");
  if (!a->workspace)
    return acl__set_error("acl_solve_batch: workspace is NULL (acl_solve_workspace_bytes)");
  if (a->do_control && (!F->gains || !F->gain_off || !a->vel))
    return acl__set_error("acl_solve_batch: do_control needs gains, gain_off and vel");
  if (a->do_control && F->gain_planes != 0 && F->gain_planes != 9 && F->gain_planes != 5)
    return acl__set_error("acl_solve_batch: gain_planes must be 9 (or 0) or 5");
  SolveParams P;
  P.n = n; P.B = a->B; P.F = F->n_formations; P.b0 = 0;
  P.p = F->p; P.adj = F->adj; P.gains = F->gains; P.gain_off = F->gain_off;
  P.fidx = a->fidx; P.q = a->q; P.vel = a->vel; P.P_in = a->P_in; P.P_out = a->P_out;
  P.status = a->status; P.u = a->u; P.u_safe = a->u_safe; P.ca_flag = a->ca_flag;
  P.who = a->who; P.align_Rt = a->align_Rt; P.g = a->cntrl; P.s = a->safety;
  P.early_exit = a->early_exit; P.do_control = a->do_control;
  P.skip_margin = a->skip_margin;
  if (a->P_rows && !a->P_rows_on)
    return acl__set_error("acl_solve_batch: P_rows needs P_rows_on");
  P.P_rows = a->P_rows;
  P.P_rows_on = a->P_rows ? a->P_rows_on : nullptr;
  P.ws = (unsigned char*)a->workspace;
  P.W = ws_layout(n, a->B);
  P.stamps = g_stamps;
  P.gate_margin = a->do_control ? a->gate_margin : nullptr;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (a->do_control) {
    CtlParams& C = P.ctl;
    C.n = n; C.B = a->B; C.b0 = 0;
    C.p = F->p; C.adj = F->adj; C.gains = F->gains; C.gain_off = F->gain_off;
    C.gain_planes = F->gain_planes == 5 ? 5 : 9;
    C.gains_tiled = (C.gain_planes == 5 && n <= kMaxN) ? F->gains_tiled : nullptr;
    C.fidx = a->fidx; C.q = a->q; C.vel = a->vel; C.P_out = a->P_out;
    C.status = a->status;
    C.u = a->u ? a->u : reinterpret_cast<double*>(P.ws + P.W.u);
    C.u_safe = a->u_safe; C.ca_flag = a->ca_flag;
    C.wsPt = reinterpret_cast<const uint16_t*>(P.ws + P.W.pt);
    C.wsMode = P.ws + P.W.mode;
    C.wsRows = reinterpret_cast<const uint16_t*>(P.ws + P.W.rows);
    C.ca_list = reinterpret_cast<unsigned*>(P.ws + P.W.calist);
    C.ca_count = reinterpret_cast<unsigned*>(P.ws + P.W.cacount);
    C.ca_mask = reinterpret_cast<uint64_t*>(P.ws + P.W.camask);
    C.stamps = P.stamps;
    C.g = a->cntrl; C.s = a->safety;
    C.only_nonuniform = 0;
    C.all_uniform = 0;
    C.F = F->n_formations;
    C.gate_margin = a->gate_margin;
    // the list counters ([0] entries, [1] workgroups done): zero unless the
    // caller keeps them zero between calls (ws_persistent)
    if (!a->ws_persistent && hipMemsetAsync(C.ca_count, 0, kCaCounterBytes, s) != hipSuccess)
      return acl__set_error("hipMemsetAsync failed");
  }
  // The control phase runs inside the auction's workgroups (one launch, the
  // gain stream overlapping the auctions) for 5-plane records, at any n (the
  // wide kernel's wide_control for n > 128); the directed gain kernel then
  // takes the swarms with per-vehicle rows.
  const bool fuse = a->do_control && P.ctl.gain_planes == 5;
  kt_record(0, 0, s);
  if (n <= kMaxN) {
    e = launch_auction(P, a->B, s, fuse);
  } else {
    e = launch_wide(P, a->B, s, fuse);
  }
  kt_record(0, 1, s);
  if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  if (!a->do_control) return ACL_OK;
  for (int which = 0; which < 2; ++which) {
    kt_record(1 + which, 0, s);
    e = launch_control(P.ctl, a->B, which == 0 ? (fuse ? 2 : 0) : 1, s);
    kt_record(1 + which, 1, s);
    if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  }
  return ACL_OK;
}

acl_status_t acl_amd::ctl_params(const acl_formations_t* F, const acl_control_args_t* a,
                                 CtlParams& C) {
  using namespace acl_amd;
  if (!F || !a) return acl__set_error("acl_control_batch: null argument");
  const int n = F->n;
  if (n < 1 || n > kMaxNWide) return acl__set_error("acl_control_batch: n out of range [1, 512]");
  if (a->B < 0) return acl__set_error("acl_control_batch: B < 0");
  if (a->B == 0) return ACL_OK;
  if (!F->p || !F->adj || !F->gains || !F->gain_off || !a->fidx || !a->q || !a->vel || !a->P ||
      !a->status || !a->workspace)
    return acl__set_error("acl_control_batch: required pointer is NULL");
  if (F->gain_planes != 0 && F->gain_planes != 9 && F->gain_planes != 5)
    return acl__set_error("acl_control_batch: gain_planes must be 9 (or 0) or 5");
  if (F->n_formations < 1) return acl__set_error("acl_control_batch: n_formations < 1");
  const WsLayout W = ws_layout(n, a->B);
  unsigned char* ws = (unsigned char*)a->workspace;
  C = CtlParams{};
  C.n = n; C.B = a->B; C.b0 = 0;
  C.p = F->p; C.adj = F->adj; C.gains = F->gains; C.gain_off = F->gain_off;
  C.gain_planes = F->gain_planes == 5 ? 5 : 9;
  C.gains_tiled = (C.gain_planes == 5 && n <= kMaxN) ? F->gains_tiled : nullptr;
  C.fidx = a->fidx; C.q = a->q; C.vel = a->vel; C.P_out = a->P;
  C.status = a->status;
  C.u = a->u ? a->u : reinterpret_cast<double*>(ws + W.u);
  C.u_safe = a->u_safe; C.ca_flag = a->ca_flag;
  C.wsPt = reinterpret_cast<const uint16_t*>(ws + W.pt);
  C.wsMode = ws + W.mode;
  C.wsRows = reinterpret_cast<const uint16_t*>(ws + W.rows);
  C.ca_list = reinterpret_cast<unsigned*>(ws + W.calist);
  C.ca_count = reinterpret_cast<unsigned*>(ws + W.cacount);
  C.ca_mask = reinterpret_cast<uint64_t*>(ws + W.camask);
  C.stamps = nullptr;
  C.g = a->cntrl; C.s = a->safety;
  C.only_nonuniform = 0;
  C.all_uniform = 1;  // the hand-off of a given P is one assignment per swarm
  C.F = F->n_formations;
  C.gate_margin = a->gate_margin;
  return ACL_OK;
}

acl_status_t acl_amd::run_control(const acl_formations_t* F, const acl_control_args_t* a,
                                  hipStream_t s, int flags) {
  using namespace acl_amd;
  CtlParams C;
  const acl_status_t st = ctl_params(F, a, C);
  if (st != ACL_OK || a->B == 0) return st;
  if (flags & CTL_MIXED) C.all_uniform = 0;
  if ((flags & CTL_RESET) && hipMemsetAsync(C.ca_count, 0, kCaCounterBytes, s) != hipSuccess)
    return acl__set_error("hipMemsetAsync failed");
  hipError_t e = hipSuccess;
  if (flags & CTL_PREP) {
    e = launch_control_prep(C, a->P, a->B, s);
    if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  }
  for (int which = 0; which < 2; ++which) {
    e = launch_control(C, a->B, which, s);
    if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  }
  return ACL_OK;
}

extern "C" acl_status_t acl_control_batch(const acl_formations_t* F, const acl_control_args_t* a,
                                          void* stream) {
  return acl_amd::run_control(F, a, (hipStream_t)stream, acl_amd::CTL_PREP | acl_amd::CTL_RESET);
}

extern "C" acl_status_t acl_tile_gains(const acl_formations_t* F, double* out, void* stream) {
  using namespace acl_amd;
  if (!F || !out) return acl__set_error("acl_tile_gains: null argument");
  if (F->gain_planes != 5) return acl__set_error("acl_tile_gains: gain_planes must be 5");
  if (F->n < 1 || F->n > kMaxN) return acl__set_error("acl_tile_gains: n out of range [1, 128]");
  if (F->n_formations < 0) return acl__set_error("acl_tile_gains: n_formations < 0");
  if (F->n_formations == 0) return ACL_OK;
  if (!F->adj || !F->gains || !F->gain_off)
    return acl__set_error("acl_tile_gains: required pointer is NULL");
  if (out == F->gains) return acl__set_error("acl_tile_gains: out aliases gains");
  const hipError_t e = launch_tile_gains(F->n, F->n_formations, F->adj, F->gains, F->gain_off,
                                         out, (hipStream_t)stream);
  if (e != hipSuccess) return acl__set_error(hipGetErrorString(e));
  return ACL_OK;
}
