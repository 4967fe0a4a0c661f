// control_params.h -- the solve workspace layout and the parameters of the
// kernels acl_solve_batch launches (solve.hip, solve_wide.hip, control.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>

#include "../../include/aclswarm_amd.h"

namespace acl_amd {

// One-time per-device setup (kernel attributes such as the 160 KiB dynamic
// LDS limit are per device): f() runs once for each device it is called on,
// under a mutex; a failure is returned and retried on the next call.
class PerDeviceOnce {
 public:
  template <class F>
  hipError_t run(F&& f) {
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(m_);
    if (d >= 0 && d < 64 && ((done_ >> d) & 1ull)) return hipSuccess;
    e = f();
    if (e == hipSuccess && d >= 0 && d < 64) done_ |= 1ull << d;
    return e;
  }

 private:
  std::mutex m_;
  unsigned long long done_ = 0ull;
};

constexpr int kMaxN = 128;      // LDS-resident auction kernel (auction.hip)
constexpr int kMaxNWide = 512;  // tables-in-HBM auction kernel (solve_wide.hip)

// Solve workspace (acl_solve_workspace_bytes), 256-byte aligned regions:
//   pt      [B][n] u16    the adopted inverse assignment (point -> vehicle)
//                         when every vehicle adopted the same one
//   mode    [B]    u8     0: all vehicles use pt, 1: per-vehicle rows
//   rows    [B][n][n] u16 per-vehicle inverse assignments (mode 1)
//   u       [B][n][3] f64 DistCntrl output when the caller passes u = NULL
//   calist  [B]    u32    swarms with a vehicle whose collisionAvoidance must
//                         finish (appended once per swarm)
//   cacount u32           entries of calist, then the workgroup counters
//                         (kCaCounterBytes, below)
//   camask  [B][NW] u64   the swarm's vehicles within d_avoid_thresh of
//                         another (bit v of word v/64; every word rewritten
//                         by each control step's epilogue)
//   wide    [B] x (T u16 in 8 x 8 tiles, ceil(n/8)^2 * 64 entries): the CBAA `who` table of
//           the n > 128 kernel, which does not fit LDS
//   align   [B] x (out [n][6] f64 the work items' R, t; itm [n] u8 the item of
//           each formation row; u64 smallest alignment gap; i32 item count):
//           align_kernel's results for the n <= 128 auction kernel; for
//           n > 128 align_wide_kernel's (out [n][6] per vehicle, vadj
//           [NW][n] u64, u64 gap, u32 flags)
// The collision list's counters (WsLayout::cacount), u32 words: [0] entries,
// [1] groups done, [kCaGroupStride (1 + g)] workgroups done of group g (the
// collision-avoidance launch's workgroups g, g + kCaGroups, ...: 128 bytes
// apart, so the groups' atomics meet in different cache lines)
constexpr int kCaGroups = 64, kCaGroupStride = 32;
constexpr size_t kCaCounterBytes = (size_t)kCaGroupStride * (1 + kCaGroups) * 4;

struct WsLayout {
  size_t pt, mode, rows, vvalid, u, calist, cacount, camask, wide, wide_stride, align, align_stride,
      total;
};

__host__ __device__ inline size_t ws_al(size_t x) { return (x + 255) & ~(size_t)255; }

__host__ __device__ inline WsLayout ws_layout(int n, int B) {
  WsLayout W;
  const size_t nb = (size_t)n, bb = (size_t)B;
  size_t o = 0;
  W.pt = o;      o = ws_al(o + bb * nb * 2);
  W.mode = o;    o = ws_al(o + bb);
  W.rows = o;    o = ws_al(o + bb * nb * nb * 2);
  W.vvalid = o;  o = ws_al(o + bb * nb);  // [B][n] u8: vehicle's own table valid (rows swarms)
  W.u = o;       o = ws_al(o + bb * nb * 3 * 8);
  W.calist = o;  o = ws_al(o + bb * 4);
  W.cacount = o; o = ws_al(o + kCaCounterBytes);
  W.camask = o;  o = ws_al(o + bb * (size_t)((n + 63) >> 6) * 8);
  W.wide = o;
  W.wide_stride = n > kMaxN ? ws_al((size_t)((n + 7) >> 3) * ((n + 7) >> 3) * 64 * 2) : 0;
  o += bb * W.wide_stride;
  o = ws_al(o);
  W.align = o;
  // n > 128 (align_wide_kernel, solve_wide.hip): out [n][6] f64, the
  // vehicle-space neighbourhood masks vadj [NW][n] u64, the smallest
  // alignment gap (u64 bits) and a flags word
  W.align_stride = n <= kMaxN
                       ? ((nb * 48 + ((nb + 15) & ~(size_t)15) + 16 + 15) & ~(size_t)15)
                       : ((nb * 48 + (size_t)((n + 63) >> 6) * nb * 8 + 16 + 15) & ~(size_t)15);
  o += bb * W.align_stride;
  W.total = o;
  return W;
}

struct CtlParams {
  int n, B, b0;
  const double* p;
  const uint64_t* adj;
  const double* gains;
  const int64_t* gain_off;
  int gain_planes;  // 9 or 5 (acl_formations_t::gain_planes)
  const double* gains_tiled;  // acl_formations_t::gains_tiled (NULL: row-major records)
  const int32_t* fidx;
  const double* q;
  const double* vel;
  const uint16_t* P_out;
  acl_swarm_status_t* status;
  double* u;  // DistCntrl output: the caller's u, or workspace scratch
  double* u_safe;
  uint8_t* ca_flag;
  const uint16_t* wsPt;
  const uint8_t* wsMode;
  const uint16_t* wsRows;
  unsigned* ca_list;   // swarms with close vehicles (WsLayout::calist)
  unsigned* ca_count;
  uint64_t* ca_mask;   // [B][NW] close vehicles per swarm (WsLayout::camask)
  acl_cntrl_gains_t g;
  acl_safety_params_t s;
  int only_nonuniform;  // set by launch_control: gain_kernel skips uniform swarms
  int nb;               // set by launch_control: swarms [b0, b0 + nb) of this launch
  int all_uniform;      // every swarm has one assignment (given P): no gain_kernel pass
  int F;                // formations in the table (fidx range check of the hand-off)
  double* gate_margin;  // [B] optional: min | |e| - thr | / thr of the swarm's gates
  unsigned long long* stamps;  // diagnostic (SolveParams::stamps; NULL = off)
  // control_prep_kernel, episodes only (NULL otherwise): a swarm with
  // keep[b * keep_stride] != 0 flies per-vehicle tables already in wsRows
  // (mode 1, no permutation check)
  const uint8_t* keep = nullptr;
  int keep_stride = 0;
};

// Diagnostic stamps (acl_internal_set_stamps; scripts/phase_profile.py):
// [B][kStampStride] u64 per swarm. Slots 0..7: s_memtime (the XCD's shader
// clock: only differences within one workgroup mean anything) at the end of
// each phase, slot 7 = the end of the fused control phase; slots 8/9:
// s_memrealtime (the 100 MHz clock every XCD shares) at the swarm's start and
// end, for the kernel span and the resident-swarm count; slots 16..31: the
// section counters of the -DACL_*_PROF builds (auction, wide, collision).
constexpr int kStampStride = 32;
constexpr int kStampRt0 = 8, kStampRt1 = 9, kStampSec = 16;

struct SolveParams {
  int n, B, F, b0;
  const double* p;
  const uint64_t* adj;
  const double* gains;
  const int64_t* gain_off;
  const int32_t* fidx;
  const double* q;
  const double* vel;
  const uint16_t* P_in;
  uint16_t* P_out;
  acl_swarm_status_t* status;
  double* u;
  double* u_safe;
  uint8_t* ca_flag;
  uint16_t* who;
  double* align_Rt;
  acl_cntrl_gains_t g;
  acl_safety_params_t s;
  int early_exit;
  int do_control;
  int skip_margin;    // acl_solve_args_t::skip_margin
  const uint16_t* P_rows;    // acl_solve_args_t::P_rows / P_rows_on (optional)
  const uint8_t* P_rows_on;
  unsigned char* ws;  // workspace base (WsLayout)
  WsLayout W;
  unsigned long long* stamps;  // diagnostic: [B][kStampStride] (above; NULL = off)
  double* gate_margin;         // acl_solve_args_t::gate_margin (+inf for BAD_INPUT swarms)
  CtlParams ctl;               // the fused control phase's parameters (auction.hip, FUSE)
};


// misc int slots of the auction kernels' LDS
enum { M_BAD = 0, M_NONFIN = 1, M_NINV = 5, M_AGREE = 6, M_CHANGED = 7, M_NCA = 8,
       M_PINF = 9 /* a formation coordinate is not finite */,
       M_MARG = 10 /* u64: bits of the swarm's minimum decision gap (misc[10..11]) */,
       M_ROWBAD = 12 /* a vehicle's own row (P_rows) failed its check */ };

// Control stage: which = 0 launches the gain kernel for swarms
// [P.b0, P.b0 + nb) (DistCntrl::compute, saturation, the collision test),
// 1 the collisionAvoidance kernel over the listed swarms, 2 the directed
// gain kernel for the swarms with per-vehicle assignments only (after the
// fused auction + control kernel, which did the others).
hipError_t launch_control(const CtlParams& P, int nb, int which, hipStream_t stream);
hipError_t launch_tile_gains(int n, int F, const uint64_t* adj, const double* gains,
                             const int64_t* gain_off, double* out, hipStream_t stream);

// Hand-off of given assignments to the control kernels (acl_control_batch):
// permutation check, inverse assignment, status.
hipError_t launch_control_prep(const CtlParams& P, const uint16_t* Pgiven, int nb,
                               hipStream_t stream);

// acl_control_batch's stages (solve.hip): flags CTL_PREP runs the hand-off
// kernel (permutation check, inverse assignment, status), CTL_RESET zeroes
// the collision-avoidance count first; without them the hand-off of the
// previous call with the same P and workspace is reused (acl_episode_batch).
// CTL_MIXED: some swarms may hold per-vehicle tables (mode 1): the directed
// gain kernel runs after the pair kernel for them.
enum { CTL_PREP = 1, CTL_RESET = 2, CTL_MIXED = 4 };
acl_status_t run_control(const acl_formations_t* F, const acl_control_args_t* a, hipStream_t s,
                         int flags);
// the control stage's parameters for (F, a) (argument checks as
// acl_control_batch); ACL_OK or the error set
acl_status_t ctl_params(const acl_formations_t* F, const acl_control_args_t* a, CtlParams& C);

// The n <= 128 auction kernel (auction.hip).
// fuse: the control phase runs in the auction's workgroups (P.ctl; 5-plane
// gain records) for the swarms whose vehicles all adopted one assignment.
hipError_t launch_auction(const SolveParams& P, int nb, hipStream_t stream, bool fuse = false);

// The n > 128 auction kernel (solve_wide.hip).
// fuse: the control phase runs in the auction's workgroups (P.ctl; 5-plane
// gain records) for the swarms whose vehicles all adopted one assignment.
hipError_t launch_wide(const SolveParams& P, int nb, hipStream_t stream, bool fuse = false);

}  // namespace acl_amd
