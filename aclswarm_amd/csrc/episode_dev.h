// episode_dev.h -- pieces shared by the episode and trial drivers
// (episode.hip, trial.hip): the episode workspace layout and the
// makeSafeTraj helpers.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/aclswarm_amd.h"
#include "control_params.h"

namespace acl_amd {

constexpr int kEpBlock = 128;  // traj_kernel threads (64 for n <= 64: fewer waves per step)

// Episode workspace: the auction's solve workspace, the control stage's own
// hand-off region (the head of a WsLayout: pt, mode, rows, ...; kept apart
// so that an auction still pending does not overwrite the tables the
// vehicles fly meanwhile -- and the next auction's own rows, P_rows), the
// auction's output and the control stage's output of the current step.
struct EpLayout {
  size_t solve, ctl, Pnew, st, cst, u, us, ca, lat, hcost, hst, total;
};

inline EpLayout ep_layout(int n, int B) {
  EpLayout L;
  const size_t nb = (size_t)n, bb = (size_t)B;
  size_t o = 0;
  L.solve = o; o = ws_al(o + ws_layout(n, B).total);
  L.ctl = o;   o = ws_al(o + ws_layout(n, B).wide);  // pt .. camask: what run_control uses
  L.Pnew = o;  o = ws_al(o + bb * nb * 2);
  L.st = o;    o = ws_al(o + bb * sizeof(acl_swarm_status_t));
  L.cst = o;   o = ws_al(o + bb * sizeof(acl_swarm_status_t));
  L.u = o;     o = ws_al(o + bb * nb * 3 * 8);
  L.us = o;    o = ws_al(o + bb * nb * 3 * 8);
  L.ca = o;    o = ws_al(o + bb * nb);
  L.lat = o;   o = ws_al(o + bb * 4);  // per-swarm auction latency (control steps)
  L.hcost = o; o = ws_al(o + bb * 16);  // ACL_ASSIGN_CENTRAL: the Hungarian's cost pair
  L.hst = o;   o = ws_al(o + bb * 4);   // ... and its status
  L.total = o;
  return L;
}

// utils::rateLimit (utils.h:254-264)
__device__ __forceinline__ void rate_limit(double dt, double lo, double hi, double v0, double& v1) {
  const double upper = v0 + hi * dt;
  const double lower = v0 + lo * dt;
  if (v1 > upper) v1 = upper;
  if (v1 < lower) v1 = lower;
}

// utils::clamp (utils.h:213-227)
__device__ __forceinline__ double clamp_ind(double val, double lower, double upper, bool& clamped) {
  if (val < lower) { clamped = true; return lower; }
  if (val > upper) { clamped = true; return upper; }
  clamped = false;
  return val;
}

// Safety::makeSafeTraj (safety.cpp:330-408) of velocity goal c from goal
// position gp and velocity gv, in place; the vehicle tracks the goal exactly
// (gp, gv <- the new goal)
__device__ __forceinline__ void make_safe_traj(const acl_episode_params_t& ep, double (&gp)[3],
                                               double (&gv)[3], double (&c)[3]) {
  const double dt = ep.control_dt;
  const double amax[3] = {ep.max_accel_xy, ep.max_accel_xy, ep.max_accel_z};
#pragma unroll
  for (int a = 0; a < 3; ++a) rate_limit(dt, -amax[a], amax[a], gv[a], c[a]);
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double next = gp[a] + c[a] * dt;
    bool clamped = false;
    // std::min / std::max (b < a ? b : a, a < b ? b : a)
    const double lo = gp[a] < ep.bounds_min[a] ? gp[a] : ep.bounds_min[a];
    const double hi = ep.bounds_max[a] < gp[a] ? gp[a] : ep.bounds_max[a];
    gp[a] = clamp_ind(next, lo, hi, clamped);
    if (clamped) {
      c[a] = 0.0;
      rate_limit(dt, -amax[a], amax[a], gv[a], c[a]);
    }
    gv[a] = c[a];
  }
}

}  // namespace acl_amd
