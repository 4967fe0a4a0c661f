// episode.hip -- closed-loop batched episodes.
//
// acl_episode_batch flies B swarms for a number of control periods in
// lockstep, reusing the decision-loop kernels of acl_solve_batch /
// acl_control_batch (and acl_hungarian_batch in the centralized mode) and
// adding small kernels:
//
//   adopt_kernel   after an auto-auction: the flush/skip rule of
//                  CoordinationROS::autoauctionCb (coordination_ros.cpp:339-
//                  345) and adoption of a valid, agreed assignment
//                  (auctioneer.cpp:283-292, newAssignmentCb :284-303)
//   central_kernel ACL_ASSIGN_CENTRAL: the operator's Hungarian assignment as
//                  every vehicle's setAssignment + newAssignmentCb
//                  (coordination_ros.cpp:330-343)
//   traj_kernel    Safety::makeSafeTraj (safety.cpp:330-408) with the
//                  utils::rateLimit / clamp helpers (utils.h:213-264), the
//                  perfectly tracking vehicle (q <- goal.pos, vel <-
//                  goal.vel), and the supervisor's windowed predicates
//                  has_converged / has_gridlocked (supervisor.py:297-337)
//
// One workgroup per swarm, threads over vehicles. Both kernels are O(n) per
// swarm and latency-bound; the step's time is the gain stream of the control
// stage (control.hip). Compiled with -ffp-contract=off: every operation is
// one IEEE rounding, so the trajectory step and the supervisor's window sums
// are bit-identical to the restatement in oracle/episode_oracle.py.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/aclswarm_amd.h"
#include "control_params.h"
#include "episode_dev.h"

extern "C" acl_status_t acl__set_error(const char* msg);

namespace acl_amd {

// An auction's latency in control steps, per swarm (acl_episode_params_t::
// auction_latency): fixed, or the reference's timing -- one bid processed per
// auctioneer_dt = 1 ms tick (coordination.launch:23, auctioneer.cpp:139-160)
// and every neighbour's bid needed in each of the 2n rounds
// (auctioneer.cpp:198-241): ceil(2 n d_max 1 ms / control_dt), d_max the
// largest degree of the swarm's formation graph (the slowest vehicle gates
// its neighbours' rounds, and transitively the swarm's).
constexpr double kAuctioneerDt = 0.001;

__global__ void __launch_bounds__(64) latency_kernel(int n, const int32_t* fidx, int F,
                                                     const uint64_t* adj, int mode,
                                                     double control_dt, int32_t* lat) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (mode >= 0) {
    if (lane == 0) lat[b] = mode;
    return;
  }
  const int f = fidx[b];
  const int NW = (n + 63) >> 6;
  int dmax = 0;
  if (f >= 0 && f < F) {
    const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
    for (int i = lane; i < n; i += 64) {
      int d = 0;
      for (int w = 0; w < NW; ++w) {
        unsigned long long x = adj[((size_t)f * n + i) * NW + w];
        if (w == NW - 1) x &= lastmask;
        d += __popcll(x & ~(w == (i >> 6) ? (1ull << (i & 63)) : 0ull));
      }
      dmax = d > dmax ? d : dmax;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int y = __shfl_xor(dmax, o, 64);
    dmax = y > dmax ? y : dmax;
  }
  if (lane == 0) lat[b] = (int32_t)ceil(2.0 * n * dmax * kAuctioneerDt / control_dt);
}

// CoordinationROS::autoauctionCb and the auction's completion.
// mode 0 (an auto-auction step, after the auction kernel ran on every swarm):
//   a swarm flagged by its last completed auction (didConvergeOnInvalid-
//   Assignment) flushes and skips this one (coordination_ros.cpp:339-345);
//   otherwise the auction (re)starts -- a pending one is restarted, :355-358
//   -- and completes after lat[b] steps (lat == NULL or 0: now).
// mode 1 (every other step when auctions take time): a pending auction whose
//   step has come completes.
// Completion, each vehicle as auctioneer.cpp:250-295 (oracle
// episode_oracle.adopt): agreed and valid -- every vehicle adopts the one
// table (P, the control stage's shared row); agreed and invalid -- all
// keep theirs and the swarm skips its next auto-auction; disagreement -- each
// vehicle whose own final table is valid adopts it (its row of the auction's
// per-vehicle hand-off, vvalid), the others keep their own, and the swarm
// flies per-vehicle tables (control mode 1, est.per_vehicle) until an agreed
// valid auction; when any vehicle was left on an invalid table, the swarm's
// next auto-auction is skipped too (that vehicle flushes instead of starting,
// and the others' auction stalls on its START bid). The control hand-off (ctlPt / ctlMode / ctlRows, and the
// control status cst) is written here, so no hand-off pass runs per step.
struct AdoptArgs {
  int n, step, mode;
  const int32_t* lat;
  uint16_t* P;
  const uint16_t* Pnew;
  const acl_swarm_status_t* st;
  const uint16_t* sRows;   // the auction's per-vehicle rows / validity (solve workspace)
  const uint8_t* sValid;
  uint8_t* flush;
  acl_episode_status_t* est;
  uint16_t* ctlPt;
  uint8_t* ctlMode;
  uint16_t* ctlRows;
  acl_swarm_status_t* cst;
};

__global__ void __launch_bounds__(256) adopt_kernel(const AdoptArgs A) {
  const int b = blockIdx.x, tid = threadIdx.x, n = A.n;
  __shared__ int take;  // 0 none, 1 one table, 2 per vehicle
  if (tid == 0) {
    acl_episode_status_t e = A.est[b];
    bool complete = false;
    if (A.mode == 0) {
      if (A.flush[b] != 0) {
        A.flush[b] = 0;
        ++e.n_skipped;
      } else {
        ++e.n_auctions;
        if (A.lat && e.pending_step > 0) ++e.n_restarted;
        const int L = A.lat ? A.lat[b] : 0;
        e.pending_step = L > 0 ? A.step + L + 1 : 0;  // completion step + 1; 0: none
        complete = L <= 0;
      }
    } else if (e.pending_step > 0 && e.pending_step - 1 <= A.step) {
      e.pending_step = 0;
      complete = true;
    }
    take = 0;
    if (complete) {
      const acl_swarm_status_t s = A.st[b];
      const bool valid = (s.flags & ACL_SWARM_VALID) != 0, agree = (s.flags & ACL_SWARM_AGREE) != 0;
      if (agree && valid) {
        take = 1;
        e.per_vehicle = 0;
      } else if (agree) {
        A.flush[b] = 1;
        ++e.n_invalid;
      } else {
        ++e.n_disagree;
        const bool bad = (s.flags & ACL_SWARM_BAD_INPUT) != 0;
        if (s.n_invalid < n && !bad) take = 2;
        // a vehicle left on an invalid table sets invalid_assignment_
        // (auctioneer.cpp:291) and skips its next start; its neighbours'
        // auction then waits on its START bid (bidIterComplete,
        // auctioneer.cpp:419-439) until they restart at the tick after: the
        // swarm's next auction completes nowhere -- the flush rule
        if (s.n_invalid > 0 && !bad) A.flush[b] = 1;
      }
    }
    A.est[b] = e;
  }
  __syncthreads();
  if (take == 0) return;
  const size_t bn = (size_t)b * n;
  if (take == 1) {
    for (int v = tid; v < n; v += 256) {
      const uint16_t pv = A.Pnew[bn + v];
      A.P[bn + v] = pv;
      A.ctlPt[bn + pv] = (uint16_t)v;  // a valid permutation
    }
    if (tid == 0) {
      A.ctlMode[b] = 0;
      A.cst[b] = acl_swarm_status_t{};
    }
    return;
  }
  // per vehicle: the rows of vehicles with a valid table; the others keep
  // theirs (their row as flown so far: the shared row while the swarm was
  // uniform, else their own)
  const bool was_rows = A.ctlMode[b] != 0;
  const uint16_t* pt = A.ctlPt + bn;
  uint16_t* rows = A.ctlRows + bn * n;
  const uint16_t* srows = A.sRows + bn * n;
  const uint8_t* vv = A.sValid + bn;
  for (size_t k = tid; k < (size_t)n * n; k += 256) {
    const int v = (int)(k / n), jj = (int)(k - (size_t)v * n);
    if (vv[v]) rows[k] = srows[k];
    else if (!was_rows) rows[k] = pt[jj];
  }
  for (int v = tid; v < n; v += 256)
    if (vv[v]) A.P[bn + v] = A.Pnew[bn + v];  // the vehicle's own point in its table
  __syncthreads();
  if (tid == 0) {
    A.ctlMode[b] = 1;
    A.est[b].per_vehicle = 1;
    A.cst[b] = acl_swarm_status_t{};
  }
}

// ACL_ASSIGN_CENTRAL: CoordinationROS::autoauctionCb in the centralized
// comparison mode (coordination_ros.cpp:330-343). The operator's assignment
// -- acl_hungarian_batch's P_opt from the current q with last = the swarm's
// P (operator.py:219-240) -- becomes every vehicle's assignment
// (Auctioneer::setAssignment + newAssignmentCb): one table, control mode 0.
// A swarm whose Hungarian problem was BAD_INPUT / NONFINITE keeps its P.
struct CentralArgs {
  int n;
  uint16_t* P;
  const uint16_t* Popt;
  const int32_t* hst;
  acl_episode_status_t* est;
  uint16_t* ctlPt;
  uint8_t* ctlMode;
  acl_swarm_status_t* cst;
};

__global__ void __launch_bounds__(256) central_kernel(const CentralArgs A) {
  const int b = blockIdx.x, tid = threadIdx.x, n = A.n;
  const bool ok = A.hst[b] == 0;  // workgroup-uniform
  if (tid == 0) {
    acl_episode_status_t e = A.est[b];
    if (ok) {
      ++e.n_auctions;
      e.per_vehicle = 0;
    } else {
      ++e.n_invalid;
    }
    A.est[b] = e;
  }
  if (!ok) return;
  const size_t bn = (size_t)b * n;
  for (int v = tid; v < n; v += 256) {
    const uint16_t pv = A.Popt[bn + v];
    A.P[bn + v] = pv;
    A.ctlPt[bn + pv] = (uint16_t)v;  // a permutation (status 0)
  }
  if (tid == 0) {
    A.ctlMode[b] = 0;
    A.cst[b] = acl_swarm_status_t{};
  }
}

struct TrajParams {
  int n, B, step, k, tick;
  double* q;
  double* vel;
  const double* u;
  const double* us;
  const uint8_t* ca;
  const uint16_t* P;
  acl_episode_status_t* est;
  double* ring_u;
  uint8_t* ring_ca;
  double* q_hist;
  double* vel_hist;
  double* u_hist;
  uint8_t* ca_hist;
  uint16_t* P_hist;
  unsigned* ca_count;  // the control stage's collision-avoidance count
  acl_episode_params_t ep;
};

__global__ void __launch_bounds__(kEpBlock) traj_kernel(const TrajParams T) {
  __shared__ int s_all_conv, s_any_grid, s_nca;
  const int n = T.n, b = blockIdx.x, tid = threadIdx.x;
  const acl_episode_params_t ep = T.ep;
  if (tid == 0) {
    s_all_conv = 1;
    s_any_grid = 0;
    s_nca = 0;
    // ca_kernel has consumed the list (stream order): reset for the next step
    if (b == 0) *T.ca_count = 0u;
  }
  __syncthreads();
  const uint32_t m0 = T.est[b].n_samples;  // ticks before this one
  const int L = ep.bufflen;
  int nca = 0;
  for (int v = tid; v < n; v += (int)blockDim.x) {
    const size_t iv = (size_t)b * n + v;
    double gp[3] = {T.q[3 * iv], T.q[3 * iv + 1], T.q[3 * iv + 2]};
    double gv[3] = {T.vel[3 * iv], T.vel[3 * iv + 1], T.vel[3 * iv + 2]};
    double c[3] = {T.us[3 * iv], T.us[3 * iv + 1], T.us[3 * iv + 2]};
    make_safe_traj(ep, gp, gv, c);
    // the vehicle tracks its goal exactly
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      T.q[3 * iv + a] = gp[a];
      T.vel[3 * iv + a] = gv[a];
    }
    const uint8_t cav = T.ca[iv];
    nca += cav != 0;
    const size_t ih = (size_t)T.k * T.B * n + iv;
    if (T.q_hist)
      for (int a = 0; a < 3; ++a) T.q_hist[3 * ih + a] = gp[a];
    if (T.vel_hist)
      for (int a = 0; a < 3; ++a) T.vel_hist[3 * ih + a] = gv[a];
    if (T.u_hist)
      for (int a = 0; a < 3; ++a) T.u_hist[3 * ih + a] = T.u[3 * iv + a];
    if (T.ca_hist) T.ca_hist[ih] = cav;
    if (T.P_hist) T.P_hist[ih] = T.P[iv];
    if (T.tick) {
      // supervisor tick: |voriggoal| (the DistCntrl command) and the CA flag
      // enter the ring; with a full window, the per-vehicle means
      const double u0 = T.u[3 * iv], u1 = T.u[3 * iv + 1], u2 = T.u[3 * iv + 2];
      const double speed = sqrt((u0 * u0 + u1 * u1) + u2 * u2);
      double* ru = T.ring_u + (size_t)b * L * n;
      uint8_t* rc = T.ring_ca + (size_t)b * L * n;
      ru[(size_t)(m0 % L) * n + v] = speed;
      rc[(size_t)(m0 % L) * n + v] = cav;
      const uint32_t m = m0 + 1;
      if (m >= (uint32_t)L) {
        double su = 0.0, sc = 0.0;
        for (int i = 0; i < L; ++i) {  // oldest -> newest (deque order)
          const size_t slot = (size_t)((m - L + i) % L) * n + v;
          su = su + ru[slot];
          sc = sc + (double)rc[slot];
        }
        const double mu = su / (double)L, mc = sc / (double)L;
        if (!(mu < ep.orig_zero_vel_thr)) atomicAnd(&s_all_conv, 0);
        if (mc > ep.avg_active_ca_thr) atomicOr(&s_any_grid, 1);
      }
    }
  }
  if (nca) atomicAdd(&s_nca, nca);
  __syncthreads();
  if (tid == 0) {
    acl_episode_status_t e = T.est[b];
    e.n_ca_steps += (uint32_t)s_nca;
    if (T.tick) {
      e.n_samples = m0 + 1;
      if (m0 + 1 >= (uint32_t)L) {
        e.converged = s_all_conv;
        e.gridlocked = s_any_grid;
        if (s_all_conv && e.converged_step < 0) e.converged_step = T.step;
        if (s_any_grid && e.gridlock_step < 0) e.gridlock_step = T.step;
      }
    }
    T.est[b] = e;
  }
}

}  // namespace acl_amd

extern "C" void acl_default_episode_params(acl_episode_params_t* e) {
  e->control_dt = 0.01;
  e->auction_every = 120;
  e->sample_every = 2;
  e->bufflen = 50;
  e->auction_latency = 0;
  e->max_accel_xy = 0.5;
  e->max_accel_z = 0.8;
  e->bounds_min[0] = -100.0; e->bounds_min[1] = -100.0; e->bounds_min[2] = 0.0;
  e->bounds_max[0] = 100.0;  e->bounds_max[1] = 100.0;  e->bounds_max[2] = 30.0;
  e->orig_zero_vel_thr = 1.0;
  e->avg_active_ca_thr = 0.95;
  e->assignment = ACL_ASSIGN_CBAA;
}

extern "C" size_t acl_episode_workspace_bytes(int32_t n, int32_t B) {
  if (n < 1 || B < 0) return 0;
  return acl_amd::ep_layout(n, B).total;
}

extern "C" acl_status_t acl_episode_batch(const acl_formations_t* F, const acl_episode_args_t* a,
                                          void* stream) {
  using namespace acl_amd;
  if (!F || !a) return acl__set_error("acl_episode_batch: null argument");
  const int n = F->n, B = a->B;
  if (n < 1 || n > kMaxNWide) return acl__set_error("acl_episode_batch: n out of range [1, 512]");
  if (B < 0 || a->steps < 0 || a->step0 < 0)
    return acl__set_error("acl_episode_batch: B, steps and step0 must be >= 0");
  if (B == 0 || a->steps == 0) return ACL_OK;
  if (!a->fidx || !a->q || !a->vel || !a->P || !a->flush || !a->est || !a->ring_u ||
      !a->ring_ca || !a->workspace)
    return acl__set_error("acl_episode_batch: required pointer is NULL");
  const acl_episode_params_t& ep = a->ep;
  if (ep.auction_every < 1 || ep.sample_every < 1 || ep.bufflen < 1 || !(ep.control_dt > 0.0))
    return acl__set_error("acl_episode_batch: auction_every, sample_every, bufflen must be "
                          ">= 1 and control_dt > 0");
  if (ep.assignment != ACL_ASSIGN_CBAA && ep.assignment != ACL_ASSIGN_CENTRAL)
    return acl__set_error("acl_episode_batch: assignment must be ACL_ASSIGN_CBAA or "
                          "ACL_ASSIGN_CENTRAL");
  const bool central = ep.assignment == ACL_ASSIGN_CENTRAL;
  const EpLayout W = ep_layout(n, B);
  unsigned char* ws = (unsigned char*)a->workspace;
  hipStream_t s = (hipStream_t)stream;
  uint16_t* Pnew = reinterpret_cast<uint16_t*>(ws + W.Pnew);
  acl_swarm_status_t* st = reinterpret_cast<acl_swarm_status_t*>(ws + W.st);
  double* u = reinterpret_cast<double*>(ws + W.u);
  double* us = reinterpret_cast<double*>(ws + W.us);
  uint8_t* ca = ws + W.ca;

  const WsLayout WS = ws_layout(n, B);
  unsigned char* wc = ws + W.ctl;  // the control stage's hand-off region

  // every auction starts from the vehicles' own assignments: P (each
  // vehicle's point) and, for swarms flying per-vehicle tables (the control
  // hand-off's mode 1), each vehicle's own table as its row
  // (acl_solve_args_t::P_rows: alignment and neighbours, auctioneer.cpp:
  // 357,369,422-427)
  acl_solve_args_t sa = {};
  sa.B = B; sa.fidx = a->fidx; sa.q = a->q; sa.vel = a->vel; sa.P_in = a->P; sa.P_out = Pnew;
  sa.P_rows = reinterpret_cast<const uint16_t*>(wc + WS.rows);
  sa.P_rows_on = wc + WS.mode;
  sa.status = st; sa.workspace = ws + W.solve;
  sa.cntrl = a->cntrl; sa.safety = a->safety; sa.early_exit = 1; sa.do_control = 0;
  sa.skip_margin = 1;  // the episode reads assignments and flags, never the decision margin
  acl_control_args_t cs = {};
  cs.B = B; cs.fidx = a->fidx; cs.q = a->q; cs.vel = a->vel; cs.P = a->P;
  cs.u = u; cs.u_safe = us; cs.ca_flag = ca;
  cs.status = reinterpret_cast<acl_swarm_status_t*>(ws + W.cst);
  cs.workspace = wc; cs.cntrl = a->cntrl; cs.safety = a->safety;

  TrajParams T;
  T.n = n; T.B = B; T.q = a->q; T.vel = a->vel; T.u = u; T.us = us; T.ca = ca; T.P = a->P;
  T.est = a->est; T.ring_u = a->ring_u; T.ring_ca = a->ring_ca;
  T.q_hist = a->q_hist; T.vel_hist = a->vel_hist; T.u_hist = a->u_hist; T.ca_hist = a->ca_hist; T.P_hist = a->P_hist;
  T.ep = ep;
  // the collision-avoidance count is zeroed by traj_kernel after each step
  T.ca_count = reinterpret_cast<unsigned*>(wc + WS.cacount);

  // The call's hand-off, before its first auction: swarms flying one
  // assignment get the inverse of P (permutation check, as
  // acl_control_batch); swarms flying per-vehicle tables (est.per_vehicle,
  // from an earlier call on this workspace) keep theirs.
  {
    CtlParams C;
    const acl_status_t r = ctl_params(F, &cs, C);
    if (r != ACL_OK) return r;
    C.keep = reinterpret_cast<const uint8_t*>(a->est) + offsetof(acl_episode_status_t, per_vehicle);
    C.keep_stride = (int)sizeof(acl_episode_status_t);
    if (hipMemsetAsync(C.ca_count, 0, kCaCounterBytes, s) != hipSuccess)
      return acl__set_error("hipMemsetAsync failed");
    if (launch_control_prep(C, a->P, B, s) != hipSuccess)
      return acl__set_error("control_prep launch failed");
  }
  AdoptArgs A;
  A.n = n; A.lat = nullptr; A.P = a->P; A.Pnew = Pnew; A.st = st;
  A.sRows = reinterpret_cast<const uint16_t*>(ws + W.solve + WS.rows);
  A.sValid = ws + W.solve + WS.vvalid;
  A.flush = a->flush; A.est = a->est;
  A.ctlPt = reinterpret_cast<uint16_t*>(wc + WS.pt);
  A.ctlMode = wc + WS.mode;
  A.ctlRows = reinterpret_cast<uint16_t*>(wc + WS.rows);
  A.cst = cs.status;
  // ACL_ASSIGN_CENTRAL: the operator's Hungarian from the swarm's current P
  acl_hungarian_args_t ha = {};
  ha.B = B; ha.fidx = a->fidx; ha.q = a->q; ha.P_last = a->P; ha.P_opt = Pnew;
  ha.cost = reinterpret_cast<double*>(ws + W.hcost);
  ha.status = reinterpret_cast<int32_t*>(ws + W.hst);
  CentralArgs CA;
  CA.n = n; CA.P = a->P; CA.Popt = Pnew; CA.hst = ha.status; CA.est = a->est;
  CA.ctlPt = A.ctlPt; CA.ctlMode = A.ctlMode; CA.cst = A.cst;
  // auctions that take time: each swarm's latency in control steps
  // (the centralized mode applies its assignment at the auto-auction itself)
  const bool timed = !central && ep.auction_latency != 0;
  int32_t* lat = reinterpret_cast<int32_t*>(ws + W.lat);
  if (timed) {
    hipLaunchKernelGGL(latency_kernel, dim3(B), dim3(64), 0, s, n, a->fidx, F->n_formations,
                       F->adj, ep.auction_latency < 0 ? -1 : ep.auction_latency, ep.control_dt,
                       lat);
    if (hipGetLastError() != hipSuccess) return acl__set_error("latency_kernel launch failed");
    A.lat = lat;
  }
  for (int k = 0; k < a->steps; ++k) {
    const int step = a->step0 + k;
    A.step = step;
    if (step % ep.auction_every == 0 && central) {
      const acl_status_t r = acl_hungarian_batch(F, &ha, stream);
      if (r != ACL_OK) return r;
      hipLaunchKernelGGL(central_kernel, dim3(B), dim3(256), 0, s, CA);
      if (hipGetLastError() != hipSuccess) return acl__set_error("central_kernel launch failed");
    } else if (step % ep.auction_every == 0) {
      const acl_status_t r = acl_solve_batch(F, &sa, stream);
      if (r != ACL_OK) return r;
      A.mode = 0;
      hipLaunchKernelGGL(adopt_kernel, dim3(B), dim3(256), 0, s, A);
      if (hipGetLastError() != hipSuccess) return acl__set_error("adopt_kernel launch failed");
    } else if (timed) {
      // a pending auction completing at this step: adopt_kernel writes those
      // swarms' control hand-off itself
      A.mode = 1;
      hipLaunchKernelGGL(adopt_kernel, dim3(B), dim3(256), 0, s, A);
      if (hipGetLastError() != hipSuccess) return acl__set_error("adopt_kernel launch failed");
    }
    const acl_status_t r = run_control(F, &cs, s, CTL_MIXED);
    if (r != ACL_OK) return r;
    T.step = step;
    T.k = k;
    T.tick = (step % ep.sample_every) == 0;
    hipLaunchKernelGGL(traj_kernel, dim3(B), dim3(n <= 64 ? 64 : kEpBlock), 0, s, T);
    if (hipGetLastError() != hipSuccess) return acl__set_error("traj_kernel launch failed");
  }
  return ACL_OK;
}
