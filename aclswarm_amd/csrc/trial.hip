// trial.hip -- batched Monte-Carlo trials (the widening of
// row f1): aclswarm_sim's supervisor (aclswarm_sim/nodes/supervisor.py) over
// the closed loop of acl_episode_batch, B independent trials in lockstep.
//
// One control step (acl_trial_batch's host loop; every launch is B
// workgroups, one per swarm, threads over vehicles):
//
//   trial_pre_kernel    a formation the last supervisor tick requested is
//                       committed (CoordinationROS::spin, coordination_ros.cpp:
//                       95-153: controllers stop and send one zero command,
//                       Auctioneer::setFormation resets the assignment to
//                       identity, auctioneer.cpp:42-62; the first
//                       auto-auction is due form_settle_time later); each
//                       swarm's auto-auction countdown (autoauctionCb, :322-
//                       359) and the flush rule (:339-345) decide whether its
//                       auction runs this step: the swarms that do not run
//                       one get formation index -1, so the batched auction
//                       (acl_solve_batch / acl_hungarian_batch) treats them as
//                       BAD_INPUT and reads nothing of them
//   acl_solve_batch     CBAA from every vehicle's own assignment (as the
//   | hungarian_batch   episode), or the operator's Hungarian (ACL_ASSIGN_
//                       CENTRAL, coordination_ros.cpp:330-343)
//   trial_adopt_kernel  each vehicle's adoption (auctioneer.cpp:250-295,
//                       shouldUseAssignment :310-321), its controller's start
//                       on its first assignment (newAssignmentCb, :284-303),
//                       vehicle 0's assignment message to the supervisor
//                       (supervisor.py:147-150) and its count while logging
//   run_control         DistCntrl + Safety for every swarm (control.hip)
//   trial_traj_kernel   makeSafeTraj of the running controllers' safe
//                       commands (safety.cpp:330-408), the zero command at a
//                       commit, the last goal held by stopped controllers
//                       (safety.cpp:268-290)
//   trial_tick_kernel   every sample_every steps, one supervisor tick
//                       (supervisor.py:160-236): timer, the state machine,
//                       the predicates with their own sample buffers
//                       (:297-337), logging (:238-265,376-402) and
//                       log_signals (:452-487), the watchdog (:229-232)
//
// Compiled with -ffp-contract=off: the supervisor's window sums, filters and
// distance sums are the oracle's operations in the oracle's order
// (oracle/trial_oracle.py), bit for bit.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/aclswarm_amd.h"
#include "control_params.h"
#include "episode_dev.h"

extern "C" acl_status_t acl__set_error(const char* msg);

namespace acl_amd {

constexpr int kTrBlock = 128;

// the trial workspace: the episode's layout (auction workspace, control
// hand-off, auction and control outputs) and three per-step arrays
struct TrLayout {
  EpLayout E;
  size_t afidx, due, zstep, total;
};

inline TrLayout tr_layout(int n, int B) {
  TrLayout L;
  L.E = ep_layout(n, B);
  const size_t bb = (size_t)B;
  size_t o = L.E.total;
  L.afidx = o; o = ws_al(o + bb * 4);  // this step's auction: the formation, or -1
  L.due = o;   o = ws_al(o + bb);      // the swarm's auction runs this step
  L.zstep = o; o = ws_al(o + bb);      // the swarm commits a formation this step
  L.total = o;
  return L;
}

struct TrialDev {
  int n, B, K, step, k;
  int F;  // formations in the table (acl_trial_init: 0, no range to check yet)
  int central;
  const int32_t* fseq;
  int32_t* fidx;
  double* q;
  double* vel;
  uint16_t* P;
  uint8_t* flush;
  acl_trial_status_t* ts;
  uint8_t* ctl_on;
  double* ring_u;
  uint8_t* ring_ca;
  double* posf;
  double* dist;
  double* t_conv;
  double* t_avoid;
  int32_t* n_assign;
  // workspace
  int32_t* afidx;
  uint8_t* due;
  uint8_t* zstep;
  const uint16_t* Pnew;
  const acl_swarm_status_t* st;
  const uint16_t* sRows;
  const uint8_t* sValid;
  const int32_t* hst;
  uint16_t* ctlPt;
  uint8_t* ctlMode;
  uint16_t* ctlRows;
  acl_swarm_status_t* cst;
  const double* u;
  const double* us;
  const uint8_t* ca;
  unsigned* ca_count;
  // histories (optional)
  double* q_hist;
  double* vel_hist;
  double* u_hist;
  uint8_t* ca_hist;
  uint8_t* ctl_hist;
  uint16_t* P_hist;
  int32_t* state_hist;
  acl_trial_params_t tp;
};

// ---- the start of a trial (acl_trial_init) ----------------------------------
__global__ void __launch_bounds__(kTrBlock) trial_init_kernel(const TrialDev D) {
  const int b = blockIdx.x, tid = threadIdx.x, n = D.n, K = D.K;
  const size_t bn = (size_t)b * n;
  const int L = D.tp.ep.bufflen;
  for (int v = tid; v < n; v += kTrBlock) {
    D.P[bn + v] = (uint16_t)v;  // before any formation: the identity (setFormation)
    D.ctlPt[bn + v] = (uint16_t)v;
    D.ctl_on[bn + v] = 0;
    D.dist[bn + v] = 0.0;
    D.posf[2 * bn + v] = 0.0;
    D.posf[2 * bn + n + v] = 0.0;
  }
  for (int k = tid; k < K; k += kTrBlock) {
    D.t_conv[(size_t)b * K + k] = 0.0;
    D.t_avoid[(size_t)b * K + k] = 0.0;
    D.n_assign[(size_t)b * K + k] = 0;
  }
  for (size_t k = tid; k < (size_t)L * n; k += kTrBlock) {
    D.ring_u[(size_t)b * L * n + k] = 0.0;
    D.ring_ca[(size_t)b * L * n + k] = 0;
  }
  if (tid == 0) {
    acl_trial_status_t t = {};
    t.state = ACL_TRIAL_HOVERING;
    t.last_state = 0;  // (None)
    t.timer_ticks = -1;
    t.formation = -1;
    t.t_start = t.t_grid = 0;
    t.done_step = -1;
    D.ts[b] = t;
    D.flush[b] = 0;
    D.fidx[b] = D.fseq[(size_t)b * K];  // (range-checked at every step: trial_pre_kernel)
    D.ctlMode[b] = 0;
    D.cst[b] = acl_swarm_status_t{};
  }
}

// ---- 1. commit / schedule ---------------------------------------------------
__global__ void __launch_bounds__(64) trial_pre_kernel(const TrialDev D) {
  const int b = blockIdx.x, tid = threadIdx.x, n = D.n;
  const size_t bn = (size_t)b * n;
  acl_trial_status_t t = D.ts[b];  // (every thread: uniform decisions)
  int due = 0, zs = 0, f = D.fidx[b];
  // a formation index outside the table ends the trial before anything of
  // the table is read (the control stage reads fidx[b] every step)
  bool fbad = false;
  for (int k = 0; k < D.K; ++k) {
    const int x = D.fseq[(size_t)b * D.K + k];
    fbad |= x < 0 || x >= D.F;
  }
  if (fbad && t.done_step < 0) {
    t.last_state = t.state;
    t.state = ACL_TRIAL_TERMINATE;
    t.done_step = D.step;
  }
  if (fbad) f = 0;
  if (t.done_step < 0) {
    bool now = false;
    if (t.commit) {
      // the formation the supervisor requested: controllers stop (one zero
      // command), the assignment resets to identity, auctions restart after
      // form_settle_time. (invalid_assignment_ -- the flush flag -- is kept:
      // setFormation does not clear it.)
      f = D.fseq[(size_t)b * D.K + t.formation];
      for (int v = tid; v < n; v += 64) {
        D.P[bn + v] = (uint16_t)v;
        D.ctlPt[bn + v] = (uint16_t)v;
        D.ctl_on[bn + v] = 0;
      }
      zs = 1;
      t.commit = 0;
      t.per_vehicle = 0;
      t.next_auction = D.tp.settle_steps;
      now = t.next_auction <= 0;
      if (now) t.next_auction = D.tp.ep.auction_every;
    } else if (t.next_auction > 0) {
      if (--t.next_auction == 0) {
        now = true;
        t.next_auction = D.tp.ep.auction_every;
      }
    }
    if (now) {
      if (!D.central && D.flush[b]) {
        // didConvergeOnInvalidAssignment: flush and skip (coordination_ros.cpp:339-345)
        if (tid == 0) D.flush[b] = 0;
        ++t.n_skipped;
      } else {
        due = 1;
      }
    }
  }
  if (tid == 0) {
    if (fbad) D.fidx[b] = 0;
    if (zs) {
      D.fidx[b] = f;
      D.ctlMode[b] = 0;
      D.cst[b] = acl_swarm_status_t{};
    }
    D.afidx[b] = due ? f : -1;
    D.due[b] = (uint8_t)due;
    D.zstep[b] = (uint8_t)zs;
    D.ts[b] = t;
  }
}

// ---- 2. adoption ------------------------------------------------------------
__global__ void __launch_bounds__(256) trial_adopt_kernel(const TrialDev D) {
  const int b = blockIdx.x, tid = threadIdx.x, n = D.n;
  if (!D.due[b]) return;  // workgroup-uniform
  __shared__ int take, v0_adopts, changed0;
  __shared__ acl_trial_status_t S;
  const size_t bn = (size_t)b * n;
  if (tid == 0) {
    S = D.ts[b];
    take = 0;
    v0_adopts = 0;
    changed0 = 0;
    if (D.central) {
      // the operator's assignment applied to every vehicle
      if (D.hst[b] == 0) {
        ++S.n_auctions;
        take = 1;
        v0_adopts = 1;
      } else {
        ++S.n_invalid;
      }
    } else {
      ++S.n_auctions;
      const acl_swarm_status_t s = D.st[b];
      const bool valid = (s.flags & ACL_SWARM_VALID) != 0, agree = (s.flags & ACL_SWARM_AGREE) != 0;
      if (agree && valid) {
        take = 1;
        v0_adopts = 1;
      } else if (agree) {
        D.flush[b] = 1;
        ++S.n_invalid;
      } else {
        ++S.n_disagree;
        const bool bad = (s.flags & ACL_SWARM_BAD_INPUT) != 0;
        if (s.n_invalid < n && !bad) {
          take = 2;
          v0_adopts = D.sValid[bn] != 0;
        }
        if (s.n_invalid > 0 && !bad) D.flush[b] = 1;
      }
    }
  }
  __syncthreads();
  if (take == 0) {
    if (tid == 0) D.ts[b] = S;
    return;
  }
  // vehicle 0's table before and after (formation point -> vehicle): its
  // assignment message needs a change (shouldUseAssignment, auctioneer.cpp:
  // 310-321) unless it is the formation's first (formation_just_received_ /
  // first_assignment_ -- the vehicle's controller not started yet)
  const bool was_rows = D.ctlMode[b] != 0;
  if (v0_adopts) {
    const uint16_t* old0 = was_rows ? D.ctlRows + bn * n : D.ctlPt + bn;
    int ch = 0;
    if (take == 1) {
      for (int v = tid; v < n; v += 256) ch |= old0[D.Pnew[bn + v]] != (uint16_t)v;
    } else {
      const uint16_t* new0 = D.sRows + bn * n;
      for (int j = tid; j < n; j += 256) ch |= old0[j] != new0[j];
    }
    if (ch) atomicOr(&changed0, 1);
  }
  __syncthreads();
  const bool first0 = D.ctl_on[bn] == 0;
  if (take == 1) {
    for (int v = tid; v < n; v += 256) {
      const uint16_t pv = D.Pnew[bn + v];
      D.P[bn + v] = pv;
      D.ctlPt[bn + pv] = (uint16_t)v;
    }
    __syncthreads();  // (first0 read above by every thread before ctl_on changes)
    for (int v = tid; v < n; v += 256) D.ctl_on[bn + v] = 1;
    if (tid == 0) {
      D.ctlMode[b] = 0;
      D.cst[b] = acl_swarm_status_t{};
      S.per_vehicle = 0;
    }
  } else {
    // per vehicle: the rows of the vehicles with a valid table; the others
    // keep theirs (as acl_episode_batch's adopt_kernel)
    const uint16_t* pt = D.ctlPt + bn;
    uint16_t* rows = D.ctlRows + bn * n;
    const uint16_t* srows = D.sRows + bn * n;
    const uint8_t* vv = D.sValid + bn;
    for (size_t k = tid; k < (size_t)n * n; k += 256) {
      const int v = (int)(k / n), jj = (int)(k - (size_t)v * n);
      if (vv[v]) rows[k] = srows[k];
      else if (!was_rows) rows[k] = pt[jj];
    }
    __syncthreads();
    for (int v = tid; v < n; v += 256)
      if (vv[v]) {
        D.P[bn + v] = D.Pnew[bn + v];
        D.ctl_on[bn + v] = 1;
      }
    if (tid == 0) {
      D.ctlMode[b] = 1;
      D.cst[b] = acl_swarm_status_t{};
      S.per_vehicle = 1;
    }
  }
  if (tid == 0) {
    if (v0_adopts && (first0 || changed0)) {
      // vehicle 0's assignment message (supervisor.py:147-150)
      S.received = 1;
      if (S.logging && S.formation >= 0) ++D.n_assign[(size_t)b * D.K + S.formation];
    }
    D.ts[b] = S;
  }
}

// ---- 3. trajectories --------------------------------------------------------
__global__ void __launch_bounds__(kTrBlock) trial_traj_kernel(const TrialDev D) {
  const int b = blockIdx.x, tid = threadIdx.x, n = D.n;
  const size_t bn = (size_t)b * n;
  if (tid == 0 && b == 0) *D.ca_count = 0u;  // the control stage's CA list, consumed
  const acl_trial_status_t t = D.ts[b];
  const bool done = t.done_step >= 0;
  const bool zs = D.zstep[b] != 0;
  const acl_episode_params_t& ep = D.tp.ep;
  for (int v = tid; v < n; v += kTrBlock) {
    const size_t iv = bn + v;
    double gp[3] = {D.q[3 * iv], D.q[3 * iv + 1], D.q[3 * iv + 2]};
    double gv[3] = {D.vel[3 * iv], D.vel[3 * iv + 1], D.vel[3 * iv + 2]};
    const bool on = !done && D.ctl_on[iv] != 0;
    if (on) {
      double c[3] = {D.us[3 * iv], D.us[3 * iv + 1], D.us[3 * iv + 2]};
      make_safe_traj(ep, gp, gv, c);
    } else if (!done && zs) {
      double c[3] = {0.0, 0.0, 0.0};  // sendZeroControl (coordination_ros.cpp:101)
      make_safe_traj(ep, gp, gv, c);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      D.q[3 * iv + a] = gp[a];
      D.vel[3 * iv + a] = gv[a];
    }
    const size_t ih = (size_t)D.k * D.B * n + iv;
    if (D.q_hist)
      for (int a = 0; a < 3; ++a) D.q_hist[3 * ih + a] = gp[a];
    if (D.vel_hist)
      for (int a = 0; a < 3; ++a) D.vel_hist[3 * ih + a] = gv[a];
    if (D.u_hist)
      for (int a = 0; a < 3; ++a) D.u_hist[3 * ih + a] = on ? D.u[3 * iv + a] : 0.0;
    if (D.ca_hist) D.ca_hist[ih] = on ? D.ca[iv] : 0;
    if (D.ctl_hist) D.ctl_hist[ih] = on ? 1 : 0;
    if (D.P_hist) D.P_hist[ih] = D.P[iv];
  }
  if (D.state_hist && tid == 0) D.state_hist[(size_t)D.k * D.B + b] = t.state;
}

// ---- 4. the supervisor tick -------------------------------------------------
// Every thread follows the same control flow (the state is read from LDS);
// thread 0 writes it, with a barrier before the next read.
__global__ void __launch_bounds__(kTrBlock) trial_tick_kernel(const TrialDev D) {
  __shared__ acl_trial_status_t S;
  __shared__ int flag;
  const int b = blockIdx.x, tid = threadIdx.x, n = D.n, K = D.K;
  const size_t bn = (size_t)b * n;
  const acl_trial_params_t& tp = D.tp;
  const int L = tp.ep.bufflen;
  const int step = D.step;
  const double dt = tp.ep.control_dt;
  if (tid == 0) S = D.ts[b];
  __syncthreads();
  if (S.done_step >= 0) return;  // workgroup-uniform

  // this tick's samples: |voriggoal| (the last DistCntrl command; the zero
  // command of a stopped controller) and collision_avoidance_active
  auto speed = [&](int v) -> double {
    if (!D.ctl_on[bn + v]) return 0.0;
    const double* u = D.u + 3 * (bn + v);
    return sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
  };
  auto caf = [&](int v) -> uint8_t { return D.ctl_on[bn + v] ? (D.ca[bn + v] != 0) : 0; };

  // a predicate's sample enters its deque (maxlen BUFFLEN); with the deque
  // full, the per-vehicle window means, oldest -> newest, / BUFFLEN
  auto push = [&](bool conv) {
    const int slot = conv ? S.conv_head : S.grid_head;
    for (int v = tid; v < n; v += kTrBlock) {
      if (conv) D.ring_u[((size_t)b * L + slot) * n + v] = speed(v);
      else D.ring_ca[((size_t)b * L + slot) * n + v] = caf(v);
    }
    __syncthreads();
    if (tid == 0) {
      if (conv) {
        S.conv_head = (slot + 1) % L;
        S.conv_len = S.conv_len + 1 < L ? S.conv_len + 1 : L;
      } else {
        S.grid_head = (slot + 1) % L;
        S.grid_len = S.grid_len + 1 < L ? S.grid_len + 1 : L;
      }
      flag = conv ? 1 : 0;
    }
    __syncthreads();
  };
  // has_converged (supervisor.py:297-316)
  auto has_converged = [&]() -> bool {
    push(true);
    if (S.conv_len < L) return false;
    const int old = S.conv_head;
    bool ok = true;
    for (int v = tid; v < n; v += kTrBlock) {
      double su = 0.0;
      for (int i = 0; i < L; ++i) su = su + D.ring_u[((size_t)b * L + (old + i) % L) * n + v];
      ok &= su / (double)L < tp.ep.orig_zero_vel_thr;
    }
    if (!ok) atomicAnd(&flag, 0);
    __syncthreads();
    const bool r = flag != 0;
    __syncthreads();
    return r;
  };
  // has_gridlocked (supervisor.py:318-337)
  auto has_gridlocked = [&]() -> bool {
    push(false);
    if (S.grid_len < L) return false;
    const int old = S.grid_head;
    bool any = false;
    for (int v = tid; v < n; v += kTrBlock) {
      double sc = 0.0;
      for (int i = 0; i < L; ++i)
        sc = sc + (double)D.ring_ca[((size_t)b * L + (old + i) % L) * n + v];
      any |= sc / (double)L > tp.ep.avg_active_ca_thr;
    }
    if (any) atomicOr(&flag, 1);
    __syncthreads();
    const bool r = flag != 0;
    __syncthreads();
    return r;
  };
  // has_left_gridlock (supervisor.py:339-348)
  auto has_left_gridlock = [&]() -> bool {
    const bool g = has_gridlocked();
    if (S.grid_len < L) return false;
    return !g;
  };
  auto elapsed = [&](double secs) {
    return (double)S.timer_ticks / (double)tp.tick_rate >= secs;
  };
  // next_state (supervisor.py:238-265)
  auto next_state = [&](int ns, bool reset) {
    __syncthreads();
    if (tid == 0) {
      S.last_state = S.state;
      S.state = ns;
      S.timer_ticks = -1;
      if (reset) S.conv_len = S.conv_head = S.grid_len = S.grid_head = 0;
      if (ns == ACL_TRIAL_GRIDLOCK) S.t_grid = step;
      if (S.last_state == ACL_TRIAL_GRIDLOCK && S.formation >= 0)
        D.t_avoid[(size_t)b * K + S.formation] = (double)(step - S.t_grid) * dt;
    }
    __syncthreads();
  };
  // start_logging / stop_logging (supervisor.py:376-402)
  auto start_logging = [&]() {
    if (tid == 0 && !S.logging) {
      D.n_assign[(size_t)b * K + S.formation] = 1;
      D.t_avoid[(size_t)b * K + S.formation] = 0.0;
      S.t_start = step;
      S.logging = 1;
    }
    __syncthreads();
  };
  auto stop_logging = [&]() {
    if (tid == 0 && S.logging) {
      S.logging = 0;
      D.t_conv[(size_t)b * K + S.formation] = (double)(step - S.t_start) * dt;
    }
    __syncthreads();
  };

  if (tid == 0) S.timer_ticks += 1;
  __syncthreads();
  bool finished = false;
  switch (S.state) {  // (workgroup-uniform)
    case ACL_TRIAL_HOVERING:
      if (elapsed(tp.hover_wait)) {
        if (S.formation == K - 1) {  // has_cycled_through_formations
          next_state(ACL_TRIAL_COMPLETE, true);
        } else {
          // next_formation: the operator sends the next formation
          if (tid == 0) {
            S.formation += 1;
            S.received = 0;
            S.commit = 1;
          }
          next_state(ACL_TRIAL_WAITING_ON_ASSIGNMENT, true);
        }
      }
      break;
    case ACL_TRIAL_WAITING_ON_ASSIGNMENT:
      if (S.received) {
        start_logging();
        next_state(ACL_TRIAL_FLYING, true);
      } else if (elapsed(tp.assignment_timeout)) {
        next_state(ACL_TRIAL_TERMINATE, true);
      }
      break;
    case ACL_TRIAL_FLYING:
      if (elapsed(tp.formation_received_wait)) {
        if (has_converged()) next_state(ACL_TRIAL_IN_FORMATION, false);
        else if (has_gridlocked()) next_state(ACL_TRIAL_GRIDLOCK, true);
      }
      break;
    case ACL_TRIAL_IN_FORMATION:
      if (elapsed(tp.converged_wait)) {
        stop_logging();
        next_state(ACL_TRIAL_HOVERING, true);
      } else if (!has_converged()) {
        next_state(ACL_TRIAL_FLYING, true);
      }
      break;
    case ACL_TRIAL_GRIDLOCK:
      if (has_left_gridlock()) next_state(ACL_TRIAL_FLYING, true);
      else if (elapsed(tp.gridlock_timeout)) next_state(ACL_TRIAL_TERMINATE, true);
      break;
    default:  // COMPLETE: complete() writes the record; TERMINATE: terminate()
      finished = true;
      break;
  }
  // log_signals (supervisor.py:452-487): x / y smoothed, planar distance
  if (S.logging) {
    const double a = tp.alpha, om = 1.0 - tp.alpha;
    double* px = D.posf + 2 * bn;
    double* py = px + n;
    for (int v = tid; v < n; v += kTrBlock) {
      const double x = D.q[3 * (bn + v)], y = D.q[3 * (bn + v) + 1];
      if (!S.log_init) {
        px[v] = x;
        py[v] = y;
      }
      const double lx = px[v], ly = py[v];
      const double nx = a * lx + om * x, ny = a * ly + om * y;
      px[v] = nx;
      py[v] = ny;
      const double dx = fabs(nx - lx), dy = fabs(ny - ly);
      D.dist[bn + v] = D.dist[bn + v] + sqrt(dx * dx + dy * dy);
    }
    __syncthreads();
    if (tid == 0) S.log_init = 1;
  }
  if (tid == 0) {
    if (finished) {
      S.done_step = step;
    } else {
      // the trial watchdog (supervisor.py:229-232): the tick's time since the
      // first tick past TRIAL_TIMEOUT
      const int k = S.ticks;
      if ((double)k / (double)tp.tick_rate > tp.trial_timeout) {
        S.last_state = S.state;
        S.state = ACL_TRIAL_TERMINATE;
        S.timer_ticks = -1;
        S.conv_len = S.conv_head = S.grid_len = S.grid_head = 0;
        if (S.last_state == ACL_TRIAL_GRIDLOCK && S.formation >= 0)
          D.t_avoid[(size_t)b * K + S.formation] = (double)(step - S.t_grid) * dt;
      }
    }
    S.ticks += 1;
    D.ts[b] = S;
    if (D.state_hist) D.state_hist[(size_t)D.k * D.B + b] = S.state;
  }
}

}  // namespace acl_amd

extern "C" void acl_default_trial_params(acl_trial_params_t* t) {
  acl_default_episode_params(&t->ep);
  t->tick_rate = 50;
  t->settle_steps = 150;
  t->hover_wait = 5.0;
  t->assignment_timeout = 20.0;
  t->formation_received_wait = 1.0;
  t->converged_wait = 1.0;
  t->gridlock_timeout = 90.0;
  t->trial_timeout = 600.0;
  t->alpha = 0.98;
}

extern "C" size_t acl_trial_workspace_bytes(int32_t n, int32_t B) {
  if (n < 1 || B < 0) return 0;
  return acl_amd::tr_layout(n, B).total;
}

namespace {

acl_status_t trial_check(const acl_trial_args_t* a, int n, const char* who) {
  static char msg[160];
  auto fail = [&](const char* what) {
    snprintf(msg, sizeof(msg), "%s: %s", who, what);
    return acl__set_error(msg);
  };
  if (!a) return fail("null argument");
  if (n < 1 || n > acl_amd::kMaxNWide) return fail("n out of range [1, 512]");
  if (a->B < 0 || a->K < 1 || a->steps < 0 || a->step0 < 0)
    return fail("B, steps and step0 must be >= 0, K >= 1");
  if (!a->fseq || !a->fidx || !a->q || !a->vel || !a->P || !a->flush || !a->ts || !a->ctl_on ||
      !a->ring_u || !a->ring_ca || !a->posf || !a->dist || !a->t_conv || !a->t_avoid ||
      !a->n_assign || !a->workspace)
    return fail("required pointer is NULL");
  const acl_trial_params_t& tp = a->tp;
  const acl_episode_params_t& ep = tp.ep;
  if (ep.auction_every < 1 || ep.sample_every < 1 || ep.bufflen < 1 || !(ep.control_dt > 0.0) ||
      tp.tick_rate < 1 || tp.settle_steps < 0)
    return fail("auction_every, sample_every, bufflen, tick_rate must be >= 1, control_dt > 0, "
                "settle_steps >= 0");
  if (ep.auction_latency != 0) return fail("auction_latency must be 0 in trials");
  if (ep.assignment != ACL_ASSIGN_CBAA && ep.assignment != ACL_ASSIGN_CENTRAL)
    return fail("assignment must be ACL_ASSIGN_CBAA or ACL_ASSIGN_CENTRAL");
  return ACL_OK;
}

acl_amd::TrialDev trial_dev(const acl_trial_args_t* a, int n) {
  using namespace acl_amd;
  const TrLayout W = tr_layout(n, a->B);
  const WsLayout WS = ws_layout(n, a->B);
  unsigned char* ws = (unsigned char*)a->workspace;
  unsigned char* wc = ws + W.E.ctl;
  TrialDev D;
  D.n = n; D.B = a->B; D.K = a->K; D.step = 0; D.k = 0; D.F = 0;
  D.central = a->tp.ep.assignment == ACL_ASSIGN_CENTRAL;
  D.fseq = a->fseq; D.fidx = a->fidx; D.q = a->q; D.vel = a->vel; D.P = a->P;
  D.flush = a->flush; D.ts = a->ts; D.ctl_on = a->ctl_on; D.ring_u = a->ring_u;
  D.ring_ca = a->ring_ca; D.posf = a->posf; D.dist = a->dist; D.t_conv = a->t_conv;
  D.t_avoid = a->t_avoid; D.n_assign = a->n_assign;
  D.afidx = reinterpret_cast<int32_t*>(ws + W.afidx);
  D.due = ws + W.due;
  D.zstep = ws + W.zstep;
  D.Pnew = reinterpret_cast<const uint16_t*>(ws + W.E.Pnew);
  D.st = reinterpret_cast<const acl_swarm_status_t*>(ws + W.E.st);
  D.sRows = reinterpret_cast<const uint16_t*>(ws + W.E.solve + WS.rows);
  D.sValid = ws + W.E.solve + WS.vvalid;
  D.hst = reinterpret_cast<const int32_t*>(ws + W.E.hst);
  D.ctlPt = reinterpret_cast<uint16_t*>(wc + WS.pt);
  D.ctlMode = wc + WS.mode;
  D.ctlRows = reinterpret_cast<uint16_t*>(wc + WS.rows);
  D.cst = reinterpret_cast<acl_swarm_status_t*>(ws + W.E.cst);
  D.u = reinterpret_cast<const double*>(ws + W.E.u);
  D.us = reinterpret_cast<const double*>(ws + W.E.us);
  D.ca = ws + W.E.ca;
  D.ca_count = reinterpret_cast<unsigned*>(wc + WS.cacount);
  D.q_hist = a->q_hist; D.vel_hist = a->vel_hist; D.u_hist = a->u_hist; D.ca_hist = a->ca_hist;
  D.ctl_hist = a->ctl_hist; D.P_hist = a->P_hist; D.state_hist = a->state_hist;
  D.tp = a->tp;
  return D;
}

}  // namespace

extern "C" acl_status_t acl_trial_init(const acl_trial_args_t* a, int32_t n, void* stream) {
  using namespace acl_amd;
  const acl_status_t r = trial_check(a, n, "acl_trial_init");
  if (r != ACL_OK) return r;
  if (a->B == 0) return ACL_OK;
  const TrialDev D = trial_dev(a, n);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(D.ca_count, 0, kCaCounterBytes, s) != hipSuccess)
    return acl__set_error("hipMemsetAsync failed");
  hipLaunchKernelGGL(trial_init_kernel, dim3(a->B), dim3(kTrBlock), 0, s, D);
  if (hipGetLastError() != hipSuccess) return acl__set_error("trial_init_kernel launch failed");
  return ACL_OK;
}

extern "C" acl_status_t acl_trial_batch(const acl_formations_t* F, const acl_trial_args_t* a,
                                        void* stream) {
  using namespace acl_amd;
  if (!F) return acl__set_error("acl_trial_batch: null argument");
  const int n = F->n;
  const acl_status_t r0 = trial_check(a, n, "acl_trial_batch");
  if (r0 != ACL_OK) return r0;
  const int B = a->B;
  if (B == 0 || a->steps == 0) return ACL_OK;
  TrialDev D = trial_dev(a, n);
  D.F = F->n_formations;
  if (D.F < 1) return acl__set_error("acl_trial_batch: n_formations < 1");
  const TrLayout W = tr_layout(n, B);
  unsigned char* ws = (unsigned char*)a->workspace;
  unsigned char* wc = ws + W.E.ctl;
  const WsLayout WS = ws_layout(n, B);
  hipStream_t s = (hipStream_t)stream;

  // the batched auction: every swarm; those without an auction this step
  // carry formation -1 (BAD_INPUT: nothing of them is read)
  acl_solve_args_t sa = {};
  sa.B = B; sa.fidx = D.afidx; sa.q = a->q; sa.vel = a->vel; sa.P_in = a->P;
  sa.P_out = const_cast<uint16_t*>(D.Pnew);
  sa.P_rows = reinterpret_cast<const uint16_t*>(wc + WS.rows);
  sa.P_rows_on = wc + WS.mode;
  sa.status = const_cast<acl_swarm_status_t*>(D.st);
  sa.workspace = ws + W.E.solve;
  sa.cntrl = a->cntrl; sa.safety = a->safety; sa.early_exit = 1; sa.do_control = 0;
  sa.skip_margin = 1;
  acl_hungarian_args_t ha = {};
  ha.B = B; ha.fidx = D.afidx; ha.q = a->q; ha.P_last = a->P;
  ha.P_opt = const_cast<uint16_t*>(D.Pnew);
  ha.cost = reinterpret_cast<double*>(ws + W.E.hcost);
  ha.status = const_cast<int32_t*>(D.hst);
  // the control stage on the current formations and the hand-off region
  acl_control_args_t cs = {};
  cs.B = B; cs.fidx = a->fidx; cs.q = a->q; cs.vel = a->vel; cs.P = a->P;
  cs.u = const_cast<double*>(D.u);
  cs.u_safe = const_cast<double*>(D.us);
  cs.ca_flag = const_cast<uint8_t*>(D.ca);
  cs.status = D.cst;
  cs.workspace = wc; cs.cntrl = a->cntrl; cs.safety = a->safety;
  if (hipMemsetAsync(D.ca_count, 0, kCaCounterBytes, s) != hipSuccess)
    return acl__set_error("hipMemsetAsync failed");

  const acl_episode_params_t& ep = a->tp.ep;
  for (int k = 0; k < a->steps; ++k) {
    D.step = a->step0 + k;
    D.k = k;
    hipLaunchKernelGGL(trial_pre_kernel, dim3(B), dim3(64), 0, s, D);
    if (hipGetLastError() != hipSuccess) return acl__set_error("trial_pre_kernel launch failed");
    const acl_status_t r = D.central ? acl_hungarian_batch(F, &ha, stream)
                                     : acl_solve_batch(F, &sa, stream);
    if (r != ACL_OK) return r;
    hipLaunchKernelGGL(trial_adopt_kernel, dim3(B), dim3(256), 0, s, D);
    if (hipGetLastError() != hipSuccess) return acl__set_error("trial_adopt_kernel launch failed");
    const acl_status_t rc = run_control(F, &cs, s, CTL_MIXED);
    if (rc != ACL_OK) return rc;
    hipLaunchKernelGGL(trial_traj_kernel, dim3(B), dim3(kTrBlock), 0, s, D);
    if (hipGetLastError() != hipSuccess) return acl__set_error("trial_traj_kernel launch failed");
    if (D.step % ep.sample_every == 0) {
      hipLaunchKernelGGL(trial_tick_kernel, dim3(B), dim3(kTrBlock), 0, s, D);
      if (hipGetLastError() != hipSuccess) return acl__set_error("trial_tick_kernel launch failed");
    }
  }
  return ACL_OK;
}
