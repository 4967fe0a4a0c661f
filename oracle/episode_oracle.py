"""CPU restatement of the closed-loop episode.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of
acl_episode_batch; never by the product path.

What it restates, in the order one lockstep control period applies it:
  * CoordinationROS::autoauctionCb (aclswarm/src/coordination_ros.cpp:322-359):
    every `auction_every` steps, a swarm whose last auction converged on an
    invalid assignment flushes and skips (:339-345); otherwise CBAA from the
    current q (pyoracle.solve, the restatement of auctioneer.cpp) and each
    vehicle's adoption of its own final table when it is valid
    (auctioneer.cpp:250-295; `adopt`, `SwarmState`);
    In the centralized comparison mode (acl_episode_params_t::assignment =
    ACL_ASSIGN_CENTRAL, coordination_ros.cpp:330-343) the auto-auction
    applies the operator's Hungarian assignment instead (`central_assign`:
    pyoracle.hungarian, the restatement of assignment.py:94-137, with last =
    the swarm's current P, operator.py:219-240);
  * DistCntrl::compute + Safety::cmdinCb + collisionAvoidance for every
    vehicle (pyoracle.control / saturate / collision_avoidance, i.e.
    distcntrl.cpp:46-102, safety.cpp:172-197,412-541);
  * Safety::makeSafeTraj (safety.cpp:330-408) with utils::rateLimit and
    utils::clamp (aclswarm/include/aclswarm/utils.h:213-264); the vehicle
    tracks its goal exactly (the outer loop / simulator are out of scope);
  * the supervisor's has_converged / has_gridlocked
    (aclswarm_sim/nodes/supervisor.py:297-337) at every `sample_every`-th
    step over a window of `bufflen` ticks (deque(maxlen=BUFFLEN), mean over
    the window as a sequential sum oldest -> newest, then / BUFFLEN).

Parity: pinned only through its parts -- the CBAA/control/safety restatement
is oracle/aclswarm_oracle.c; makeSafeTraj and the
supervisor predicates are restated here from the reference text and are
"parity unpinned" (no reference test or fixture covers them; the ROS nodes
do not build here).
"""
import math

import numpy as np

import pyoracle as O


def default_params():
    """acl_default_episode_params: coordination.launch:6,24-25,
    safety.cpp:45-46, trial.sh:96, supervisor.py:47,61-62,121."""
    return dict(control_dt=0.01, auction_every=120, sample_every=2, bufflen=50,
                auction_latency=0, max_accel_xy=0.5, max_accel_z=0.8,
                bounds_min=(-100.0, -100.0, 0.0), bounds_max=(100.0, 100.0, 30.0),
                orig_zero_vel_thr=1.0, avg_active_ca_thr=0.95, assignment=0)


def params_from_struct(e):
    return dict(control_dt=e.control_dt, auction_every=e.auction_every,
                sample_every=e.sample_every, bufflen=e.bufflen,
                auction_latency=e.auction_latency,
                max_accel_xy=e.max_accel_xy, max_accel_z=e.max_accel_z,
                bounds_min=tuple(e.bounds_min), bounds_max=tuple(e.bounds_max),
                orig_zero_vel_thr=e.orig_zero_vel_thr, avg_active_ca_thr=e.avg_active_ca_thr,
                assignment=int(getattr(e, "assignment", 0)))


def _rate_limit(dt, lo, hi, v0, v1):
    """utils::rateLimit (utils.h:254-264), elementwise."""
    upper = v0 + hi * dt
    lower = v0 + lo * dt
    v1 = np.where(v1 > upper, upper, v1)
    return np.where(v1 < lower, lower, v1)


def make_safe_traj(pos, vel, cmd, ep):
    """Safety::makeSafeTraj (safety.cpp:330-408) for arrays [..., 3] of goal
    positions, goal velocities and velocity goals. Returns (pos, vel)."""
    dt = ep["control_dt"]
    amax = np.array([ep["max_accel_xy"], ep["max_accel_xy"], ep["max_accel_z"]])
    bmin = np.array(ep["bounds_min"], dtype=np.float64)
    bmax = np.array(ep["bounds_max"], dtype=np.float64)
    pos = np.asarray(pos, np.float64)
    vel = np.asarray(vel, np.float64)
    c = _rate_limit(dt, -amax, amax, vel, np.asarray(cmd, np.float64))
    nxt = pos + c * dt
    lo = np.where(pos < bmin, pos, bmin)         # std::min(bounds_min, pos)
    hi = np.where(bmax < pos, pos, bmax)         # std::max(bounds_max, pos)
    below = nxt < lo
    above = ~below & (nxt > hi)
    clamped = below | above
    newpos = np.where(below, lo, np.where(above, hi, nxt))
    c = np.where(clamped, _rate_limit(dt, -amax, amax, vel, np.zeros_like(c)), c)
    return newpos, c


class Supervisor:
    """supervisor.py:297-337 for one swarm of n vehicles."""

    def __init__(self, n, ep):
        self.L = ep["bufflen"]
        self.ep = ep
        self.speed = []
        self.ca = []
        self.n_samples = 0
        self.converged = False
        self.gridlocked = False

    def tick(self, u, ca):
        """u [n][3] DistCntrl commands (voriggoal), ca [n] flags."""
        u = np.asarray(u, np.float64)
        sp = np.sqrt((u[:, 0] * u[:, 0] + u[:, 1] * u[:, 1]) + u[:, 2] * u[:, 2])
        self.speed.append(sp)
        self.ca.append(np.asarray(ca).astype(np.float64))
        self.speed = self.speed[-self.L:]
        self.ca = self.ca[-self.L:]
        self.n_samples += 1
        if self.n_samples < self.L:
            return None
        su = np.zeros_like(sp)
        sc = np.zeros_like(sp)
        for a, b in zip(self.speed, self.ca):   # oldest -> newest
            su = su + a
            sc = sc + b
        mu = su / float(self.L)
        mc = sc / float(self.L)
        self.converged = bool((mu < self.ep["orig_zero_vel_thr"]).all())
        self.gridlocked = bool((mc > self.ep["avg_active_ca_thr"]).any())
        return self.converged, self.gridlocked


def control_step(q, vel, p, adj, gains, P, g=None, s=None, tables=None):
    """DistCntrl::compute + cmdinCb + collisionAvoidance for every vehicle of
    one swarm. P: vehicle -> point (each vehicle's own point); tables: None
    (one assignment, inverse of P) or [n][n] per-vehicle inverse tables
    (row v: vehicle v's formation point -> vehicle). Returns u, u_safe, ca."""
    n = q.shape[0]
    if tables is None:
        Pt = inverse(P)
    u = np.zeros((n, 3))
    us = np.zeros((n, 3))
    ca = np.zeros(n, np.uint8)
    for v in range(n):
        Ptv = Pt if tables is None else np.asarray(tables[v], np.uint16)
        u[v] = O.control(v, q, vel[v], Ptv, adj, gains, p, g)
        c = O.saturate(u[v], s)
        us[v], mod = O.collision_avoidance(v, q, c, s)
        ca[v] = mod
    return u, us, ca


def inverse(P):
    P = np.asarray(P, np.int64)
    Pt = np.zeros(len(P), np.uint16)
    Pt[P] = np.arange(len(P), dtype=np.uint16)
    return Pt


def is_perm(w):
    w = np.asarray(w, np.int64)
    return bool(((w >= 0) & (w < len(w))).all()) and len(set(w.tolist())) == len(w)


class SwarmState:
    """One swarm's assignment state across auctions: P (each vehicle's own
    formation point) and tables (None while every vehicle holds one
    assignment, else [n][n] per-vehicle inverse tables: row v = vehicle v's
    own assignment as formation point -> vehicle)."""

    def __init__(self, P):
        self.P = np.array(P, np.uint16)
        self.tables = None

    def copy(self):
        c = SwarmState(self.P)
        c.tables = None if self.tables is None else self.tables.copy()
        return c

    def solve_args(self):
        """(P_in, P_rows) of the swarm's next auction: every vehicle starts
        from its own assignment (auctioneer.cpp:357,369,422-427) --
        acl_solve_args_t::P_rows while the vehicles hold different ones."""
        return self.P, self.tables


def adopt(state, flush, res):
    """autoauctionCb's flush rule + each vehicle's adoption
    (auctioneer.cpp:250-295) for one swarm after an auction result `res`
    (pyoracle.solve from state.solve_args()). Mutates `state`; returns (flush, event)
    with event one of 'skipped', 'adopted', 'invalid', 'disagree'.

    agree + valid: every vehicle adopts the one table. agree + invalid: every
    vehicle keeps its table and the swarm skips its next auto-auction
    (coordination_ros.cpp:339-345). Disagreement: each vehicle whose own final
    table is a permutation adopts it (its row of `who`), the others keep
    theirs; the swarm then flies per-vehicle tables until an agreed valid
    auction, and each vehicle starts its next auction (alignment and
    neighbours) from its own table, as the reference's vehicles do.

    A vehicle whose own table is invalid after a disagreeing auction keeps
    its old table and sets invalid_assignment_ (auctioneer.cpp:291): at the
    next auto-auction it flushes instead of starting (coordination_ros.cpp:
    339-345), so its neighbours wait on its START bid (bidIterComplete,
    auctioneer.cpp:419-439) and, through them, the whole (connected) swarm's
    auction completes nowhere until every vehicle restarts at the tick after
    (:355-358). The lockstep model: the swarm skips its next auto-auction,
    as after an agreed invalid result. Model limit: stale START bids the
    stalled auction leaves in the reference's queues are not modelled, and a
    formation graph with several components stalls only the flagged
    vehicle's component there (here the whole swarm)."""
    if flush:
        return 0, "skipped"
    fl = res["status"]["flags"]
    valid, agree = bool(fl & 0x01), bool(fl & 0x02)
    if agree and valid:
        state.P = res["P_out"].astype(np.uint16).copy()
        state.tables = None
        return 0, "adopted"
    if agree:
        return 1, "invalid"
    who = res["who"]
    n = len(state.P)
    vv = [is_perm(who[v]) for v in range(n)]
    if any(vv):
        cur = (np.tile(inverse(state.P), (n, 1)) if state.tables is None
               else state.tables.copy())
        P = state.P.copy()
        for v in range(n):
            if vv[v]:
                cur[v] = who[v]
                P[v] = int(np.nonzero(who[v] == v)[0][0])
        state.tables = cur.astype(np.uint16)
        state.P = P
    bad = bool(fl & 0x10)  # ACL_SWARM_BAD_INPUT
    return (0 if all(vv) or bad else 1), "disagree"


def central_assign(state, q, p):
    """ACL_ASSIGN_CENTRAL's auto-auction (coordination_ros.cpp:330-343): the
    operator's find_optimal_assignment(q, p, last) (operator.py:219-240,
    assignment.py:94-137; pyoracle.hungarian) with last = the swarm's current
    P becomes every vehicle's assignment (Auctioneer::setAssignment +
    newAssignmentCb): one table. A BAD_INPUT / NONFINITE problem (scipy
    would raise in the operator) leaves the swarm on its P. Mutates `state`;
    returns 'central' or 'invalid'."""
    P, _, _, st = O.hungarian(q, p, P_last=state.P)
    if st != 0:
        return "invalid"
    state.P = P.astype(np.uint16).copy()
    state.tables = None
    return "central"


AUCTIONEER_DT = 0.001  # coordination.launch:23: one bid processed per tick


def auction_latency_steps(n, adj, ep):
    """Control steps from an auto-auction's start to its completion
    (acl_episode_params_t::auction_latency): fixed, or the reference's timing
    ceil(2 n d_max auctioneer_dt / control_dt) -- one bid per 1 ms tick
    (auctioneer.cpp:139-160), every neighbour's bid in each of the 2n rounds
    (auctioneer.cpp:198-241), d_max the formation graph's largest degree."""
    L = int(ep.get("auction_latency", 0))
    if L >= 0:
        return L
    a = np.asarray(adj) != 0
    np.fill_diagonal(a, False)
    dmax = int(a.sum(axis=1).max()) if n else 0
    return int(math.ceil(2.0 * n * dmax * AUCTIONEER_DT / ep["control_dt"]))


class Auctions:
    """CoordinationROS::autoauctionCb and the auction's completion for one
    swarm, with auctions that take `latency` control steps (0: complete in
    their own step). An auto-auction that finds one pending restarts it
    (coordination_ros.cpp:355-358); the flush rule (:339-345) skips one."""

    def __init__(self, latency, flush=0, central=False):
        self.latency = 0 if central else latency
        self.flush = flush
        self.central = central
        self.pending = -1
        self.res = None
        self.counts = dict(skipped=0, auctions=0, adopted=0, invalid=0, disagree=0, restarted=0,
                           central=0)

    def auto(self, step, state, solve, central=None):
        """An auto-auction step; solve(P_in, P_rows) runs CBAA from the
        current q with the vehicles' own assignments (state.solve_args()).
        In the centralized mode central() applies the operator's assignment
        instead (`central_assign`). Mutates `state`."""
        if self.central:
            ev = central()
            self.counts[ev] += 1
            if ev == "central":
                self.counts["auctions"] += 1
            return state
        if self.flush:
            self.flush = 0
            self.counts["skipped"] += 1
            return state
        self.counts["auctions"] += 1
        if self.pending >= 0:
            self.counts["restarted"] += 1
        self.res = solve(*state.solve_args())
        if self.latency <= 0:
            self.pending = -1
            return self._complete(state)
        self.pending = step + self.latency
        return state

    def tick(self, step, state):
        """Any other step: a pending auction whose step has come completes."""
        if 0 <= self.pending <= step:
            self.pending = -1
            return self._complete(state)
        return state

    def _complete(self, state):
        self.flush, ev = adopt(state, 0, self.res)
        self.counts[ev] += 1
        return state


def run_episode(q, vel, P, p, adj, gains, steps, ep, step0=0, g=None, s=None):
    """The whole closed loop for one swarm on the CPU (small cases only)."""
    q = np.array(q, np.float64)
    vel = np.array(vel, np.float64)
    st = SwarmState(P)
    sup = Supervisor(q.shape[0], ep)
    auc = Auctions(auction_latency_steps(q.shape[0], adj, ep), central=ep.get("assignment", 0) == 1)
    conv_step = grid_step = -1
    qs = []
    for k in range(steps):
        step = step0 + k
        if step % ep["auction_every"] == 0:
            auc.auto(step, st, lambda P_in, rows: O.solve(q, vel, p, adj, gains, P_in, g, s,
                                                          P_rows=rows),
                     central=lambda: central_assign(st, q, p))
        else:
            auc.tick(step, st)
        u, us, ca = control_step(q, vel, p, adj, gains, st.P, g, s, st.tables)
        q, vel = make_safe_traj(q, vel, us, ep)
        if step % ep["sample_every"] == 0:
            r = sup.tick(u, ca)
            if r is not None:
                if r[0] and conv_step < 0:
                    conv_step = step
                if r[1] and grid_step < 0:
                    grid_step = step
        qs.append(q.copy())
    return dict(q=q, vel=vel, P=st.P, tables=st.tables, flush=auc.flush, counts=auc.counts, converged_step=conv_step,
                gridlock_step=grid_step, q_hist=np.array(qs))
