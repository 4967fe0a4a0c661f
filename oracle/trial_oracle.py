"""CPU restatement of the batched Monte-Carlo trial (acl_trial_batch; SURVEY
§8f, the widening of row f1): aclswarm_sim's supervisor state machine over
the closed loop of episode_oracle.

TEST INFRASTRUCTURE ONLY: imported by tests/ (the checker of
acl_trial_batch) and the trial bench's cpu_baseline leg; never by the product
path.

What it restates, per control step s of one swarm, in the order
acl_trial_batch applies it:
  * `TrialSwarm.pre`: a formation requested by the last supervisor tick is
    committed -- CoordinationROS::spin (aclswarm/src/coordination_ros.cpp:
    95-153): the controllers stop after one zero command (sendZeroControl),
    Auctioneer::setFormation resets the assignment to identity
    (auctioneer.cpp:42-62; invalid_assignment_, the flush flag, is not
    cleared), the first auto-auction is due form_settle_time later and then
    every autoauction_dt (autoauctionCb :322-359, with the flush rule
    :339-345);
  * `TrialSwarm.adopt`: the auction's adoption per vehicle (episode_oracle's
    rules, auctioneer.cpp:250-295) or the operator's Hungarian in the
    centralized mode (coordination_ros.cpp:330-343); a vehicle's controller
    starts with its first assignment (newAssignmentCb :284-303); vehicle 0's
    assignment message (a new table or the formation's first,
    shouldUseAssignment auctioneer.cpp:310-321 / centralAssignmentCb
    coordination_ros.cpp:271-280) reaches the supervisor (supervisor.py:
    147-150);
  * `TrialSwarm.control` / `traj`: DistCntrl + Safety of the running
    controllers and makeSafeTraj of their safe commands (episode_oracle),
    makeSafeTraj of the zero command at a commit, the last goal held by
    stopped controllers (Safety::controlCb, safety.cpp:268-290);
  * `Supervisor.tick` (every sample_every steps): supervisor.py's tick()
    (:160-236) line by line -- timer, states, has_converged /
    has_gridlocked / has_left_gridlock on their own deques (:297-348),
    next_state's buffer reset and gridlock timing (:238-265),
    start_logging / stop_logging (:376-402), log_signals (:452-487), the
    watchdog (:229-232). Time is the step clock: now = s * control_dt.

Model limits (as acl_trial_batch, include/aclswarm_amd.h): the trial starts
in HOVERING in the air; a formation commits at the step after the tick that
requested it; the zero command's collision-avoidance flag is 0; the
operator's central assignment is computed at the auto-auction itself.

Parity: the supervisor is restated from the reference text and is "parity
unpinned" (no reference test or fixture covers supervisor.py; its ROS node
does not run here); the CBAA / control / safety steps are pinned as
episode_oracle's.
"""
import numpy as np

import episode_oracle as E
import pyoracle as O

HOVERING, WAITING, FLYING, IN_FORMATION, GRIDLOCK, COMPLETE, TERMINATE = 3, 4, 5, 6, 7, 8, 9


def default_params():
    """acl_default_trial_params: supervisor.py:47-62,88,121; coordination.launch:5."""
    return dict(ep=E.default_params(), tick_rate=50, settle_steps=150, hover_wait=5.0,
                assignment_timeout=20.0, formation_received_wait=1.0, converged_wait=1.0,
                gridlock_timeout=90.0, trial_timeout=600.0, alpha=0.98)


def params_from_struct(t):
    return dict(ep=E.params_from_struct(t.ep), tick_rate=t.tick_rate,
                settle_steps=t.settle_steps, hover_wait=t.hover_wait,
                assignment_timeout=t.assignment_timeout,
                formation_received_wait=t.formation_received_wait,
                converged_wait=t.converged_wait, gridlock_timeout=t.gridlock_timeout,
                trial_timeout=t.trial_timeout, alpha=t.alpha)


class Supervisor:
    """supervisor.py's Supervisor for one swarm of n vehicles flying K
    formations (the trial model of acl_trial_batch)."""

    def __init__(self, n, K, tp):
        self.n, self.K, self.tp = n, K, tp
        self.L = tp["ep"]["bufflen"]
        self.dt = tp["ep"]["control_dt"]
        self.state = HOVERING
        self.last_state = 0           # None
        self.timer_ticks = -1
        self.formation = -1           # curr_formation_idx
        self.received = False         # received_assignment
        self.logging = False          # is_logging
        self.commit = False           # the operator sent a formation (acl_trial_batch)
        self.buffers = {}
        self.ticks = 0
        self.done_step = -1
        self.t_start = 0
        self.t_grid = 0
        self.log = {}
        self.time = [0.0] * K         # log['time'] per formation (seconds)
        self.time_avoidance = [0.0] * K
        self.assignments = [0] * K

    # -- predicates (supervisor.py:279-348)
    def has_elapsed(self, secs):
        return self.timer_ticks / self.tp["tick_rate"] >= secs

    def _window(self, key, sample):
        buf = self.buffers.setdefault(key, [])
        buf.append(np.asarray(sample, np.float64))
        del buf[:-self.L]             # deque(maxlen=BUFFLEN)
        if len(buf) < self.L:
            return None
        s = np.zeros(self.n)
        for a in buf:                 # oldest -> newest
            s = s + a
        return s / float(self.L)

    def has_converged(self, speeds):
        m = self._window("converged_orig_vel", speeds)
        return False if m is None else bool((m < self.tp["ep"]["orig_zero_vel_thr"]).all())

    def has_gridlocked(self, cas):
        m = self._window("gridlocked_active_ca", np.asarray(cas, np.float64))
        return False if m is None else bool((m > self.tp["ep"]["avg_active_ca_thr"]).any())

    def has_left_gridlock(self, cas):
        g = self.has_gridlocked(cas)
        if len(self.buffers["gridlocked_active_ca"]) < self.L:
            return False
        return not g

    # -- transitions and logging (supervisor.py:238-265,376-402)
    def next_state(self, state, step, reset=True):
        self.last_state = self.state
        self.state = state
        self.timer_ticks = -1
        if reset:
            self.buffers = {}
        if self.state == GRIDLOCK:
            self.t_grid = step        # log['time_avoidance'][-1] = now
        if self.last_state == GRIDLOCK:
            self.time_avoidance[self.formation] = (step - self.t_grid) * self.dt

    def start_logging(self, step):
        if self.logging:
            return
        self.assignments[self.formation] = 1
        self.t_start = step
        self.time_avoidance[self.formation] = 0.0
        self.logging = True

    def stop_logging(self, step):
        if not self.logging:
            return
        self.logging = False
        self.time[self.formation] = (step - self.t_start) * self.dt

    def assignment_msg(self):
        """assignmentCb (supervisor.py:147-150)."""
        self.received = True
        if self.logging:
            self.assignments[self.formation] += 1

    def log_signals(self, q):
        x = np.asarray(q)[:, 0].copy()
        y = np.asarray(q)[:, 1].copy()
        if "position_x" not in self.log:
            self.log["position_x"] = x
        if "position_y" not in self.log:
            self.log["position_y"] = y
        if "dist" not in self.log:
            self.log["dist"] = np.zeros_like(x)
        a = self.tp["alpha"]
        lastx = self.log["position_x"]
        self.log["position_x"] = a * lastx + (1 - a) * x
        dx = np.abs(self.log["position_x"] - lastx)
        lasty = self.log["position_y"]
        self.log["position_y"] = a * lasty + (1 - a) * y
        dy = np.abs(self.log["position_y"] - lasty)
        self.log["dist"] = self.log["dist"] + np.sqrt(dx * dx + dy * dy)

    def tick(self, step, speeds, cas, q):
        """One tick at global step `step` (after the step's trajectories):
        speeds [n] |voriggoal|, cas [n] collision_avoidance_active, q [n][3]."""
        if self.done_step >= 0:
            return
        tp = self.tp
        self.timer_ticks += 1
        finished = False
        if self.state == HOVERING:
            if self.has_elapsed(tp["hover_wait"]):
                if self.formation == self.K - 1:        # has_cycled_through_formations
                    self.next_state(COMPLETE, step)
                else:                                   # next_formation
                    self.formation += 1
                    self.received = False
                    self.commit = True
                    self.next_state(WAITING, step)
        elif self.state == WAITING:
            if self.received:
                self.start_logging(step)
                self.next_state(FLYING, step)
            elif self.has_elapsed(tp["assignment_timeout"]):
                self.next_state(TERMINATE, step)
        elif self.state == FLYING:
            if self.has_elapsed(tp["formation_received_wait"]):
                if self.has_converged(speeds):
                    self.next_state(IN_FORMATION, step, reset=False)
                elif self.has_gridlocked(cas):
                    self.next_state(GRIDLOCK, step)
        elif self.state == IN_FORMATION:
            if self.has_elapsed(tp["converged_wait"]):
                self.stop_logging(step)
                self.next_state(HOVERING, step)
            elif not self.has_converged(speeds):
                self.next_state(FLYING, step)
        elif self.state == GRIDLOCK:
            if self.has_left_gridlock(cas):
                self.next_state(FLYING, step)
            elif self.has_elapsed(tp["gridlock_timeout"]):
                self.next_state(TERMINATE, step)
        else:                                           # COMPLETE / TERMINATE
            finished = True
        if self.logging:
            self.log_signals(q)
        if finished:
            self.done_step = step
        elif self.ticks / tp["tick_rate"] > tp["trial_timeout"]:
            self.next_state(TERMINATE, step)             # the watchdog
        self.ticks += 1

    def record(self):
        """The per-trial record (complete(), supervisor.py:404-415)."""
        d = self.log.get("dist", np.zeros(self.n))
        return dict(dist=d, time=list(self.time), time_avoidance=list(self.time_avoidance),
                    assignments=list(self.assignments), state=self.state,
                    last_state=self.last_state, done_step=self.done_step)


class TrialSwarm:
    """One swarm's trial: the coordination state (assignment, per-vehicle
    tables, controllers running, flush flag, auction countdown) and its
    supervisor. forms: list of (p, adj, gains) indexed by fseq."""

    def __init__(self, n, fseq, forms, tp):
        self.n = n
        self.fseq = list(fseq)
        self.forms = forms
        self.tp = tp
        self.central = tp["ep"].get("assignment", 0) == 1
        self.sup = Supervisor(n, len(self.fseq), tp)
        self.state = E.SwarmState(np.arange(n, dtype=np.uint16))
        self.ctl_on = np.zeros(n, bool)
        self.flush = 0
        self.next_auction = 0
        self.fidx = self.fseq[0]
        self.zs = False
        self.counts = dict(auctions=0, invalid=0, skipped=0, disagree=0)

    @property
    def done(self):
        return self.sup.done_step >= 0

    def pre(self):
        """The commit and the auto-auction schedule; True when an auction
        runs this step."""
        self.zs = False
        if self.done:
            return False
        now = False
        if self.sup.commit:
            self.fidx = self.fseq[self.sup.formation]
            self.state = E.SwarmState(np.arange(self.n, dtype=np.uint16))
            self.ctl_on[:] = False
            self.zs = True
            self.sup.commit = False
            self.next_auction = self.tp["settle_steps"]
            now = self.next_auction <= 0
            if now:
                self.next_auction = self.tp["ep"]["auction_every"]
        elif self.next_auction > 0:
            self.next_auction -= 1
            if self.next_auction == 0:
                now = True
                self.next_auction = self.tp["ep"]["auction_every"]
        if not now:
            return False
        if not self.central and self.flush:
            self.flush = 0
            self.counts["skipped"] += 1
            return False
        return True

    def _table0(self):
        """vehicle 0's table, formation point -> vehicle"""
        if self.state.tables is not None:
            return self.state.tables[0].copy()
        return E.inverse(self.state.P)

    def adopt(self, q, vel):
        """The due auction from (q, vel): CBAA (pyoracle.solve from each
        vehicle's own assignment) or the operator's Hungarian; adoption,
        controller starts and vehicle 0's message."""
        p, adj, G = self.forms[self.fidx]
        n = self.n
        old0 = self._table0()
        first0 = not self.ctl_on[0]
        v0 = False
        new0 = None
        if self.central:
            P, _, _, st = O.hungarian(q, p, P_last=self.state.P)
            if st != 0:
                self.counts["invalid"] += 1
                return
            self.counts["auctions"] += 1
            self.state.P = P.astype(np.uint16).copy()
            self.state.tables = None
            self.ctl_on[:] = True
            v0, new0 = True, E.inverse(self.state.P)
        else:
            self.counts["auctions"] += 1
            P_in, rows = self.state.solve_args()
            res = O.solve(q, vel, p, adj, G, P_in, P_rows=rows)
            fl = int(res["status"]["flags"])
            valid, agree, bad = bool(fl & 0x01), bool(fl & 0x02), bool(fl & 0x10)
            if agree and valid:
                self.state.P = res["P_out"].astype(np.uint16).copy()
                self.state.tables = None
                self.ctl_on[:] = True
                v0, new0 = True, E.inverse(self.state.P)
            elif agree:
                self.flush = 1
                self.counts["invalid"] += 1
            else:
                self.counts["disagree"] += 1
                who = res["who"]
                vv = [E.is_perm(who[v]) for v in range(n)]
                n_inv = n - sum(vv)
                if n_inv < n and not bad:
                    cur = (np.tile(E.inverse(self.state.P), (n, 1)) if self.state.tables is None
                           else self.state.tables.copy())
                    P = self.state.P.copy()
                    for v in range(n):
                        if vv[v]:
                            cur[v] = who[v]
                            P[v] = int(np.nonzero(who[v] == v)[0][0])
                            self.ctl_on[v] = True
                    self.state.tables = cur.astype(np.uint16)
                    self.state.P = P
                    if vv[0]:
                        v0, new0 = True, np.asarray(who[0], np.uint16)
                if n_inv > 0 and not bad:
                    self.flush = 1
        if v0 and (first0 or (old0 != new0).any()):
            self.sup.assignment_msg()

    def control(self, q, vel):
        p, adj, G = self.forms[self.fidx]
        return E.control_step(q, vel, p, adj, G, self.state.P, tables=self.state.tables)

    def traj(self, q, vel, us):
        """makeSafeTraj of the running controllers' commands, the zero
        command at a commit, the last goal otherwise."""
        qn = np.array(q, np.float64)
        vn = np.array(vel, np.float64)
        if self.done:
            return qn, vn
        on = self.ctl_on
        if on.any():
            a, b = E.make_safe_traj(qn[on], vn[on], np.asarray(us)[on], self.tp["ep"])
            qn[on], vn[on] = a, b
        if self.zs:
            off = ~on
            a, b = E.make_safe_traj(qn[off], vn[off], np.zeros((int(off.sum()), 3)), self.tp["ep"])
            qn[off], vn[off] = a, b
        return qn, vn

    def samples(self, u, ca):
        """The tick's |voriggoal| and CA flags: running controllers' own, 0
        for stopped ones."""
        u = np.asarray(u, np.float64)
        sp = np.sqrt((u[:, 0] * u[:, 0] + u[:, 1] * u[:, 1]) + u[:, 2] * u[:, 2])
        return np.where(self.ctl_on, sp, 0.0), np.where(self.ctl_on, np.asarray(ca) != 0, False)

    def step(self, s, q, vel):
        """One free-running step; returns (q, vel, u, ca) (u, ca masked to
        the running controllers)."""
        if self.pre():
            self.adopt(q, vel)
        u, us, ca = self.control(q, vel)
        qn, vn = self.traj(q, vel, us)
        um = np.where(self.ctl_on[:, None], u, 0.0)
        cam = np.where(self.ctl_on, ca, 0).astype(np.uint8)
        if s % self.tp["ep"]["sample_every"] == 0:
            sp, cs = self.samples(u, ca)
            self.sup.tick(s, sp, cs, qn)
        return qn, vn, um, cam


def run_trial(q, vel, fseq, forms, tp, steps, step0=0):
    """A whole trial of one swarm on the CPU (small cases only)."""
    t = TrialSwarm(q.shape[0], fseq, forms, tp)
    q = np.array(q, np.float64)
    vel = np.array(vel, np.float64)
    states = []
    for k in range(steps):
        q, vel, _, _ = t.step(step0 + k, q, vel)
        states.append(t.sup.state)
        if t.done:
            break
    return t, q, vel, states
