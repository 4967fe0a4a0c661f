"""CPU suite for closed-loop episodes: the episode
oracle's makeSafeTraj / supervisor / adoption rules against scalar
restatements written from the reference text, a whole CPU episode on
swarm6_3d, and the episode ABI (struct layout, workspace size, argument
errors) without a GPU."""
import ctypes as ct
import math
import os
import subprocess

import numpy as np
import pytest

import episode_oracle as E
import helpers as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# -- scalar restatements, line by line from the reference -------------------

def _rate_limit(dt, lo, hi, v0, v1):          # utils.h:254-264
    upper = v0 + hi * dt
    lower = v0 + lo * dt
    if v1 > upper:
        v1 = upper
    if v1 < lower:
        v1 = lower
    return v1


def _clamp(val, lower, upper):                # utils.h:213-227
    if val < lower:
        return lower, True
    if val > upper:
        return upper, True
    return val, False


def _make_safe_traj_scalar(pos, vel, cmd, ep):  # safety.cpp:330-408
    dt = ep["control_dt"]
    ax, az = ep["max_accel_xy"], ep["max_accel_z"]
    lim = (ax, ax, az)
    c = [_rate_limit(dt, -lim[a], lim[a], vel[a], cmd[a]) for a in range(3)]
    newpos, cl = [], []
    for a in range(3):
        nxt = pos[a] + c[a] * dt
        p, k = _clamp(nxt, min(ep["bounds_min"][a], pos[a]), max(ep["bounds_max"][a], pos[a]))
        newpos.append(p)
        cl.append(k)
    for a in range(3):
        if cl[a]:
            c[a] = 0.0
    for a in range(3):
        if cl[a]:
            c[a] = _rate_limit(dt, -lim[a], lim[a], vel[a], c[a])
    return newpos, c


def test_make_safe_traj_matches_scalar_restatement():
    ep = E.default_params()
    ep = dict(ep, bounds_min=(-5.0, -4.0, 0.5), bounds_max=(5.0, 4.0, 3.0))
    rng = np.random.RandomState(3)
    N = 4000
    pos = rng.uniform(-6, 6, (N, 3))
    pos[:, 2] = rng.uniform(0.0, 3.5, N)
    vel = rng.normal(0, 0.4, (N, 3))
    cmd = rng.normal(0, 0.6, (N, 3))
    # edge cases: exactly on the bound, outside the room moving in/out, zero
    pos[0] = (5.0, 4.0, 3.0); cmd[0] = (1.0, 1.0, 1.0)
    pos[1] = (7.0, -6.0, 0.2); cmd[1] = (-1.0, 1.0, -0.5)
    pos[2] = (7.0, -6.0, 0.2); cmd[2] = (1.0, -1.0, 0.5)
    vel[3] = 0.0; cmd[3] = 0.0
    p, v = E.make_safe_traj(pos, vel, cmd, ep)
    for i in range(N):
        ps, vs = _make_safe_traj_scalar(list(pos[i]), list(vel[i]), list(cmd[i]), ep)
        assert list(p[i]) == ps and list(v[i]) == vs, i
    # rate limit: |dv| <= a dt, bounds: never leaves a room it was inside
    dv = np.abs(v - vel)
    assert (dv[:, :2] <= 0.5 * 0.01 + 1e-15).all() and (dv[:, 2] <= 0.8 * 0.01 + 1e-15).all()
    inside = ((pos >= np.array(ep["bounds_min"])) & (pos <= np.array(ep["bounds_max"]))).all(1)
    pin = p[inside]
    assert ((pin >= np.array(ep["bounds_min"])) & (pin <= np.array(ep["bounds_max"]))).all()
    # a vehicle outside the room may only move back towards it
    assert p[1, 0] <= pos[1, 0] and p[1, 1] >= pos[1, 1] and p[1, 2] >= pos[1, 2]


def test_supervisor_window_rules():
    ep = dict(E.default_params(), bufflen=5)
    n = 3
    S = E.Supervisor(n, ep)
    small = np.full((n, 3), 0.1)
    big = np.zeros((n, 3)); big[1] = (6.0, 0.0, 0.0)
    for k in range(4):
        assert S.tick(small, np.zeros(n)) is None     # not enough data yet
    assert S.tick(small, np.zeros(n)) == (True, False)
    # one fast vehicle: window mean (4 sqrt(0.03) + 6) / 5 > 1 -> not converged
    assert S.tick(big, np.zeros(n)) == (False, False)
    # gridlock: a vehicle in collision avoidance > 95% of the window
    S2 = E.Supervisor(n, dict(ep, bufflen=20))
    ca = np.array([0, 1, 0])
    res = None
    for k in range(20):
        res = S2.tick(small, ca if k else np.zeros(n))  # 19 of 20 active = 0.95, not > 0.95
    assert res == (True, False)
    assert S2.tick(small, ca) == (True, True)        # 20 of 20


def test_adopt_rule():
    P = np.arange(4, dtype=np.uint16)
    newP = np.array([1, 0, 3, 2], np.uint16)
    who_new = np.tile(E.inverse(newP), (4, 1))
    ok = {"P_out": newP, "status": {"flags": 0x03}, "who": who_new}
    bad = {"P_out": newP, "status": {"flags": 0x02}, "who": who_new}
    st = E.SwarmState(P)
    assert E.adopt(st, 0, ok) == (0, "adopted") and (st.P == newP).all() and st.tables is None
    P_in, rows = st.solve_args()
    assert (P_in == newP).all() and rows is None  # the next auction: one shared P_in
    st = E.SwarmState(P)
    assert E.adopt(st, 0, bad) == (1, "invalid") and (st.P == P).all()
    assert E.adopt(st, 1, ok) == (0, "skipped") and (st.P == P).all()   # flushed: skipped
    # disagreement: vehicles 0 and 1 end on valid but different tables,
    # vehicles 2 and 3 on invalid ones (a task nobody holds)
    who = np.array([[1, 0, 3, 2], [0, 1, 2, 3], [1, 0, 4, 4], [4, 4, 4, 4]], np.uint16)
    dis = {"P_out": np.array([1, 1, 2, 3], np.uint16), "status": {"flags": 0x00}, "who": who}
    st = E.SwarmState(P)
    # vehicles 2 and 3 set invalid_assignment_ (auctioneer.cpp:291): the
    # swarm's next auto-auction stalls on them and is skipped (flush = 1)
    assert E.adopt(st, 0, dis) == (1, "disagree")
    assert st.P.tolist() == [1, 1, 2, 3]          # own points: 0 and 1 adopted, 2, 3 kept
    assert st.tables[0].tolist() == [1, 0, 3, 2] and st.tables[1].tolist() == [0, 1, 2, 3]
    assert st.tables[2].tolist() == [0, 1, 2, 3] and st.tables[3].tolist() == [0, 1, 2, 3]
    P_in, rows = st.solve_args()                  # the next auction: each vehicle's own
    assert P_in.tolist() == [1, 1, 2, 3] and rows is st.tables
    for v in range(4):
        assert rows[v][P_in[v]] == v              # acl_solve_args_t::P_rows' contract
    # a second disagreement: the invalid vehicle keeps its own previous row
    who2 = np.array([[4, 4, 4, 4], [2, 3, 0, 1], [3, 2, 1, 0], [0, 1, 2, 3]], np.uint16)
    assert E.adopt(st, 0, {"P_out": None, "status": {"flags": 0x00}, "who": who2}) == (1, "disagree")
    assert st.tables[0].tolist() == [1, 0, 3, 2] and st.P[0] == 1
    assert st.tables[1].tolist() == [2, 3, 0, 1] and st.P[1] == 3
    # a disagreement with every table valid sets no flush
    who3 = np.stack([E.inverse(newP), E.inverse(P), E.inverse(P), E.inverse(newP)])
    assert E.adopt(st, 0, {"P_out": None, "status": {"flags": 0x00}, "who": who3}) == (0, "disagree")
    # agreement clears the per-vehicle state
    assert E.adopt(st, 0, ok) == (0, "adopted") and st.tables is None


def test_per_vehicle_control_uses_each_table():
    """control_step with per-vehicle tables equals control_step with each
    vehicle's own assignment, vehicle by vehicle."""
    rng = np.random.RandomState(2)
    pts, adj, gains, q0 = H.swarm6()
    n = 6
    q = q0 + rng.normal(0, 0.3, q0.shape)
    vel = rng.normal(0, 0.1, q.shape)
    Ps = [H.random_perm(rng, n) for _ in range(n)]
    tables = np.stack([E.inverse(P) for P in Ps])
    own = np.array([Ps[v][v] for v in range(n)], np.uint16)
    u, us, ca = E.control_step(q, vel, pts[0], adj[0], gains[0], own, tables=tables)
    for v in range(n):
        uv, usv, cav = E.control_step(q, vel, pts[0], adj[0], gains[0], Ps[v])
        np.testing.assert_array_equal(u[v], uv[v])
        np.testing.assert_array_equal(us[v], usv[v])


def test_cpu_episode_swarm6_flies_towards_formation():
    pts, adj, gains, q0 = H.swarm6()
    ep = dict(E.default_params(), auction_every=60)
    n = 6
    r = E.run_episode(q0, np.zeros((n, 3)), np.arange(n), pts[0], adj[0], gains[0], 130, ep)
    assert r["counts"]["adopted"] == 3                # auctions at steps 0, 60, 120
    assert sorted(r["P"].tolist()) == list(range(n))
    assert np.isfinite(r["q_hist"]).all()
    step = np.abs(np.diff(r["q_hist"], axis=0))
    assert (step[:, :, :2] <= 0.5 * 0.01 * 1.0000001).all()  # |v| <= max_vel_xy per axis


# -- ABI ------------------------------------------------------------------

_LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "aclswarm_amd.h"
#define P(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f));
int main(void) {
  printf("params %zu status %zu args %zu\n", sizeof(acl_episode_params_t),
         sizeof(acl_episode_status_t), sizeof(acl_episode_args_t));
  P(acl_episode_params_t, max_accel_xy) P(acl_episode_params_t, bounds_max)
  P(acl_episode_params_t, avg_active_ca_thr) P(acl_episode_params_t, auction_latency)
  P(acl_episode_status_t, n_auctions) P(acl_episode_status_t, n_ca_steps)
  P(acl_episode_status_t, pending_step) P(acl_episode_status_t, n_restarted)
  P(acl_episode_args_t, step0) P(acl_episode_args_t, vel_hist) P(acl_episode_args_t, workspace)
  P(acl_episode_args_t, cntrl) P(acl_episode_args_t, safety) P(acl_episode_args_t, ep)
  return 0;
}
"""


def test_episode_struct_layout_matches_ctypes(tmp_path):
    from aclswarm_amd import _lib as L
    src = tmp_path / "layout.c"
    src.write_text(_LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I" + os.path.join(ROOT, "include"), str(src),
                           "-o", str(exe)])
    out = subprocess.check_output([str(exe)]).decode().split("\n")
    sizes = out[0].split()
    assert int(sizes[1]) == ct.sizeof(L.EpisodeParams)
    assert int(sizes[3]) == L.EPISODE_STATUS_DTYPE.itemsize
    assert int(sizes[5]) == ct.sizeof(L.EpisodeArgs)
    cls = {"acl_episode_params_t": L.EpisodeParams, "acl_episode_args_t": L.EpisodeArgs}
    for line in out[1:]:
        if not line:
            continue
        name, off = line.split()
        T, f = name.split(".")
        if T == "acl_episode_status_t":
            assert L.EPISODE_STATUS_DTYPE.fields[f][1] == int(off), name
        else:
            assert getattr(cls[T], f).offset == int(off), name


def test_episode_defaults_and_argument_errors_without_gpu():
    from aclswarm_amd import _lib as L
    lib = L.lib()
    e = L.default_episode_params()
    assert (e.control_dt, e.auction_every, e.sample_every, e.bufflen) == (0.01, 120, 2, 50)
    assert (e.max_accel_xy, e.max_accel_z) == (0.5, 0.8)
    assert tuple(e.bounds_min) == (-100.0, -100.0, 0.0) and tuple(e.bounds_max) == (100.0, 100.0, 30.0)
    assert (e.orig_zero_vel_thr, e.avg_active_ca_thr) == (1.0, 0.95)
    d = E.default_params()
    assert E.params_from_struct(e) == d
    assert lib.acl_episode_workspace_bytes(100, 1024) > lib.acl_solve_workspace_bytes(100, 1024)
    assert lib.acl_episode_workspace_bytes(0, 4) == 0
    F = L.Formations()
    F.n = 6
    a = L.EpisodeArgs()
    a.B = 4
    a.steps = 1
    a.ep = e
    assert lib.acl_episode_batch(ct.byref(F), ct.byref(a), None) != 0   # NULL pointers
    assert b"NULL" in lib.acl_last_error()
    a.steps = -1
    assert lib.acl_episode_batch(ct.byref(F), ct.byref(a), None) != 0
    a.steps = 0
    assert lib.acl_episode_batch(ct.byref(F), ct.byref(a), None) == 0   # nothing to do
    F.n = 600
    a.steps = 1
    assert lib.acl_episode_batch(ct.byref(F), ct.byref(a), None) != 0
    assert math.isfinite(e.control_dt)


def test_formation_generator_argument_errors_without_gpu():
    from aclswarm_amd import _lib as L
    lib = L.lib()
    z = None
    assert lib.acl_generate_formation_groups(4, 4, z, 0, 1.0, 1.0, 1.0, 2.0, 0, z, z, z, z, z) != 0
    assert b"n >= 5" in lib.acl_last_error()
    assert lib.acl_generate_formation_groups(4, 600, z, 1, 1.0, 1.0, 1.0, 2.0, 0, z, z, z, z, z) != 0
    assert lib.acl_generate_formation_groups(0, 20, z, 1, 1.0, 1.0, 1.0, 2.0, 0, z, z, z, z, z) == 0
    assert lib.acl_generate_formation_groups(2, 20, z, 1, 1.0, 1.0, 1.0, 2.0, 0, z, z, z, z, z) != 0


def test_auction_latency_model():
    """acl_episode_params_t::auction_latency on the CPU: the reference timing
    ceil(2 n d_max 1 ms / control_dt), and the autoauctionCb state machine --
    an auction completes after its latency, one still pending at the next
    auto-auction is restarted (coordination_ros.cpp:355-358)."""
    pts, adj, gains, q0 = H.swarm6()
    ep = dict(E.default_params(), auction_latency=-1)
    n = 6
    for A in adj:
        d = int(((np.asarray(A) != 0) & ~np.eye(n, dtype=bool)).sum(axis=1).max())
        assert E.auction_latency_steps(n, A, ep) == math.ceil(2.0 * n * d * 0.001 / 0.01)
    a = np.ones((100, 100), np.uint8) - np.eye(100, dtype=np.uint8)
    a[0, 1:51] = a[1:51, 0] = 0
    assert E.auction_latency_steps(100, a, ep) == 1980  # 2 * 100 * 99 ms / 10 ms
    assert E.auction_latency_steps(n, adj[0], dict(ep, auction_latency=7)) == 7
    # latency longer than the auto-auction period: every auction restarts
    ep2 = dict(E.default_params(), auction_every=10, auction_latency=25)
    P0 = np.array([1, 0, 2, 3, 5, 4])
    r = E.run_episode(q0, np.zeros((n, 3)), P0, pts[0], adj[0], gains[0], 60, ep2)
    assert r["counts"]["auctions"] == 6 and r["counts"]["restarted"] == 5
    assert r["counts"]["adopted"] == 0 and (r["P"] == P0).all()
    # shorter: every auction completes `latency` steps after it started
    ep3 = dict(ep2, auction_latency=4)
    r = E.run_episode(q0, np.zeros((n, 3)), P0, pts[0], adj[0], gains[0], 60, ep3)
    assert r["counts"]["restarted"] == 0 and r["counts"]["adopted"] == 6
