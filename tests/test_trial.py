"""CPU suite for batched Monte-Carlo trials (acl_trial_batch):
the supervisor restatement (oracle/trial_oracle.py) on scripted signals
against supervisor.py's rules, a whole CPU trial on swarm6_3d, and the trial
ABI (struct layout, defaults, argument errors) without a GPU."""
import ctypes as ct
import os
import subprocess

import numpy as np

import helpers as H
import trial_oracle as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tp(**kw):
    tp = T.default_params()
    tp["ep"] = dict(tp["ep"], bufflen=3)
    tp.update(hover_wait=0.1, formation_received_wait=0.04, converged_wait=0.04, **kw)
    return tp


def test_supervisor_scripted_cycle():
    """HOVERING -(HOVER_WAIT)-> WAITING -(assignment)-> FLYING -(wait, then a
    full window of small |u|)-> IN_FORMATION -(CONVERGED_WAIT)-> HOVERING ...
    -> COMPLETE, with supervisor.py's timer arithmetic: a state entered at a
    tick runs its first body at the next tick with timer_ticks = 0, and
    has_elapsed(s) is timer_ticks / 50 >= s."""
    n, K = 3, 2
    s = T.Supervisor(n, K, _tp())
    q = np.zeros((n, 3))
    zero, big = np.zeros(n), np.full(n, 5.0)
    no = np.zeros(n, bool)
    seq = []
    for tick in range(60):
        step = 2 * tick
        if s.state == T.WAITING and s.timer_ticks == 1:
            s.assignment_msg()
        speeds = big if tick < 20 else zero
        s.tick(step, speeds, no, q)
        seq.append(s.state)
        if s.done_step >= 0:
            break
    # hover_wait 0.1 s = 5 ticks: the 6th tick (timer 5) leaves HOVERING
    assert seq[:5] == [T.HOVERING] * 5 and seq[5] == T.WAITING
    assert s.formation == K - 1 and s.state == T.COMPLETE and s.done_step >= 0
    r = s.record()
    assert r["assignments"] == [1, 1] and all(t > 0 for t in r["time"])
    assert r["time_avoidance"] == [0.0, 0.0]


def test_supervisor_gridlock_and_release():
    """FLYING -> GRIDLOCK when a vehicle's CA flag is on for > 95% of a full
    window; has_left_gridlock needs a full window again (next_state clears the
    buffers); time_avoidance keeps the gridlock's duration."""
    n = 2
    s = T.Supervisor(n, 1, _tp(gridlock_timeout=100.0))
    s.state, s.formation, s.logging, s.timer_ticks = T.FLYING, 0, True, 10
    q = np.zeros((n, 3))
    on = np.array([True, False])
    big = np.full(n, 5.0)
    step = 0
    for _ in range(3):
        s.tick(step, big, on, q)
        step += 2
    assert s.state == T.GRIDLOCK and s.t_grid == 4
    for _ in range(2):          # the window refills: no decision yet
        s.tick(step, big, ~on & on, q)
        step += 2
        assert s.state == T.GRIDLOCK
    s.tick(step, big, ~on & on, q)
    assert s.state == T.FLYING
    assert s.time_avoidance[0] == (step - 4) * 0.01


def test_cpu_trial_swarm6_runs_to_an_end():
    pts, adj, gains, q0 = H.swarm6()
    forms = list(zip(pts, adj, gains))
    tp = _tp(settle_steps=10)
    tp["ep"] = dict(tp["ep"], auction_every=20, bufflen=10)
    q = q0.copy()
    q[:, 2] = 1.0
    t, qf, vf, states = T.run_trial(q, np.zeros_like(q), [0, 1, 2], forms, tp, 3000)
    assert t.done and t.sup.state in (T.COMPLETE, T.TERMINATE)
    assert np.isfinite(qf).all()
    assert t.counts["auctions"] > 0


# -- ABI ------------------------------------------------------------------

_LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "aclswarm_amd.h"
#define P(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f));
int main(void) {
  printf("params %zu status %zu args %zu\n", sizeof(acl_trial_params_t),
         sizeof(acl_trial_status_t), sizeof(acl_trial_args_t));
  P(acl_trial_params_t, tick_rate) P(acl_trial_params_t, settle_steps)
  P(acl_trial_params_t, hover_wait) P(acl_trial_params_t, alpha)
  P(acl_trial_status_t, next_auction) P(acl_trial_status_t, done_step)
  P(acl_trial_status_t, n_auctions) P(acl_trial_status_t, n_disagree)
  P(acl_trial_status_t, per_vehicle)
  P(acl_trial_args_t, fseq) P(acl_trial_args_t, n_assign) P(acl_trial_args_t, step0)
  P(acl_trial_args_t, steps) P(acl_trial_args_t, q_hist) P(acl_trial_args_t, state_hist)
  P(acl_trial_args_t, workspace) P(acl_trial_args_t, cntrl) P(acl_trial_args_t, safety)
  P(acl_trial_args_t, tp)
  return 0;
}
"""


def test_trial_struct_layout_matches_ctypes(tmp_path):
    from aclswarm_amd import _lib as L
    src = tmp_path / "layout.c"
    src.write_text(_LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I" + os.path.join(ROOT, "include"), str(src),
                           "-o", str(exe)])
    out = subprocess.check_output([str(exe)]).decode().split("\n")
    sizes = out[0].split()
    assert int(sizes[1]) == ct.sizeof(L.TrialParams)
    assert int(sizes[3]) == L.TRIAL_STATUS_DTYPE.itemsize == 80
    assert int(sizes[5]) == ct.sizeof(L.TrialArgs)
    cls = {"acl_trial_params_t": L.TrialParams, "acl_trial_args_t": L.TrialArgs}
    for line in out[1:]:
        if not line:
            continue
        name, off = line.split()
        Tn, f = name.split(".")
        if Tn == "acl_trial_status_t":
            assert L.TRIAL_STATUS_DTYPE.fields[f][1] == int(off), name
        else:
            assert getattr(cls[Tn], f).offset == int(off), name


def test_trial_defaults_and_argument_errors_without_gpu():
    from aclswarm_amd import _lib as L
    lib = L.lib()
    t = L.default_trial_params()
    assert (t.tick_rate, t.settle_steps) == (50, 150)
    assert (t.hover_wait, t.assignment_timeout, t.formation_received_wait, t.converged_wait,
            t.gridlock_timeout, t.trial_timeout, t.alpha) == (5.0, 20.0, 1.0, 1.0, 90.0, 600.0, 0.98)
    assert t.ep.auction_every == 120 and t.ep.assignment == 0
    oracle = T.default_params()
    for k in ("tick_rate", "settle_steps", "hover_wait", "gridlock_timeout", "trial_timeout"):
        assert oracle[k] == getattr(t, k)
    assert lib.acl_trial_workspace_bytes(100, 16) > lib.acl_episode_workspace_bytes(100, 16)
    a = L.TrialArgs()
    a.B, a.K, a.tp = 4, 2, t
    assert lib.acl_trial_init(ct.byref(a), 6, None) != 0
    assert b"required pointer" in lib.acl_last_error()
    a.K = 0
    assert lib.acl_trial_init(ct.byref(a), 6, None) != 0
    assert b"K >= 1" in lib.acl_last_error()
    for k in [f[0] for f in L.TrialArgs._fields_ if f[1] is ct.c_void_p]:
        setattr(a, k, 16)  # non-NULL placeholders: argument checks only
    a.K = 2
    a.tp.ep.auction_latency = 3
    assert lib.acl_trial_init(ct.byref(a), 6, None) != 0
    assert b"auction_latency" in lib.acl_last_error()
    a.tp.ep.auction_latency = 0
    a.tp.ep.assignment = 7
    assert lib.acl_trial_init(ct.byref(a), 6, None) != 0
    assert b"assignment" in lib.acl_last_error()
