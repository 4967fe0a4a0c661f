"""GPU parity of batched Monte-Carlo trials (acl_trial_batch: supervisor.py
over the closed loop) against oracle/trial_oracle.py.

Teacher-forced: every recorded step of the GPU trial is re-derived on the CPU
from the GPU's own state before that step -- the formation commit and the
auction schedule, the auction (CBAA from each vehicle's own table, or the
operator's Hungarian) and each vehicle's adoption and controller start
(assignments and running controllers bit-exact), DistCntrl + Safety of the
running controllers (u within 1e-5 relative, CA flags exact), makeSafeTraj
(state within 1e-9), and the supervisor's tick from the GPU's recorded
commands, flags and positions (its state after every step exact). Then the
per-trial records -- the CSV row of complete() (supervisor.py:404-415): the
smoothed planar distance per vehicle, time to converge, gridlock time and
assignments per formation -- and the counters, bit for bit.
"""
import numpy as np
import pytest

import helpers as H
import trial_oracle as T

pytestmark = pytest.mark.gpu

U_RTOL = 1e-5
Q_ATOL = 1e-9

# short supervisor timings so that the CPU restatement stays fast: the state
# machine is the reference's, the clocks are scaled down
FAST = dict(settle_steps=10, hover_wait=0.2, formation_received_wait=0.1, converged_wait=0.2,
            gridlock_timeout=2.0, trial_timeout=60.0, assignment_timeout=2.0)
FAST_EP = dict(auction_every=20, bufflen=10)


def _swarm6_case(B=4, seed=3, central=False, **tp):
    pts, adj, gains, q0 = H.swarm6()
    rng = np.random.RandomState(seed)
    q = np.stack([q0 + rng.normal(0, 0.4, q0.shape) for _ in range(B)])
    q[..., 2] = 1.0
    fseq = np.stack([np.roll(np.arange(3), b) for b in range(B)]).astype(np.int32)
    return dict(pts=pts, adj=adj, gains=gains, q=q, vel=np.zeros_like(q), fseq=fseq,
                tp=dict(FAST, **tp), ep=dict(FAST_EP, assignment=1 if central else 0))


def _chain_case(n=10, B=3, seed=21):
    """Chain formations whose first auctions end with vehicles on different
    tables: some controllers start before others (per-vehicle
    first_assignment_), the flush rule fires."""
    import test_gpu_episode as GE
    c = GE._chain_case(n, 2 * B, seed)
    # swarm b starts on formation b (its start disagrees there), then B + b
    fseq = np.stack([np.arange(B), B + np.arange(B)], axis=1).astype(np.int32)
    return dict(pts=c["pts"], adj=c["adj"], gains=c["gains"], q=c["q"][:B], vel=c["vel"][:B],
                fseq=fseq, tp=dict(FAST, trial_timeout=8.0), ep=dict(FAST_EP))


def _run(case, dev, steps, chunks=None):
    import torch
    from aclswarm_amd import _lib as L
    from aclswarm_amd import engine
    Tb = engine.FormationTable.from_host(case["pts"], case["adj"], case["gains"], device=dev)
    tp = L.default_trial_params()
    for k, v in case["tp"].items():
        setattr(tp, k, v)
    for k, v in case["ep"].items():
        setattr(tp.ep, k, v)
    tr = engine.Trial(Tb, torch.from_numpy(case["fseq"]).to(dev),
                      torch.from_numpy(np.ascontiguousarray(case["q"])).to(dev),
                      torch.from_numpy(np.ascontiguousarray(case["vel"])).to(dev), params=tp)
    hs = []
    for c in (chunks or [steps]):
        hs.append(tr.run(c, history=True))
    torch.cuda.synchronize()
    h = {k: np.concatenate([x[k].cpu().numpy() for x in hs]) for k in hs[0]}
    h["P"] = h["P"].view(np.uint16)
    return tr, h, T.params_from_struct(tp)


def _teacher_forced(case, tr, h, tp, steps):
    B, n = case["q"].shape[:2]
    forms = list(zip(case["pts"], case["adj"], case["gains"]))
    st = tr.status()
    rec = tr.records()
    finals = []
    for b in range(B):
        t = T.TrialSwarm(n, case["fseq"][b], forms, tp)
        qprev, vprev = case["q"][b], case["vel"][b]
        for k in range(steps):
            if t.pre():
                t.adopt(qprev, vprev)
            assert (h["P"][k, b] == t.state.P).all(), (b, k)
            on = t.ctl_on & (not t.done)
            assert (h["ctl"][k, b] == on).all(), (b, k)
            u, us, ca = t.control(qprev, vprev)
            if on.any():
                np.testing.assert_allclose(h["u"][k, b][on], u[on], rtol=U_RTOL, atol=U_RTOL)
                assert (h["ca"][k, b][on] == ca[on]).all(), (b, k)
            assert (h["u"][k, b][~on] == 0).all() and (h["ca"][k, b][~on] == 0).all()
            qn, vn = t.traj(qprev, vprev, us)
            np.testing.assert_allclose(h["q"][k, b], qn, rtol=0, atol=Q_ATOL)
            np.testing.assert_allclose(h["vel"][k, b], vn, rtol=0, atol=Q_ATOL)
            if k % tp["ep"]["sample_every"] == 0:
                # the tick from the GPU's own recorded commands, flags, positions
                sp, cs = t.samples(h["u"][k, b], h["ca"][k, b])
                t.sup.tick(k, sp, cs, h["q"][k, b])
            assert h["state"][k, b] == t.sup.state, (b, k, h["state"][k, b], t.sup.state)
            qprev, vprev = h["q"][k, b], h["vel"][k, b]
        r = t.sup.record()
        s = st[b]
        assert (s["state"], s["last_state"], s["done_step"]) == \
            (r["state"], r["last_state"], r["done_step"]), b
        assert (s["formation"], s["timer_ticks"], s["ticks"]) == \
            (t.sup.formation, t.sup.timer_ticks, t.sup.ticks), b
        np.testing.assert_array_equal(rec["dist"][b].view(np.uint64),
                                      np.asarray(r["dist"], np.float64).view(np.uint64))
        np.testing.assert_array_equal(rec["time"][b], r["time"])
        np.testing.assert_array_equal(rec["time_avoidance"][b], r["time_avoidance"])
        np.testing.assert_array_equal(rec["assignments"][b], r["assignments"])
        c = t.counts
        assert (s["n_auctions"], s["n_invalid"], s["n_skipped"], s["n_disagree"]) == \
            (c["auctions"], c["invalid"], c["skipped"], c["disagree"]), (b, s, c)
        finals.append(r)
    return finals


@pytest.mark.parametrize("central", [False, True])
def test_trial_teacher_forced_swarm6(cuda, central):
    """formations.yaml swarm6_3d's three formations per trial, four starts:
    trials that COMPLETE (all three formations converged) and trials that
    TERMINATE in GRIDLOCK (the gridlock timeout), in both assignment modes."""
    steps = 700
    case = _swarm6_case(central=central)
    tr, h, tp = _run(case, cuda, steps)
    fin = _teacher_forced(case, tr, h, tp, steps)
    states = {r["state"] for r in fin}
    assert all(r["done_step"] >= 0 for r in fin)   # every trial ended within the steps
    assert T.COMPLETE in states                    # at least one full record
    for r in fin:
        if r["state"] == T.COMPLETE:
            assert all(x > 0 for x in r["time"]) and all(a >= 1 for a in r["assignments"])


def test_trial_teacher_forced_disagreeing_chain(cuda):
    """Chain formations: the first auction of a formation ends with vehicles
    on different tables, so controllers start vehicle by vehicle and the
    flush rule skips auctions; the supervisor still sees vehicle 0's
    assignment message only."""
    steps = 400
    case = _chain_case()
    tr, h, tp = _run(case, cuda, steps)
    _teacher_forced(case, tr, h, tp, steps)
    st = tr.status()
    assert int(st["n_disagree"].sum()) > 0
    # some step ran with part of a swarm's controllers started
    partial = ((h["ctl"].sum(axis=2) > 0) & (h["ctl"].sum(axis=2) < case["q"].shape[1])).any()
    assert partial


@pytest.mark.parametrize("what", ["assignment", "watchdog", "gridlock"])
def test_trial_terminations(cuda, what):
    """The three ways supervisor.py terminates a trial: no assignment within
    ASSIGNMENT_TIMEOUT (here shorter than form_settle_time), the trial
    watchdog, and GRIDLOCK_TIMEOUT (a crowded start)."""
    steps = 300
    if what == "assignment":
        case = _swarm6_case(B=2, assignment_timeout=0.04)
    elif what == "watchdog":
        case = _swarm6_case(B=2, trial_timeout=1.5)
    else:
        case = _swarm6_case(B=3, seed=5, gridlock_timeout=0.4)
        case["q"][..., :2] *= 0.3
    tr, h, tp = _run(case, cuda, steps)
    fin = _teacher_forced(case, tr, h, tp, steps)
    st = tr.status()
    assert (st["state"] == T.TERMINATE).all() and (st["done_step"] >= 0).all()
    last = {r["last_state"] for r in fin}
    want = {"assignment": {T.WAITING}, "gridlock": {T.GRIDLOCK}}.get(what)
    if want is not None:
        assert last == want, last


def test_trial_chunks_equal_one_call(cuda):
    import torch
    case = _swarm6_case(B=3)
    tr1, h1, _ = _run(case, cuda, 500)
    tr2, h2, _ = _run(case, cuda, 500, chunks=[137, 200, 163])
    for k in ("q", "vel", "P", "ctl", "state"):
        assert np.array_equal(h1[k], h2[k]), k
    for k in ("q", "vel", "P", "flush", "ts", "ctl_on", "ring_u", "ring_ca", "posf", "dist",
              "t_conv", "t_avoid", "n_assign", "fidx"):
        assert torch.equal(getattr(tr1, k), getattr(tr2, k)), k


def test_trial_formation_index_out_of_range(cuda):
    """A trial whose formation sequence names a formation outside the table
    ends at its first step (TERMINATE, nothing of the table read); the other
    trials of the batch run as they do alone."""
    case = _swarm6_case(B=3)
    bad = case["fseq"].copy()
    bad[1, 2] = 7  # three formations in the table
    case_bad = dict(case, fseq=bad)
    tr_bad, h_bad, _ = _run(case_bad, cuda, 200)
    tr_ok, h_ok, _ = _run(case, cuda, 200)
    st = tr_bad.status()
    assert st[1]["state"] == T.TERMINATE and st[1]["done_step"] == 0
    for b in (0, 2):
        assert np.array_equal(h_bad["q"][:, b], h_ok["q"][:, b])
        assert np.array_equal(h_bad["state"][:, b], h_ok["state"][:, b])
