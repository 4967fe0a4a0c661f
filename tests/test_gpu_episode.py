"""GPU parity of closed-loop batched episodes (acl_episode_batch, SURVEY.md
§8f row 1) against oracle/episode_oracle.py.

Teacher-forced: every recorded step of the GPU episode is re-derived on the
CPU from the GPU's own state before that step -- the auction and adoption
(assignments bit-exact), DistCntrl + Safety (u within 1e-5 relative, CA flags
exact), makeSafeTraj (state within 1e-9 absolute), and the supervisor's
window predicates from the recorded commands (tick for tick exact). Then the
whole closed loop once more, untouched, against the CPU's own episode, and
chunked calls against one call (bit-identical).
"""
import numpy as np
import pytest

import episode_oracle as E
import helpers as H
import pyoracle as O

pytestmark = pytest.mark.gpu

U_RTOL = 1e-5      # control commands: fp64, within 1e-5 relative (north_star)
Q_ATOL = 1e-9      # one makeSafeTraj step from commands within U_RTOL * dt


def _cases():
    rng = np.random.RandomState(11)
    pts, adj, gains, q0 = H.swarm6()
    B = 6
    q = np.stack([q0 + (rng.normal(0, 0.4, q0.shape) if b else 0) for b in range(B)])
    q[..., 2] = 1.0
    a = dict(name="swarm6_3d", pts=list(pts), adj=list(adj), gains=list(gains),
             fidx=np.arange(B) % 3, q=q, vel=np.zeros((B, 6, 3)),
             P=np.stack([H.random_perm(rng, 6) for _ in range(B)]),
             steps=250, ep=dict())
    P20, A20 = H.simform("simform20_nc")
    p20 = [P20[0, 0], P20[1, 1]]
    a20 = [A20[0], A20[1]]
    g20 = [H.synth_gains(rng, x) for x in a20]
    B = 8
    q = np.stack([H.dense_positions(rng, 20, 7.0 + b) for b in range(B)])
    b_ = dict(name="simform20_dense", pts=p20, adj=a20, gains=g20, fidx=np.arange(B) % 2,
              q=q, vel=rng.normal(0, 0.2, (B, 20, 3)),
              P=np.stack([H.random_perm(rng, 20) for _ in range(B)]),
              steps=160, ep=dict(auction_every=40, bufflen=20))
    return [a, b_, _chain_case()]


def _chain_case(n=10, B=6, seed=21, tail=None):
    """Chain (path-graph) formations, n = 10: lockstep CBAA needs more than
    the reference's 2n rounds to reach consensus along a chain for many
    starts, so auctions end with vehicles on different tables, some of them
    valid (found with the CPU oracle; the GPU auction is bit-exact with it).

    tail: a lollipop instead -- a clique of n - tail vehicles with a chain of
    `tail` vehicles hanging off it; at n = 100 / 136 a plain chain almost
    never leaves a valid table, a long enough tail often does. These reach the
    per-vehicle control paths of the larger workgroups (33 <= n <= 128: the
    256-thread pair/gain kernels; n > 128: the 1 024-thread directed walk)."""
    rng = np.random.RandomState(seed)
    pts, adjs, gains, qs = [], [], [], []
    L = 5.0 if tail is None else n / 4.0
    tries = 0
    while len(qs) < B:
        tries += 1
        assert tries < 400, "no disagreeing case found"
        adj = np.zeros((n, n), np.uint8)
        perm = rng.permutation(n)
        if tail is None:
            chain = perm
        else:
            core = perm[:n - tail]
            adj[np.ix_(core, core)] = 1
            np.fill_diagonal(adj, 0)
            chain = perm[n - tail - 1:]
        for x, y in zip(chain[:-1], chain[1:]):
            adj[x, y] = adj[y, x] = 1
        p = np.c_[rng.uniform(-L, L, (n, 2)), rng.uniform(0, 2, n)]
        q = np.c_[rng.uniform(-L, L, (n, 2)), np.ones(n)]
        P0 = np.arange(n, dtype=np.uint16)
        r = O.solve(q, np.zeros((n, 3)), p, adj, np.zeros((3 * n, 3 * n)), P0)
        who = r["who"]
        nvalid = sum(E.is_perm(who[v]) for v in range(n))
        if r["status"]["flags"] & 0x02 or nvalid == 0:
            continue
        pts.append(p); adjs.append(adj); gains.append(H.synth_gains(rng, adj)); qs.append(q)
    name = f"chain{n}_disagree" if tail is None else f"lollipop{n}_{tail}_disagree"
    return dict(name=name, pts=pts, adj=adjs, gains=gains, fidx=np.arange(B),
                q=np.stack(qs), vel=np.zeros((B, n, 3)),
                P=np.stack([np.arange(n, dtype=np.uint16)] * B), steps=90,
                ep=dict(auction_every=30, bufflen=10), disagree=True)


def _case(ci):
    if ci < 3:
        return _cases()[ci]
    return {3: lambda: _chain_case(40, 4, 31),
            4: lambda: _chain_case(100, 3, 23, tail=40),
            5: lambda: _chain_case(136, 3, 25, tail=60)}[ci]()


def _episode(case, dev):
    import torch
    from aclswarm_amd import _lib as L
    from aclswarm_amd import engine
    T = engine.FormationTable.from_host(case["pts"], case["adj"], case["gains"], device=dev)
    ep = L.default_episode_params()
    for k, v in case["ep"].items():
        setattr(ep, k, v)
    e = engine.Episode(T, torch.from_numpy(case["fidx"].astype(np.int32)).to(dev),
                       torch.from_numpy(case["q"]).to(dev), torch.from_numpy(case["vel"]).to(dev),
                       torch.from_numpy(case["P"].astype(np.uint16).view(np.int16)).to(dev),
                       params=ep)
    return e, ep


@pytest.mark.parametrize("ci", [0, 1, 2, 3, 4, 5])
def test_episode_teacher_forced_parity(cuda, ci):
    """ci 2-5: chain (n = 10, 40) and lollipop (n = 100, 136) formations whose
    2n-round auctions end with vehicles on different tables -- each vehicle
    adopts its own valid table (auctioneer.cpp:250-295) and flies it until an
    agreed auction (per-vehicle control on the 64-, 256- and 1 024-thread
    paths)."""
    import torch
    case = _case(ci)
    e, eps = _episode(case, cuda)
    hist = e.run(case["steps"], history=True)
    torch.cuda.synchronize()
    h = {k: v.cpu().numpy() for k, v in hist.items()}
    h["P"] = h["P"].view(np.uint16)
    est = e.status()
    ep = E.params_from_struct(eps)
    B, n = case["q"].shape[:2]
    n_adopt = n_ca = n_dis = n_skip = 0
    for b in range(B):
        f = case["fidx"][b]
        p, adj, G = case["pts"][f], case["adj"][f], case["gains"][f]
        qprev, vprev = case["q"][b], case["vel"][b]
        state, flush = E.SwarmState(case["P"][b]), 0
        sup = E.Supervisor(n, ep)
        counts = dict(skipped=0, adopted=0, invalid=0, disagree=0)
        conv = grid = -1
        for k in range(case["steps"]):
            if k % ep["auction_every"] == 0:
                P_in, rows = state.solve_args()
                res = O.solve(qprev, vprev, p, adj, G, P_in, P_rows=rows)
                flush, ev = E.adopt(state, flush, res)
                counts[ev] += 1
            assert (h["P"][k, b] == state.P).all(), (b, k)
            u, us, ca = E.control_step(qprev, vprev, p, adj, G, state.P, tables=state.tables)
            np.testing.assert_allclose(h["u"][k, b], u, rtol=U_RTOL, atol=U_RTOL)
            assert (h["ca"][k, b] == ca).all(), (b, k)
            qn, vn = E.make_safe_traj(qprev, vprev, us, ep)
            np.testing.assert_allclose(h["q"][k, b], qn, rtol=0, atol=Q_ATOL)
            np.testing.assert_allclose(h["vel"][k, b], vn, rtol=0, atol=Q_ATOL)
            if k % ep["sample_every"] == 0:
                r = sup.tick(h["u"][k, b], h["ca"][k, b])
                if r is not None:
                    conv = k if (r[0] and conv < 0) else conv
                    grid = k if (r[1] and grid < 0) else grid
            qprev, vprev = h["q"][k, b], h["vel"][k, b]
            n_ca += int(ca.sum())
        st = est[b]
        assert st["n_auctions"] == counts["adopted"] + counts["invalid"] + counts["disagree"]
        assert (st["n_skipped"], st["n_invalid"], st["n_disagree"]) == \
            (counts["skipped"], counts["invalid"], counts["disagree"])
        assert (st["converged_step"], st["gridlock_step"]) == (conv, grid), b
        assert st["converged"] == int(sup.converged) and st["gridlocked"] == int(sup.gridlocked)
        assert st["n_samples"] == sup.n_samples
        assert st["n_ca_steps"] == int(h["ca"][:, b].sum())
        assert st["per_vehicle"] == int(state.tables is not None)
        n_adopt += counts["adopted"]
        n_dis += counts["disagree"]
        n_skip += counts["skipped"]
    if case.get("disagree"):
        assert n_dis > 0         # the chain formations end auctions on different tables
        assert n_skip > 0        # ... with vehicles on invalid ones: the next auction stalls
    else:
        assert n_adopt > 0
    if ci == 1:
        assert n_ca > 0          # the dense starts exercise collision avoidance


def test_episode_closed_loop_matches_cpu_episode(cuda):
    """The untouched GPU loop against the CPU's own loop, in the smooth regime
    (start grid spread 3x: no collision avoidance in 250 steps). With vehicles
    in contact the loop is not smooth -- collision avoidance snaps headings to
    sector edges -- and ulp-level differences of the atan2/asin edges can pick
    a different edge some steps later; the teacher-forced test is the per-step
    gate for those cases."""
    import torch
    case = dict(_cases()[0])
    rng = np.random.RandomState(5)
    _, _, _, q0 = H.swarm6()
    q = np.stack([3.0 * q0 + (rng.normal(0, 0.4, q0.shape) if b else 0) for b in range(6)])
    q[..., 2] = 1.0
    case["q"] = q
    e, eps = _episode(case, cuda)
    e.run(case["steps"])
    torch.cuda.synchronize()
    ep = E.params_from_struct(eps)
    qg = e.q.cpu().numpy()
    Pg = e.P.cpu().numpy().view(np.uint16)
    est = e.status()
    assert int(est["n_ca_steps"].sum()) == 0
    for b in range(case["q"].shape[0]):
        f = case["fidx"][b]
        r = E.run_episode(case["q"][b], case["vel"][b], case["P"][b], case["pts"][f],
                          case["adj"][f], case["gains"][f], case["steps"], ep)
        np.testing.assert_allclose(qg[b], r["q"], rtol=0, atol=1e-9)
        assert (Pg[b] == r["P"]).all()
        assert est[b]["converged_step"] == r["converged_step"]


@pytest.mark.parametrize("ci", [1, 2])
def test_episode_chunks_equal_one_call(cuda, ci):
    """ci 2: per-vehicle tables carried across the call boundary in the
    workspace."""
    import torch
    case = _cases()[ci]
    e1, _ = _episode(case, cuda)
    e1.run(case["steps"])
    e2, _ = _episode(case, cuda)
    e2.run(57)
    e2.run(case["steps"] - 57)
    torch.cuda.synchronize()
    for k in ("q", "vel", "P", "flush", "est", "ring_u", "ring_ca"):
        assert torch.equal(getattr(e1, k), getattr(e2, k)), k


@pytest.mark.parametrize("lat,ci", [(-1, 0), (3, 0), (25, 0), (7, 2)])
def test_episode_auction_latency(cuda, lat, ci):
    """Auctions that take time (acl_episode_params_t::auction_latency): the
    reference timing (-1: ceil(2 n d_max 1 ms / control_dt), 4-6 steps for
    the swarm6 formations), a fixed 3 steps, and 25 steps > the auto-auction period of 10
    (every auction restarted, coordination_ros.cpp:355-358). Teacher-forced:
    the CPU state machine (episode_oracle.Auctions) runs CBAA from the GPU's
    own state at each auto-auction and must give the assignment the GPU's
    controller used at every step, and the same counters."""
    import torch
    per_vehicle = ci == 2    # chain formations: pending auctions end in disagreement
    case = dict(_cases()[ci], ep=dict(auction_every=10, auction_latency=lat), steps=64)
    e, eps = _episode(case, cuda)
    hist = e.run(40, history=True)
    hist2 = e.run(24, history=True)  # a pending auction crosses the call boundary
    torch.cuda.synchronize()
    h = {k: np.concatenate([v.cpu().numpy(), hist2[k].cpu().numpy()]) for k, v in hist.items()}
    h["P"] = h["P"].view(np.uint16)
    est = e.status()
    ep = E.params_from_struct(eps)
    B, n = case["q"].shape[:2]
    for b in range(B):
        f = case["fidx"][b]
        p, adj, G = case["pts"][f], case["adj"][f], case["gains"][f]
        auc = E.Auctions(E.auction_latency_steps(n, adj, ep))
        state = E.SwarmState(case["P"][b])
        qprev, vprev = case["q"][b], case["vel"][b]
        for k in range(case["steps"]):
            if k % ep["auction_every"] == 0:
                auc.auto(k, state, lambda P_in, rows: O.solve(qprev, vprev, p, adj, G, P_in,
                                                              P_rows=rows))
            else:
                auc.tick(k, state)
            assert (h["P"][k, b] == state.P).all(), (lat, b, k)
            if per_vehicle:
                u, _, _ = E.control_step(qprev, vprev, p, adj, G, state.P, tables=state.tables)
                np.testing.assert_allclose(h["u"][k, b], u, rtol=U_RTOL, atol=U_RTOL)
            qprev, vprev = h["q"][k, b], h["vel"][k, b]
        st, c = est[b], auc.counts
        assert (st["n_auctions"], st["n_restarted"], st["n_skipped"]) == \
            (c["auctions"], c["restarted"], c["skipped"]), (st, c)
        assert (st["n_invalid"], st["n_disagree"]) == (c["invalid"], c["disagree"])
        assert st["pending_step"] == (auc.pending + 1 if auc.pending >= 0 else 0)
        assert st["per_vehicle"] == int(state.tables is not None)
        if lat == 25:
            assert c["adopted"] == 0 and c["restarted"] == c["auctions"] - 1
        elif not per_vehicle:
            assert c["adopted"] > 0


def test_episode_zeroed_status_mid_period(cuda):
    """A status zeroed at the start (pending_step 0 = none; only converged_step
    and gridlock_step -1), with auctions that take time and a first step that
    is not an auto-auction step: the first auction counts no restart, nothing
    completes before it, and the teacher-forced state machine agrees."""
    import torch
    case = dict(_cases()[0], ep=dict(auction_every=10, auction_latency=3), steps=40)
    e, eps = _episode(case, cuda)
    est0 = np.zeros(e.B, dtype=e.status().dtype)
    est0["converged_step"] = -1
    est0["gridlock_step"] = -1
    e.est.copy_(torch.from_numpy(est0.view(np.uint8).reshape(e.B, -1).copy()))
    e.step = 5
    hist = e.run(case["steps"], history=True)
    torch.cuda.synchronize()
    h = {k: v.cpu().numpy() for k, v in hist.items()}
    h["P"] = h["P"].view(np.uint16)
    est = e.status()
    ep = E.params_from_struct(eps)
    B, n = case["q"].shape[:2]
    for b in range(B):
        f = case["fidx"][b]
        p, adj, G = case["pts"][f], case["adj"][f], case["gains"][f]
        auc = E.Auctions(3)
        state = E.SwarmState(case["P"][b])
        qprev, vprev = case["q"][b], case["vel"][b]
        for k in range(case["steps"]):
            s = 5 + k
            if s % ep["auction_every"] == 0:
                auc.auto(s, state, lambda P_in, rows: O.solve(qprev, vprev, p, adj, G, P_in,
                                                              P_rows=rows))
            else:
                auc.tick(s, state)
            assert (h["P"][k, b] == state.P).all(), (b, k)
            qprev, vprev = h["q"][k, b], h["vel"][k, b]
        st, c = est[b], auc.counts
        assert st["n_restarted"] == c["restarted"] == 0
        assert (st["n_auctions"], st["n_skipped"]) == (c["auctions"], c["skipped"])
        assert st["pending_step"] == (auc.pending + 1 if auc.pending >= 0 else 0)


@pytest.mark.parametrize("ci", [0, 1, 3, 5])
def test_episode_central_teacher_forced(cuda, ci):
    """ACL_ASSIGN_CENTRAL (coordination_ros.cpp:330-343): every auto-auction
    applies the operator's Hungarian assignment (assignment.py:94-137 with
    last = the swarm's current P) instead of CBAA. Teacher-forced: at each
    auto-auction the CPU's Hungarian (oracle/hungarian_oracle.c) from the
    GPU's own q and P must give the assignment the GPU's controller used
    (bit-exact), and every step's commands, flags and state as in the CBAA
    test; counters (assignments applied) equal."""
    import torch
    case = dict(_case(ci))
    case["ep"] = dict(case["ep"], assignment=1, auction_latency=7)  # (latency: ignored)
    e, eps = _episode(case, cuda)
    hist = e.run(case["steps"], history=True)
    torch.cuda.synchronize()
    h = {k: v.cpu().numpy() for k, v in hist.items()}
    h["P"] = h["P"].view(np.uint16)
    est = e.status()
    ep = E.params_from_struct(eps)
    assert ep["assignment"] == 1
    B, n = case["q"].shape[:2]
    changed = 0
    for b in range(B):
        f = case["fidx"][b]
        p, adj, G = case["pts"][f], case["adj"][f], case["gains"][f]
        auc = E.Auctions(7, central=True)
        state = E.SwarmState(case["P"][b])
        qprev, vprev = case["q"][b], case["vel"][b]
        for k in range(case["steps"]):
            P0 = state.P.copy()
            if k % ep["auction_every"] == 0:
                auc.auto(k, state, None, central=lambda: E.central_assign(state, qprev, p))
            else:
                auc.tick(k, state)
            changed += int((P0 != state.P).any())
            assert (h["P"][k, b] == state.P).all(), (b, k)
            assert state.tables is None
            u, us, ca = E.control_step(qprev, vprev, p, adj, G, state.P)
            np.testing.assert_allclose(h["u"][k, b], u, rtol=U_RTOL, atol=U_RTOL)
            assert (h["ca"][k, b] == ca).all(), (b, k)
            qn, vn = E.make_safe_traj(qprev, vprev, us, ep)
            np.testing.assert_allclose(h["q"][k, b], qn, rtol=0, atol=Q_ATOL)
            qprev, vprev = h["q"][k, b], h["vel"][k, b]
        st, c = est[b], auc.counts
        assert (st["n_auctions"], st["n_invalid"]) == (c["auctions"], c["invalid"]), (st, c)
        assert (st["n_skipped"], st["n_disagree"], st["n_restarted"]) == (0, 0, 0)
        assert st["pending_step"] == 0 and st["per_vehicle"] == 0
    assert changed > 0  # the operator's assignment replaced the starting ones


def test_episode_central_bad_problem_keeps_P(cuda):
    """A swarm whose Hungarian problem is NONFINITE (a vehicle position is
    NaN: scipy's linear_sum_assignment would raise in the operator) keeps its
    assignment and counts n_invalid; the others get theirs."""
    import torch
    case = dict(_cases()[0], steps=3, ep=dict(auction_every=2, assignment=1))
    q = case["q"].copy()
    q[2, 3, 0] = np.nan
    case["q"] = q
    e, _ = _episode(case, cuda)
    hist = e.run(case["steps"], history=True)
    torch.cuda.synchronize()
    Ph = hist["P"].cpu().numpy().view(np.uint16)
    est = e.status()
    assert (Ph[:, 2] == case["P"][2]).all()
    assert est[2]["n_invalid"] == 2 and est[2]["n_auctions"] == 0
    for b in (0, 1, 3):
        P, _, _, st = O.hungarian(case["q"][b], case["pts"][case["fidx"][b]],
                                  P_last=case["P"][b])
        assert st == 0 and (Ph[0, b] == P).all()
        assert est[b]["n_auctions"] == 2 and est[b]["n_invalid"] == 0
