"""GPU: acl_solve_batch's fused auction + control kernel (the control phase of a
swarm whose vehicles all adopted one assignment runs in the auction's own
workgroup; swarms with per-vehicle rows go to the directed gain kernel).

Checked through the C ABI against the CPU restatement (tables, assignments,
flags, margins bit-exact; commands 1e-5 relative) and against
acl_control_batch on the same assignments (the stand-alone pair kernel: the
same terms in another summation order, so 1e-12)."""
import numpy as np
import pytest

import helpers as H
import pyoracle as O
from test_gpu_parity import _compare, _gpu_solve, _oracle

pytestmark = pytest.mark.gpu


def _two_components(rng, n):
    """A formation graph with two components (vehicles in different components
    never exchange bids: their tables end different, so the swarm's vehicles
    hold per-vehicle assignments)."""
    a = np.zeros((n, n), np.uint8)
    h = n // 2
    a[:h, :h] = 1
    a[h:, h:] = 1
    np.fill_diagonal(a, 0)
    return a


def _case(rng, n, F, disconnected):
    pts, adjs = [], []
    for f in range(F):
        pts.append(np.c_[rng.uniform(-n, n, (n, 2)), rng.uniform(0, 2, n)])
        if disconnected and f == F - 1 and n >= 4:
            a = _two_components(rng, n)
        else:
            a = np.ones((n, n), np.uint8) - np.eye(n, dtype=np.uint8)
            for _ in range(max(1, n // 3)):
                i, j = rng.randint(0, n, 2)
                if i != j:
                    a[i, j] = a[j, i] = 0
        adjs.append(a)
    gains = [H.synth_gains(rng, a, scale=1.0) for a in adjs]
    return pts, adjs, gains


@pytest.mark.parametrize("n", [2, 7, 20, 33, 64, 65, 100, 128, 129, 200])
def test_fused_solve_vs_oracle_and_control(cuda, n):
    """n > 128: the wide solve's fused control phase (wide_control, 5-plane
    records) for the uniform swarms, the directed gain kernel for the
    disconnected formation's per-vehicle swarms, gate margins on."""
    import torch
    from aclswarm_amd import engine
    rng = np.random.RandomState(4000 + n)
    F, B = 3, 24
    pts, adjs, gains = _case(rng, n, F, disconnected=True)
    fidx = np.arange(B) % F
    q = np.stack([H.dense_positions(rng, n, 2.0 * n) for _ in range(B)])
    vel = rng.normal(0, 0.3, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    ref = _oracle(pts, adjs, gains, fidx, q, vel, P_in)
    _compare(gpu, ref)
    # the disconnected formation's swarms really took the per-vehicle path
    if n >= 4:
        agree = (gpu["status"]["flags"] & 0x2) != 0
        assert not agree[fidx == F - 1].all()
    # uniform swarms: the fused phase vs the stand-alone pair kernel
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(pts, adjs, gains, device=dev, planes=5)
    uni = [b for b in range(B) if gpu["status"]["flags"][b] & 0x3 == 0x3]
    assert uni
    P = torch.from_numpy(gpu["P_out"][uni].view(np.int16)).to(dev)
    out = engine.control(T, torch.from_numpy(fidx[uni].astype(np.int32)).to(dev),
                         torch.from_numpy(q[uni]).to(dev), torch.from_numpy(vel[uni]).to(dev), P,
                         want_gate_margin=True)
    torch.cuda.synchronize()
    c = {k: v.cpu().numpy() for k, v in out.items()}
    np.testing.assert_array_equal(c["ca_flag"], gpu["ca_flag"][uni])
    for k in ("u", "u_safe"):
        np.testing.assert_allclose(c[k], gpu[k][uni], rtol=1e-12, atol=1e-12, err_msg=k)
    np.testing.assert_array_equal(c["gate_margin"], gpu["gate_margin"][uni])


def test_fused_is_deterministic_and_order_free(cuda):
    """The same C3-shaped batch solved twice, and in reverse order: every
    output bit-identical (fixed tile order and wave-order sums in the fused
    phase; no cross-workgroup state but the collision list)."""
    import torch
    from aclswarm_amd import engine
    P100, A100 = H.simform("simform100_nc")
    rng = np.random.RandomState(17)
    n, B = 100, 48
    pts = [P100[s, k] for s in range(P100.shape[0]) for k in range(2)]
    adjs = [A100[s] for s in range(A100.shape[0]) for k in range(2)]
    gains = [H.synth_gains(rng, a) for a in adjs]
    F = len(pts)
    fidx = np.arange(B) % F
    q = np.stack([H.random_positions(rng, n, 40.0) for _ in range(B)])
    q[::5, :, :2] *= 0.3  # crowded: collision avoidance active in some swarms
    vel = rng.normal(0, 0.2, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    a = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    b = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    r = _gpu_solve(pts, adjs, gains, fidx[::-1].copy(), q[::-1].copy(), vel[::-1].copy(),
                   P_in[::-1].copy())
    for k in ("P_out", "u", "u_safe", "ca_flag", "who", "gate_margin"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        np.testing.assert_array_equal(a[k], r[k][::-1], err_msg=k)
    assert (a["status"]["flags"] & 0x20).any()  # CA_ACTIVE somewhere
    sample = [0, 5, 17, 47]
    ref = _oracle(pts, adjs, gains, fidx[sample], q[sample], vel[sample], P_in[sample])
    _compare({k: v[sample] for k, v in a.items()}, ref)


@pytest.mark.parametrize("n", [20, 100, 129, 320])
def test_skip_margin_same_outcome(cuda, n):
    """acl_solve_args_t::skip_margin: the auction without its decision-margin
    bookkeeping gives the same tables, assignments, round counts and commands
    bit for bit; the status margin is -1 and FRAGILE is never set. n = 129 is
    the wide kernel, whose level walk then stops at each vehicle's winner."""
    rng = np.random.RandomState(5100 + n)
    F, B = 3, 32
    pts, adjs, gains = _case(rng, n, F, disconnected=True)
    fidx = np.arange(B) % F
    q = np.stack([H.dense_positions(rng, n, 2.0 * n) for _ in range(B)])
    vel = rng.normal(0, 0.3, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    for early in (True, False):
        a = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in, early_exit=early)
        b = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in, early_exit=early, margin=False)
        for k in ("P_out", "who", "u", "u_safe", "ca_flag", "gate_margin"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        for k in ("eff_rounds", "rounds", "n_invalid", "n_ca"):
            np.testing.assert_array_equal(a["status"][k], b["status"][k], err_msg=k)
        np.testing.assert_array_equal(a["status"]["flags"] & np.uint32(0xFFFFFFBF), b["status"]["flags"])
        assert (b["status"]["margin"] == -1.0).all()
    ref = _oracle(pts, adjs, gains, fidx[:6], q[:6], vel[:6], P_in[:6])
    _compare({k: v[:6] for k, v in a.items()}, ref)


@pytest.mark.parametrize("n", [20, 100, 200])
def test_persistent_workspace_same_as_memset(cuda, n):
    """acl_solve_args_t::ws_persistent (ABI 10): the collision-avoidance
    launch leaves the list counters zero, so solves without the per-call
    memset -- crowded swarms listed every call, an acl_control_batch call on
    the same workspace in between -- give the outputs (n_ca counts and CA
    flags included) of a solve that zeroes them first; a call of another
    shape in between makes the next one zero them again (their offset moves)."""
    import torch
    from aclswarm_amd import engine
    rng = np.random.RandomState(5300 + n)
    F, B = 3, 40
    pts, adjs, gains = _case(rng, n, F, disconnected=True)
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(pts, adjs, gains, device=dev, planes=5)
    fidx = torch.from_numpy((np.arange(B) % F).astype(np.int32)).to(dev)
    q = np.stack([H.random_positions(rng, n, 2.0 * n) for _ in range(B)])
    q[::3, :, :2] *= 0.05  # crowded: listed for collision avoidance
    qd = torch.from_numpy(q).to(dev)
    vel = torch.from_numpy(rng.normal(0, 0.3, (B, n, 3))).to(dev)
    P_in = torch.from_numpy(np.stack([H.random_perm(rng, n) for _ in range(B)]).view(np.int16)).to(dev)

    def run(persistent, b=B):
        o = engine.solve(T, fidx[:b], qd[:b], vel[:b], P_in[:b], persistent=persistent)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in o.items()}

    def same(got, ref, what):
        for k in ("P_out", "status", "u", "u_safe", "ca_flag"):
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{k} ({what})")

    ref = run(False)
    st = engine.status_to_numpy(torch.from_numpy(ref["status"]))
    assert (st["n_ca"] > 0).sum() >= B // 4  # many swarms listed
    for it in range(3):
        assert engine._counters_zero(dev, n, B)  # this call runs without the memset
        same(run(True), ref, f"call {it}")
        # a control call of the same shape on the same workspace between solves
        engine.control(T, fidx, qd, vel, torch.from_numpy(ref["P_out"]).to(dev))
    small = run(True, 9)  # another shape: its counters are zeroed by that call
    same(small, {k: v[:9] for k, v in ref.items()}, "small")
    assert not engine._counters_zero(dev, n, B)
    same(run(True), ref, "after the small batch")
    assert engine._counters_zero(dev, n, B)
    same(run(True), ref, "persistent again")
