"""GPU: decision margin, gate decisions near their thresholds, bad formation
indices, directed graphs on the tiled pair kernel -- through the C ABI,
against the CPU restatement (oracle/)."""
import numpy as np
import pytest

import helpers as H
import pyoracle as O
from test_gpu_parity import U_RTOL, _compare, _gpu_solve, _oracle

pytestmark = pytest.mark.gpu


def test_fidx_out_of_range_is_bad_input(cuda):
    """A swarm whose formation index is outside [0, F) is flagged BAD_INPUT,
    gets P_out = P_in, zero commands, margin 1 and gate margin +inf, and
    nothing of the formation table is read for it; the other swarms of the
    batch are solved as usual."""
    import torch
    from aclswarm_amd import engine
    P, A = H.simform("simform20_nc")
    rng = np.random.RandomState(31)
    pts, adjs = [P[0, 0], P[1, 0]], [A[0], A[1]]
    gains = [H.synth_gains(rng, a) for a in adjs]
    B, n = 8, 20
    fidx = np.array([0, 2, 1, -1, 0, 1, 7, 0], np.int32)
    q = np.stack([H.random_positions(rng, n, 20.0) for _ in range(B)])
    vel = rng.normal(0, 0.2, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    gpu = _gpu_solve(pts, adjs, gains, fidx, q, vel, P_in)
    bad = (fidx < 0) | (fidx >= 2)
    for b in np.nonzero(bad)[0]:
        st = gpu["status"][b]
        assert st["flags"] == 0x10 and st["margin"] == 1.0, st
        np.testing.assert_array_equal(gpu["P_out"][b], P_in[b])
        assert not np.any(gpu["u"][b]) and not np.any(gpu["u_safe"][b])
        assert gpu["gate_margin"][b] == np.inf
    good = np.nonzero(~bad)[0]
    ref = _oracle(pts, adjs, gains, fidx[good], q[good], vel[good], P_in[good])
    _compare({k: v[good] for k, v in gpu.items()}, ref)
    # acl_control_batch: the same check in its hand-off kernel
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(pts, adjs, gains, device=dev)
    out = engine.control(T, torch.from_numpy(fidx).to(dev), torch.from_numpy(q).to(dev),
                         torch.from_numpy(vel).to(dev),
                         torch.from_numpy(P_in.view(np.int16)).to(dev))
    torch.cuda.synchronize()
    st = engine.status_to_numpy(out["status"])
    assert ((st["flags"] & 0x10) != 0).tolist() == bad.tolist()
    assert not np.any(out["u_safe"].cpu().numpy()[bad])


def test_margin_flags_fragile_ties(cuda):
    """Vehicles at bit-identical positions bid bit-identical prices: the
    outcome is decided by vehicle order alone -> margin 0, FRAGILE, exactly as
    the oracle; well-separated swarms are not fragile."""
    rng = np.random.RandomState(41)
    n = 10
    p = H.random_positions(rng, n, 10.0)
    adj = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
    G = H.synth_gains(rng, adj)
    B = 6
    q = np.stack([H.random_positions(rng, n, 12.0) for _ in range(B)])
    q[1, 3] = q[1, 4]          # two vehicles on one spot
    q[2, :] = q[2, 0]          # everybody on one spot
    vel = np.zeros((B, n, 3))
    P_in = np.stack([np.arange(n, dtype=np.uint16)] * B)
    gpu = _gpu_solve([p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in)
    ref = _oracle([p], [adj], [G], np.zeros(B, np.int32), q, vel, P_in)
    _compare(gpu, ref)
    assert gpu["status"]["margin"][2] == 0.0 and gpu["status"]["flags"][2] & 0x40
    assert gpu["status"]["flags"][1] & 0x40
    assert (gpu["status"]["margin"][[0, 3, 4, 5]] > 1e-6).all()


def _gate_case(rng, n, B, thr_xy, thr_z, delta):
    """Swarms whose first edges sit within |delta| of a gate threshold:
    vehicle v at formation point v (P = identity), positions built so that
    |q_ij.xy| - dstar_xy(i,j) and |q_ij.z| - dstar_z(i,j) = thr + d for chosen
    pairs (d drawn in [-delta, delta], zero included)."""
    pts, qs = [], []
    for b in range(B):
        p = np.c_[rng.uniform(-4, 4, (n, 2)), rng.uniform(0, 2, n)]
        dxy, dz = O.pdist(p)
        q = np.c_[rng.uniform(-8, 8, (n, 2)), rng.uniform(0, 2, n)]
        for (i, j) in ((0, 1), (2, 3)):
            d = rng.choice([-delta, -delta / 3, 0.0, delta / 3, delta])
            ang = rng.uniform(0, 2 * np.pi)
            r = dxy[i, j] + thr_xy + d
            q[j, 0] = q[i, 0] + r * np.cos(ang)
            q[j, 1] = q[i, 1] + r * np.sin(ang)
            dd = rng.choice([-delta, 0.0, delta])
            q[j, 2] = q[i, 2] + (dz[i, j] + thr_z + dd)
        pts.append(p)
        qs.append(q)
    return pts, np.stack(qs)


@pytest.mark.parametrize("planes", [5, 9])
def test_gates_near_threshold(cuda, planes):
    """Edges within 1e-12 of e_xy_thr / e_z_thr (distcntrl.cpp:75,80): the
    gates are decided on correctly rounded e, as the oracle decides them, so
    the commands agree to 1e-5 (a flipped gate would move u by ~K1 atan(K2
    thr) |q|, far more) and the gate margin agrees to 1e-10. planes 5 runs the
    pair kernel, 9 the directed walk."""
    import torch
    from aclswarm_amd import engine
    rng = np.random.RandomState(7 + planes)
    n, B = 6, 64
    g = O.default_gains()
    pts, q = _gate_case(rng, n, B, g.e_xy_thr, g.e_z_thr, 1e-12)
    adj = (np.ones((n, n)) - np.eye(n)).astype(np.uint8)
    adjs = [adj] * B
    gains = [(H.synth_gains if planes == 5 else H.random_block_gains)(rng, adj, scale=1.0)
             for _ in range(B)]
    vel = rng.normal(0, 0.1, (B, n, 3))
    P = np.stack([np.arange(n, dtype=np.uint16)] * B)
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(pts, adjs, gains, device=dev, planes=planes)
    assert T.gain_planes == planes
    fidx = np.arange(B, dtype=np.int32)
    out = engine.control(T, torch.from_numpy(fidx).to(dev), torch.from_numpy(q).to(dev),
                         torch.from_numpy(vel).to(dev), torch.from_numpy(P.view(np.int16)).to(dev),
                         want_gate_margin=True)
    torch.cuda.synchronize()
    u = out["u"].cpu().numpy()
    gm = out["gate_margin"].cpu().numpy()
    near = 0
    for b in range(B):
        dxy, dz = O.pdist(pts[b])
        gmin = np.inf
        for v in range(n):
            ur = O.control(v, q[b], vel[b, v], np.arange(n, dtype=np.uint16), adj, gains[b],
                           pts[b])
            np.testing.assert_allclose(u[b, v], ur, rtol=U_RTOL, atol=U_RTOL)
            for j in range(n):
                if adj[v, j]:
                    qij = q[b, j] - q[b, v]
                    exy = np.sqrt(qij[0] ** 2 + qij[1] ** 2) - dxy[v, j]
                    ez = np.sqrt(qij[2] ** 2) - dz[v, j]
                    mx = abs(abs(exy) - g.e_xy_thr) / g.e_xy_thr
                    mz = abs(abs(ez) - g.e_z_thr) / g.e_z_thr
                    gmin = min(gmin, mx, mz)
        near += gmin < 1e-11
        assert abs(gm[b] - gmin) <= 1e-10, (b, gm[b], gmin)
    assert near > B // 2


def test_directed_graph_tiled_pair_kernel(cuda):
    """An asymmetric adjmat (directed edges) on the tiled-record pair kernel:
    every pair with one direction only applies one gain block; the full solve
    matches the oracle (tables bit-exact, commands 1e-5)."""
    import torch
    from aclswarm_amd import engine
    rng = np.random.RandomState(77)
    n, F, B = 37, 3, 24
    pts, adjs = [], []
    for f in range(F):
        pts.append(np.c_[rng.uniform(-n, n, (n, 2)), rng.uniform(0, 2, n)])
        a = np.ones((n, n), np.uint8) - np.eye(n, dtype=np.uint8)
        for _ in range(3 * n):
            i, j = rng.randint(0, n, 2)
            a[i, j] = 0  # one direction only
        adjs.append(a)
    gains = [H.synth_gains(rng, a, scale=1.0) for a in adjs]
    for G in gains:  # keep the 5-entry structure on the diagonal blocks
        for i in range(n):
            G[3 * i + np.array([0, 1, 2, 2]), 3 * i + np.array([2, 2, 0, 1])] = 0.0
    fidx = np.arange(B) % F
    q = np.stack([H.dense_positions(rng, n, 2.0 * n) for _ in range(B)])
    vel = rng.normal(0, 0.3, (B, n, 3))
    P_in = np.stack([H.random_perm(rng, n) for _ in range(B)])
    dev = torch.device("cuda:0")
    T = engine.FormationTable.from_host(pts, adjs, gains, device=dev, planes=5)
    T.tile_gains()
    out = engine.solve(T, torch.from_numpy(fidx.astype(np.int32)).to(dev),
                       torch.from_numpy(q).to(dev), torch.from_numpy(vel).to(dev),
                       torch.from_numpy(P_in.view(np.int16)).to(dev), want_who=True,
                       want_gate_margin=True)
    torch.cuda.synchronize()
    gpu = {k: v.cpu().numpy() for k, v in out.items()}
    gpu["P_out"] = gpu["P_out"].view(np.uint16)
    gpu["who"] = gpu["who"].view(np.uint16)
    gpu["status"] = np.ascontiguousarray(gpu["status"]).view(O.STATUS_DTYPE).reshape(-1)
    ref = _oracle(pts, adjs, gains, fidx, q, vel, P_in)
    _compare(gpu, ref)
