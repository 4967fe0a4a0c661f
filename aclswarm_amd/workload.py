"""Synthetic batched workloads generated on the device (no host round trip).

Formations come from the reference generator itself
(aclswarm_sim/nodes/generate_random_formation.py:20-96, numpy MT19937 seeded
per group) run on the device by acl_generate_formation_groups, bit-exact; a
torch-Philox version of the same recipe is kept for other shapes. Start
positions follow start.sh:19-61 (discs of radius 0.75 in a square, z =
takeoff altitude) on torch Philox streams (the reference draws them from the
shell's $RANDOM).

Gains are synthetic (random values with the reference's block structure is
not needed for throughput): formation gain design for 65536 unique
formations would be the ADMM workload (config C5), not this one.
"""
import torch


def nonoverlapping_points(B, n, side_x, side_y, z_lo, z_hi, min_dist, gen, device,
                          max_tries=100000):
    """[B][n][3] f64: per swarm, n points uniform in the box, xy pairwise
    distance >= min_dist (sequential rejection, vectorized over swarms)."""
    pts = torch.zeros((B, n, 3), dtype=torch.float64, device=device)
    for k in range(n):
        todo = torch.arange(B, device=device)
        tries = 0
        while todo.numel():
            m = todo.numel()
            cx = (torch.rand(m, generator=gen, device=device, dtype=torch.float64) - 0.5) * side_x
            cy = (torch.rand(m, generator=gen, device=device, dtype=torch.float64) - 0.5) * side_y
            if k == 0:
                ok = torch.ones(m, dtype=torch.bool, device=device)
            else:
                prev = pts[todo, :k, :2]
                d2 = (prev[..., 0] - cx[:, None]) ** 2 + (prev[..., 1] - cy[:, None]) ** 2
                ok = (d2 >= min_dist * min_dist).all(dim=1)
            acc = todo[ok]
            pts[acc, k, 0] = cx[ok]
            pts[acc, k, 1] = cy[ok]
            todo = todo[~ok]
            tries += 1
            if tries > max_tries:
                raise RuntimeError("point sampler: area too small for n points")
    if z_hi > z_lo:
        pts[..., 2] = z_lo + (z_hi - z_lo) * torch.rand((B, n), generator=gen, device=device,
                                                          dtype=torch.float64)
    else:
        pts[..., 2] = z_lo
    return pts


def random_adjacency(B, n, complete, gen, device):
    """[B][n][n] bool: complete graph minus m ~ U[1, n-4] random pairs
    (generate_random_formation.py:63-74)."""
    adj = ~torch.eye(n, dtype=torch.bool, device=device).expand(B, n, n).clone()
    if complete or n < 5:
        return adj
    m = torch.randint(1, n - 4 + 1, (B,), generator=gen, device=device)
    M = n - 4
    rows = torch.randint(0, n, (B, M), generator=gen, device=device)
    cols = torch.randint(0, n, (B, M), generator=gen, device=device)
    keep = torch.arange(M, device=device)[None, :] < m[:, None]
    bidx = torch.arange(B, device=device)[:, None].expand(B, M)
    bb, rr, cc = bidx[keep], rows[keep], cols[keep]
    adj[bb, rr, cc] = False
    adj[bb, cc, rr] = False
    return adj


def pack_bits(adj):
    """[B][n][n] bool -> [B][n][W] int64 bit rows (bit j of word j//64)."""
    B, n, _ = adj.shape
    W = (n + 63) // 64
    pad = torch.zeros((B, n, W * 64), dtype=torch.int64, device=adj.device)
    pad[..., :n] = adj.to(torch.int64)
    shifts = torch.arange(64, device=adj.device, dtype=torch.int64)
    return (pad.view(B, n, W, 64) << shifts).sum(dim=-1)


def reference_formations(nf, n, L, complete, seed0, device, h=2.0, min_dist=2.0):
    """nf formations from the reference's own generator on the device
    (acl_generate_formation_groups = generate_formation_group after
    np.random.seed(seed0 + f), generate_random_formation.py:59-80): formation
    'A' of each group and the group's graph. Returns (p [nf][n][3] f64,
    adj [nf][n][n] bool)."""
    from . import engine
    seeds = torch.arange(seed0, seed0 + nf, dtype=torch.int64, device=device)
    g = engine.generate_formation_groups(seeds, n, complete, L, L, h, min_dist)
    if int((g["status"] != 0).sum().item()):
        raise RuntimeError("reference_formations: a formation did not fit the box")
    return g["points"][:, 0].contiguous(), g["adj"].bool()


def simform_workload(B, n, gen, device, F=None, L=None, complete=False, gains_scale=0.05,
                     planes=5, formations="reference", seed0=0):
    """Config C3 (n=100, noncomplete, L=40) style batch.

    F=None: every swarm has its own formation (points, graph, gains): the
    Monte-Carlo setting of the north star, and the one whose bytes are
    dominated by the per-swarm gains stream.
    planes=5: gain blocks with the structure admm::Solver::solve produces
    ([a b 0; c d 0; 0 0 e], solver.cpp:49-77), 5-entry records per edge;
    planes=9: unstructured random 3x3 blocks as 9 planes.
    formations="reference": points and graphs from the reference generator
    itself (seeds seed0 .. seed0 + F - 1, bit-exact, on the device);
    "philox": the same recipe on torch Philox streams.
    Returns dict of device tensors (formation table + swarm inputs).
    """
    if L is None:
        L = 15.0 if n <= 20 else 40.0 * (n / 100.0) ** 0.5
    nf = B if F is None else F
    if formations == "reference":
        p, adj = reference_formations(nf, n, L, complete, seed0, device)
    else:  # torch Philox streams with the same recipe
        p = nonoverlapping_points(nf, n, L, L, 0.0, 2.0, 2.0, gen, device)
        adj = random_adjacency(nf, n, complete, gen, device)
    bits = pack_bits(adj)
    E = adj.sum(dim=(1, 2)).to(torch.int64)
    goff = torch.zeros(nf, dtype=torch.int64, device=device)
    goff[1:] = torch.cumsum(E, 0)[:-1]
    Etot = int(E.sum().item())
    gains = torch.empty(planes * Etot, dtype=torch.float64, device=device)
    gains.uniform_(-gains_scale, gains_scale, generator=gen)
    side = 20.0 * (n / 20.0) ** 0.5
    q = nonoverlapping_points(B, n, side, side, 1.0, 1.0, 1.5, gen, device)
    vel = 0.1 * torch.randn((B, n, 3), generator=gen, device=device, dtype=torch.float64)
    P_in = torch.arange(n, dtype=torch.int16, device=device).expand(B, n).contiguous()
    fidx = (torch.arange(B, device=device) % nf).to(torch.int32)
    return dict(n=n, F=nf, p=p, adj=adj, bits=bits, E=E, gain_off=goff, gains=gains, planes=planes,
                q=q, vel=vel, P_in=P_in, fidx=fidx)


def dense_gains_host(w, f):
    """Unpack formation f's edge planes into the reference's dense GainMat
    layout (row-major [3n][3n] numpy array), for the CPU baseline/oracle."""
    import numpy as np
    n = w["n"]
    adj = w["adj"][f].cpu().numpy()
    E = int(w["E"][f].item())
    off = int(w["gain_off"][f].item())
    NP = w.get("planes", 9)
    flat = w["gains"][NP * off: NP * off + NP * E]
    # 9: planes of E; 5: one record of 5 per edge
    planes = (flat.view(9, E) if NP == 9 else flat.view(E, 5).t()).cpu().numpy()
    ii, jj = np.nonzero(adj)
    G = np.zeros((3 * n, 3 * n))
    rc = [(r, c) for r in range(3) for c in range(3)] if NP == 9 else \
        [(0, 0), (0, 1), (1, 0), (1, 1), (2, 2)]
    for k, (r, c) in enumerate(rc):
        G[3 * ii + r, 3 * jj + c] = planes[k]
    return G
