"""Host-side driver of the batched engine (device memory via torch tensors).

The C ABI (include/aclswarm_amd.h) takes raw device pointers; this module
packs the reference's formation data (points / adjmat / GainMat, the fields of
DistCntrl::Formation, aclswarm/include/aclswarm/distcntrl.h:26-34) into the
device layout and calls acl_solve_batch on the current torch stream.
"""
import ctypes as ct

import numpy as np
import torch

from . import _lib as L


def _ptr(t):
    return ct.c_void_p(t.data_ptr()) if t is not None else ct.c_void_p(0)


def gain_planes_host(adj, gains):
    """5 when every edge block of the GainMat has the ADMM structure (exact
    +0.0 at (0,2), (1,2), (2,0), (2,1)), else 9 (acl_gain_planes)."""
    lib = L.lib()
    n = np.asarray(adj).shape[0]
    adj_cm = np.ascontiguousarray(np.asarray(adj, dtype=np.uint8).T)
    g_cm = np.ascontiguousarray(np.asarray(gains, dtype=np.float64).T)
    return int(lib.acl_gain_planes(n, adj_cm.ctypes.data, g_cm.ctypes.data))


def pack_formation_host(points, adj, gains=None, planes=9):
    """One formation -> (p [n][3], adj bits [n][W] u64, gain planes
    [planes*E] f64, E).

    points [n][3]; adj [n][n] with adj[i][j] = adjmat(i,j); gains [3n][3n]
    with gains[r][c] = GainMat(r,c). Uses the ABI's packers, which take the
    reference's column-major Eigen layouts. planes = 9 (general blocks) or 5
    (ADMM-structured blocks, acl_formations_t::gain_planes).
    """
    lib = L.lib()
    points = np.ascontiguousarray(points, dtype=np.float64)
    n = points.shape[0]
    adj_cm = np.ascontiguousarray(np.asarray(adj, dtype=np.uint8).T)
    W = (n + 63) // 64
    bits = np.zeros((n, W), np.uint64)
    L.check(lib.acl_pack_adjacency(n, adj_cm.ctypes.data, bits.ctypes.data), "pack_adjacency")
    E = int(lib.acl_count_edges(n, adj_cm.ctypes.data))
    out = np.zeros(planes * E, np.float64)
    if gains is not None:
        g_cm = np.ascontiguousarray(np.asarray(gains, dtype=np.float64).T)
        L.check(lib.acl_pack_gains_planes(n, adj_cm.ctypes.data, g_cm.ctypes.data, planes,
                                          out.ctypes.data), "pack_gains_planes")
    return points, bits, out, E


class FormationTable:
    """Device formation table (acl_formations_t): F formations of n points,
    gains as `gain_planes` (9 or 5) edge planes per formation."""

    def __init__(self, n, p, adj_bits, gains, gain_off, gain_planes=9):
        self.n = int(n)
        self.p = p
        self.adj = adj_bits
        self.gains = gains
        self.gain_off = gain_off
        self.gain_planes = int(gain_planes)
        self.F = int(p.shape[0])
        self.gains_tiled = None

    def tile_gains(self, stream=None):
        """Formation-setup step: keep a tile-ordered copy of the 5-plane gain
        records (acl_tile_gains) for the pair kernel's contiguous tile reads."""
        if self.gain_planes != 5 or self.n > 128:
            return self
        out = torch.empty_like(self.gains)
        f = self.struct()
        if stream is None:
            stream = torch.cuda.current_stream(self.gains.device).cuda_stream
        L.check(L.lib().acl_tile_gains(ct.byref(f), out.data_ptr(), ct.c_void_p(stream)),
                "acl_tile_gains")
        self.gains_tiled = out
        return self

    @classmethod
    def from_host(cls, points, adjs, gains=None, device="cuda", planes=None):
        """planes=None picks 5 when every formation's GainMat has the ADMM
        block structure, else 9."""
        F = len(points)
        if planes is None:
            planes = 9
            if gains is not None and all(gain_planes_host(adjs[f], gains[f]) == 5
                                         for f in range(F)):
                planes = 5
        ps, bs, gs, offs = [], [], [], []
        off = 0
        for f in range(F):
            p, b, g, E = pack_formation_host(points[f], adjs[f],
                                             None if gains is None else gains[f], planes)
            ps.append(p); bs.append(b); gs.append(g); offs.append(off)
            off += E
        n = ps[0].shape[0]
        p = torch.from_numpy(np.stack(ps)).to(device)
        bits = torch.from_numpy(np.stack(bs).view(np.int64)).to(device)
        g = np.concatenate(gs) if gs else np.zeros(0)
        if g.size == 0:  # the ABI wants a valid pointer even with no edges
            g = np.zeros(9)
        g = torch.from_numpy(g).to(device)
        goff = torch.tensor(offs, dtype=torch.int64, device=device)
        return cls(n, p, bits, g, goff, planes)

    def struct(self):
        return L.Formations(self.n, self.F, self.p.data_ptr(), self.adj.data_ptr(),
                            self.gains.data_ptr(), self.gain_off.data_ptr(), self.gain_planes,
                            self.gains_tiled.data_ptr() if self.gains_tiled is not None else None)


_WS = {}
# per device: the (n, B) whose collision-list counters the cached workspace
# holds at zero ("all": freshly zero-filled). The counters' offset depends on
# n and B, so a call of another shape reuses their bytes for other data.
_WS_CLEAN = {}


def workspace(n, B, device):
    """Device workspace for acl_solve_batch / acl_control_batch (cached per
    device, grown on demand, zero-filled when allocated)."""
    need = int(L.lib().acl_solve_workspace_bytes(n, B))
    key = str(device)
    ws = _WS.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.zeros(max(need, 1), dtype=torch.uint8, device=device)
        _WS[key] = ws
        _WS_CLEAN[key] = "all"
    return ws


def _counters_zero(device, n, B):
    """acl_solve_args_t::ws_persistent applies: the cached workspace holds this
    shape's collision-list counters at zero (the last call that could touch
    them had this shape and left them zero, or the buffer is fresh)."""
    return _WS_CLEAN.get(str(device)) in ("all", (n, B))


def solve(table, fidx, q, vel, P_in, cntrl=None, safety=None, early_exit=True,
          do_control=True, want_who=False, want_align=False, want_gate_margin=False, out=None,
          stream=None, margin=True, P_rows=None, P_rows_on=None, persistent=True):
    """Run acl_solve_batch for B = q.shape[0] swarms. All tensors on device.

    margin=False sets acl_solve_args_t::skip_margin: the status margin is -1
    and FRAGILE is never set; everything else is unchanged. persistent=False
    clears acl_solve_args_t::ws_persistent (the call memsets the collision-
    list counters itself; the outputs are the same).

    P_rows [B][n][n] int16 (uint16 bits) and P_rows_on [B] uint8
    (acl_solve_args_t::P_rows): a swarm with P_rows_on[b] != 0 runs its
    auction from each vehicle's own assignment, row v = vehicle v's table
    (formation point -> vehicle) with P_in[b][v] its point in it.

    fidx [B] int32, q/vel [B][n][3] f64, P_in [B][n] int16 (uint16 bits).
    Returns a dict of device tensors: P_out, status (raw 16-byte records as
    uint8 [B][16]), u, u_safe, ca_flag, and if requested who, align_Rt,
    gate_margin [B] f64.
    """
    lib = L.lib()
    B, n = int(q.shape[0]), table.n
    dev = q.device
    if out is None:
        out = {
            "P_out": torch.empty((B, n), dtype=torch.int16, device=dev),
            "status": torch.empty((B, 16), dtype=torch.uint8, device=dev),
            "u": torch.empty((B, n, 3), dtype=torch.float64, device=dev),
            "u_safe": torch.empty((B, n, 3), dtype=torch.float64, device=dev),
            "ca_flag": torch.empty((B, n), dtype=torch.uint8, device=dev),
        }
        if want_who:
            out["who"] = torch.empty((B, n, n), dtype=torch.int16, device=dev)
        if want_align:
            out["align_Rt"] = torch.empty((B, n, 6), dtype=torch.float64, device=dev)
        if want_gate_margin:
            out["gate_margin"] = torch.empty(B, dtype=torch.float64, device=dev)
    a = L.SolveArgs()
    a.B = B
    a.fidx = fidx.data_ptr(); a.q = q.data_ptr(); a.vel = vel.data_ptr()
    a.P_in = P_in.data_ptr(); a.P_out = out["P_out"].data_ptr()
    a.status = out["status"].data_ptr()
    a.u = out["u"].data_ptr() if out.get("u") is not None else None
    a.u_safe = out["u_safe"].data_ptr() if out.get("u_safe") is not None else None
    a.ca_flag = out["ca_flag"].data_ptr() if out.get("ca_flag") is not None else None
    a.who = out["who"].data_ptr() if out.get("who") is not None else None
    a.align_Rt = out["align_Rt"].data_ptr() if out.get("align_Rt") is not None else None
    a.gate_margin = (out["gate_margin"].data_ptr() if out.get("gate_margin") is not None
                     else None)
    a.workspace = workspace(n, B, dev).data_ptr()
    a.cntrl = cntrl or L.default_gains()
    a.safety = safety or L.default_safety()
    a.early_exit = int(bool(early_exit))
    a.do_control = int(bool(do_control))
    a.skip_margin = 0 if margin else 1
    # the call's memset of the collision-list counters only when the cached
    # workspace does not hold them at zero for this shape (ABI 10)
    clean = _counters_zero(dev, n, B)
    a.ws_persistent = 1 if (persistent and clean) else 0
    if P_rows is not None:
        if P_rows_on is None or P_rows.shape != (B, n, n) or P_rows_on.shape != (B,):
            raise ValueError("P_rows [B][n][n] needs P_rows_on [B]")
        # the kernels read raw row-major u16 / u8 memory on q's device
        if P_rows.dtype not in (torch.int16, torch.uint16) or \
                P_rows_on.dtype not in (torch.uint8, torch.bool):
            raise ValueError("P_rows must be int16 (u16 bits) and P_rows_on uint8/bool")
        if not (P_rows.is_contiguous() and P_rows_on.is_contiguous()):
            raise ValueError("P_rows and P_rows_on must be contiguous")
        if P_rows.device != q.device or P_rows_on.device != q.device:
            raise ValueError("P_rows and P_rows_on must be on q's device")
        a.P_rows = P_rows.data_ptr()
        a.P_rows_on = P_rows_on.data_ptr()
    F = table.struct()
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    _WS_CLEAN[str(dev)] = None  # (until the call has been enqueued)
    L.check(lib.acl_solve_batch(ct.byref(F), ct.byref(a), ct.c_void_p(stream)), "acl_solve_batch")
    # with control the collision-avoidance launch left this shape's counters
    # zero; an auction-only call leaves them as they were (other shapes' bytes
    # may now hold its data)
    _WS_CLEAN[str(dev)] = (n, B) if (do_control or clean) else None
    return out


def status_to_numpy(status_u8):
    """[B][16] uint8 device/host tensor -> structured numpy array."""
    arr = status_u8.detach().cpu().numpy()
    return np.ascontiguousarray(arr).view(L.STATUS_DTYPE).reshape(-1)


ADMM_BASIS_LINPACK, ADMM_BASIS_COMPLEX = 0, 1   # acl_admm_params_t.basis


def admm_design(pts, adj, params=None, stream=None, basis=None):
    """Batched ADMM formation-gain design (acl_admm_solve_batch; the
    reference's admm::Solver::solve / ADMM::calculateFormationGains,
    aclswarm/lib/admm/src/solver.cpp:28-79, aclswarm/src/admm.cpp:32-51).

    pts [F][n][3] f64 and adj [F][n][n] f64 (0/1, symmetric) on the device.
    Returns (gains [F][3n][3n] f64 with gains[f][r][c] = GainMat(r, c),
    iters [F][2] int32: ADMM iterations of the xy and z designs; a PSD
    projection the sign iteration does not resolve is made by the Jacobi
    eigensolver fallback). basis overrides params.basis: ADMM_BASIS_LINPACK
    (default, the codegen's gains) or ADMM_BASIS_COMPLEX (the complex-
    structured complement basis admm::Solver's tests need, test_admm.cpp:84-187).
    """
    lib = L.lib()
    F, n = int(pts.shape[0]), int(pts.shape[1])
    dev = pts.device
    pts = pts.contiguous()          # [n][3] row-major == Eigen 3 x n column-major
    adj = adj.contiguous()          # symmetric: either layout
    out = torch.empty((F, 3 * n, 3 * n), dtype=torch.float64, device=dev)
    iters = torch.empty((F, 2), dtype=torch.int32, device=dev)
    prm = params or L.default_admm_params()
    if basis is not None:
        prm.basis = int(basis)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    L.check(lib.acl_admm_solve_batch(F, n, pts.data_ptr(), adj.data_ptr(), out.data_ptr(),
                                     iters.data_ptr(), ct.byref(prm), ct.c_void_p(stream)),
            "acl_admm_solve_batch")
    return out.transpose(1, 2), iters


def control(table, fidx, q, vel, P, cntrl=None, safety=None, want_gate_margin=False,
            stream=None):
    """acl_control_batch: DistCntrl::compute + Safety for B swarms with given
    assignments P [B][n] (int16 holding uint16 bits). Returns u, u_safe,
    ca_flag, status and, if requested (as in solve), gate_margin [B] f64
    (device tensors)."""
    lib = L.lib()
    B, n = int(q.shape[0]), table.n
    dev = q.device
    out = {
        "u": torch.empty((B, n, 3), dtype=torch.float64, device=dev),
        "u_safe": torch.empty((B, n, 3), dtype=torch.float64, device=dev),
        "ca_flag": torch.empty((B, n), dtype=torch.uint8, device=dev),
        "status": torch.empty((B, 16), dtype=torch.uint8, device=dev),
    }
    if want_gate_margin:
        out["gate_margin"] = torch.empty(B, dtype=torch.float64, device=dev)
    a = L.ControlArgs()
    a.B = B
    a.fidx = fidx.data_ptr(); a.q = q.data_ptr(); a.vel = vel.data_ptr(); a.P = P.data_ptr()
    a.u = out["u"].data_ptr(); a.u_safe = out["u_safe"].data_ptr()
    a.ca_flag = out["ca_flag"].data_ptr(); a.status = out["status"].data_ptr()
    a.gate_margin = out["gate_margin"].data_ptr() if want_gate_margin else None
    a.workspace = workspace(n, B, dev).data_ptr()
    a.cntrl = cntrl or L.default_gains()
    a.safety = safety or L.default_safety()
    F = table.struct()
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    _WS_CLEAN[str(dev)] = None
    L.check(lib.acl_control_batch(ct.byref(F), ct.byref(a), ct.c_void_p(stream)),
            "acl_control_batch")
    _WS_CLEAN[str(dev)] = (n, B)  # (it zeroes the counters first; its CA launch leaves them zero)
    return out


def hungarian(table, fidx, q, P_last=None, P_cmp=None, want_Rt=False, stream=None):
    """acl_hungarian_batch: the reference's centralized comparator
    (assignment.py:94-137 find_optimal_assignment) for B swarms. P_last /
    P_cmp [B][n] int16 holding uint16 bits (None = identity / not priced).
    Returns P_opt [B][n] int16, cost [B][2] f64, status [B] i32 and, with
    want_Rt, align_Rt [B][4] (device tensors)."""
    lib = L.lib()
    B, n = int(q.shape[0]), table.n
    dev = q.device
    out = {
        "P_opt": torch.empty((B, n), dtype=torch.int16, device=dev),
        "cost": torch.empty((B, 2), dtype=torch.float64, device=dev),
        "status": torch.empty((B,), dtype=torch.int32, device=dev),
    }
    if want_Rt:
        out["align_Rt"] = torch.empty((B, 4), dtype=torch.float64, device=dev)
    a = L.HungarianArgs()
    a.B = B
    a.fidx = fidx.data_ptr(); a.q = q.data_ptr()
    a.P_last = P_last.data_ptr() if P_last is not None else None
    a.P_cmp = P_cmp.data_ptr() if P_cmp is not None else None
    a.P_opt = out["P_opt"].data_ptr(); a.cost = out["cost"].data_ptr()
    a.align_Rt = out["align_Rt"].data_ptr() if want_Rt else None
    a.status = out["status"].data_ptr()
    F = table.struct()
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    L.check(lib.acl_hungarian_batch(ct.byref(F), ct.byref(a), ct.c_void_p(stream)),
            "acl_hungarian_batch")
    return out


def cbaa_step(table, fidx, vehid, q, Rt, start, price, who, cand_off, cand_vehid=None,
              cand_price=None, cand_who=None, stream=None):
    """acl_cbaa_step_batch (ABI 11): one CBAA bid iteration for each of V
    vehicles -- the START bid (start[k] = 1) or updateTaskAssignment over its
    candidates then selectTaskAssignment when outbid (auctioneer.cpp:182-306,
    469-542). Device tensors: fidx / vehid [V] i32, q [V][3] f64, Rt [V][6]
    f64, start [V] u8, price [V][n] f32 and who [V][n] i32 (updated in
    place), cand_off [V + 1] i32, cand_vehid [K] i32, cand_price [K][n] f32,
    cand_who [K][n] i32. Returns (task [V] i32, flags [V] i32)."""
    lib = L.lib()
    V = int(vehid.shape[0])
    dev = vehid.device
    n = table.n
    want = {"fidx": (fidx, torch.int32, (V,)), "vehid": (vehid, torch.int32, (V,)),
            "q": (q, torch.float64, (V, 3)), "Rt": (Rt, torch.float64, (V, 6)),
            "start": (start, torch.uint8, (V,)), "price": (price, torch.float32, (V, n)),
            "who": (who, torch.int32, (V, n)), "cand_off": (cand_off, torch.int32, (V + 1,))}
    K = None
    for name, t in (("cand_vehid", cand_vehid), ("cand_price", cand_price), ("cand_who", cand_who)):
        if t is not None:
            K = int(t.shape[0])
    if K is not None:
        want["cand_vehid"] = (cand_vehid, torch.int32, (K,))
        want["cand_price"] = (cand_price, torch.float32, (K, n))
        want["cand_who"] = (cand_who, torch.int32, (K, n))
    for name, (t, dt, shape) in want.items():
        if t is None or t.dtype != dt or tuple(t.shape) != shape or not t.is_contiguous() \
                or t.device != dev:
            raise ValueError(f"cbaa_step: {name} must be a contiguous {dt} tensor of shape "
                             f"{shape} on {dev}")
    task = torch.empty((V,), dtype=torch.int32, device=dev)
    flags = torch.empty((V,), dtype=torch.int32, device=dev)
    a = L.CbaaStepArgs()
    a.V = V
    a.K = K if K is not None else 0
    a.fidx = fidx.data_ptr(); a.vehid = vehid.data_ptr(); a.q = q.data_ptr()
    a.Rt = Rt.data_ptr(); a.start = start.data_ptr(); a.price = price.data_ptr()
    a.who = who.data_ptr(); a.cand_off = cand_off.data_ptr()
    a.cand_vehid = cand_vehid.data_ptr() if cand_vehid is not None else None
    a.cand_price = cand_price.data_ptr() if cand_price is not None else None
    a.cand_who = cand_who.data_ptr() if cand_who is not None else None
    a.task = task.data_ptr(); a.flags = flags.data_ptr()
    F = table.struct()
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    L.check(lib.acl_cbaa_step_batch(ct.byref(F), ct.byref(a), ct.c_void_p(stream)),
            "acl_cbaa_step_batch")
    return task, flags


def write_assignment_log(path, q, adj, lastP, p, align_Rt, P):
    """Auctioneer::logAssignment's binary record (auctioneer.cpp:577-597),
    host arrays: q, p [n][3]; adj [n][n] (adj[i][j] = adjmat(i,j)); lastP, P
    [n]; align_Rt [6] (the logging vehicle's alignment)."""
    lib = L.lib()
    q = np.ascontiguousarray(q, np.float64)
    p = np.ascontiguousarray(p, np.float64)
    adj_cm = np.ascontiguousarray(np.asarray(adj, np.uint8).T)
    lastP = np.ascontiguousarray(lastP, np.uint16)
    P = np.ascontiguousarray(P, np.uint16)
    Rt = np.ascontiguousarray(align_Rt, np.float64)
    L.check(lib.acl_write_assignment_log(str(path).encode(), q.shape[0], q.ctypes.data,
                                         adj_cm.ctypes.data, lastP.ctypes.data, p.ctypes.data,
                                         Rt.ctypes.data, P.ctypes.data), "write_assignment_log")


def read_assignment_log(path):
    """Reads a logAssignment record: dict of q, adj, lastP, p, aligned, P."""
    lib = L.lib()
    n = ct.c_int32(0)
    L.check(lib.acl_read_assignment_log(str(path).encode(), ct.byref(n), None, None, None,
                                        None, None, None), "read_assignment_log")
    n = n.value
    r = {"q": np.zeros((n, 3)), "adj_cm": np.zeros((n, n), np.uint8),
         "lastP": np.zeros(n, np.uint16), "p": np.zeros((n, 3)),
         "aligned": np.zeros((n, 3)), "P": np.zeros(n, np.uint16)}
    nn = ct.c_int32(0)
    L.check(lib.acl_read_assignment_log(str(path).encode(), ct.byref(nn), r["q"].ctypes.data,
                                        r["adj_cm"].ctypes.data, r["lastP"].ctypes.data,
                                        r["p"].ctypes.data, r["aligned"].ctypes.data,
                                        r["P"].ctypes.data), "read_assignment_log")
    r["adj"] = r.pop("adj_cm").T.copy()
    return r


class Episode:
    """Closed-loop batched episodes (acl_episode_batch):
    the per-swarm state that persists across calls -- positions, velocities,
    carried assignment, the flush flag, the supervisor's ring buffers and the
    episode counters -- so an episode can be flown in chunks of steps.

    fidx [B] int32, q/vel [B][n][3] f64, P [B][n] int16 (uint16 bits), all on
    the device; they are copied, the caller's tensors are not modified.
    """

    def __init__(self, table, fidx, q, vel, P, params=None, cntrl=None, safety=None):
        dev = q.device
        self.table = table
        self.B, self.n = int(q.shape[0]), table.n
        self.ep = params or L.default_episode_params()
        self.cntrl = cntrl or L.default_gains()
        self.safety = safety or L.default_safety()
        self.fidx = fidx.contiguous()
        self.q = q.clone().contiguous()
        self.vel = vel.clone().contiguous()
        self.P = P.clone().contiguous()
        self.flush = torch.zeros(self.B, dtype=torch.uint8, device=dev)
        est = np.zeros(self.B, L.EPISODE_STATUS_DTYPE)
        est["converged_step"] = -1  # zeroed otherwise (pending_step 0: none)
        est["gridlock_step"] = -1
        self.est = torch.from_numpy(est.view(np.uint8).reshape(self.B, -1).copy()).to(dev)
        Lb = int(self.ep.bufflen)
        self.ring_u = torch.zeros((self.B, Lb, self.n), dtype=torch.float64, device=dev)
        self.ring_ca = torch.zeros((self.B, Lb, self.n), dtype=torch.uint8, device=dev)
        need = int(L.lib().acl_episode_workspace_bytes(self.n, self.B))
        self.ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        self.step = 0

    def run(self, steps, history=False, stream=None):
        """Fly `steps` control periods. With history=True returns per-step
        device tensors q/vel/u [steps][B][n][3], ca [steps][B][n],
        P [steps][B][n] (int16); else None."""
        dev = self.q.device
        B, n = self.B, self.n
        hist = None
        if history:
            hist = {
                "q": torch.empty((steps, B, n, 3), dtype=torch.float64, device=dev),
                "vel": torch.empty((steps, B, n, 3), dtype=torch.float64, device=dev),
                "u": torch.empty((steps, B, n, 3), dtype=torch.float64, device=dev),
                "ca": torch.empty((steps, B, n), dtype=torch.uint8, device=dev),
                "P": torch.empty((steps, B, n), dtype=torch.int16, device=dev),
            }
        a = L.EpisodeArgs()
        a.B = B
        a.fidx = self.fidx.data_ptr(); a.q = self.q.data_ptr(); a.vel = self.vel.data_ptr()
        a.P = self.P.data_ptr(); a.flush = self.flush.data_ptr(); a.est = self.est.data_ptr()
        a.ring_u = self.ring_u.data_ptr(); a.ring_ca = self.ring_ca.data_ptr()
        a.step0 = self.step; a.steps = steps
        if hist is not None:
            a.q_hist = hist["q"].data_ptr(); a.vel_hist = hist["vel"].data_ptr()
            a.u_hist = hist["u"].data_ptr(); a.ca_hist = hist["ca"].data_ptr()
            a.P_hist = hist["P"].data_ptr()
        a.workspace = self.ws.data_ptr()
        a.cntrl = self.cntrl; a.safety = self.safety; a.ep = self.ep
        F = self.table.struct()
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        L.check(L.lib().acl_episode_batch(ct.byref(F), ct.byref(a), ct.c_void_p(stream)),
                "acl_episode_batch")
        self.step += steps
        return hist

    def status(self):
        """Episode counters as a structured numpy array [B]."""
        arr = np.ascontiguousarray(self.est.cpu().numpy())
        return arr.view(L.EPISODE_STATUS_DTYPE).reshape(-1)


class Trial:
    """Batched Monte-Carlo trials (acl_trial_batch; supervisor.py over the
    closed loop): each swarm flies its formation sequence fseq[b] through the
    supervisor's state machine and keeps its per-trial record. State persists
    across calls (a trial can be run in chunks of steps).

    fseq [B][K] int32, q/vel [B][n][3] f64 on the device (copied). The
    assignment starts at identity (no formation yet)."""

    def __init__(self, table, fseq, q, vel, params=None, cntrl=None, safety=None):
        dev = q.device
        self.table = table
        self.B, self.n = int(q.shape[0]), table.n
        self.K = int(fseq.shape[1])
        self.tp = params or L.default_trial_params()
        self.cntrl = cntrl or L.default_gains()
        self.safety = safety or L.default_safety()
        B, n, K = self.B, self.n, self.K
        Lb = int(self.tp.ep.bufflen)
        self.fseq = fseq.to(torch.int32).contiguous()
        if tuple(self.fseq.shape) != (B, K):
            raise ValueError("Trial: fseq must be [B][K]")
        self.fidx = torch.empty(B, dtype=torch.int32, device=dev)
        self.q = q.clone().contiguous()
        self.vel = vel.clone().contiguous()
        self.P = torch.empty((B, n), dtype=torch.int16, device=dev)
        self.flush = torch.empty(B, dtype=torch.uint8, device=dev)
        self.ts = torch.empty((B, L.TRIAL_STATUS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        self.ctl_on = torch.empty((B, n), dtype=torch.uint8, device=dev)
        self.ring_u = torch.empty((B, Lb, n), dtype=torch.float64, device=dev)
        self.ring_ca = torch.empty((B, Lb, n), dtype=torch.uint8, device=dev)
        self.posf = torch.empty((B, 2, n), dtype=torch.float64, device=dev)
        self.dist = torch.empty((B, n), dtype=torch.float64, device=dev)
        self.t_conv = torch.empty((B, K), dtype=torch.float64, device=dev)
        self.t_avoid = torch.empty((B, K), dtype=torch.float64, device=dev)
        self.n_assign = torch.empty((B, K), dtype=torch.int32, device=dev)
        need = int(L.lib().acl_trial_workspace_bytes(n, B))
        self.ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        self.step = 0
        a = self._args(0)
        L.check(L.lib().acl_trial_init(ct.byref(a), n, ct.c_void_p(
            torch.cuda.current_stream(dev).cuda_stream)), "acl_trial_init")

    def _args(self, steps, hist=None):
        a = L.TrialArgs()
        a.B, a.K = self.B, self.K
        for k in ("fseq", "fidx", "q", "vel", "P", "flush", "ts", "ctl_on", "ring_u", "ring_ca",
                  "posf", "dist", "t_conv", "t_avoid", "n_assign"):
            setattr(a, k, getattr(self, k).data_ptr())
        a.step0, a.steps = self.step, steps
        if hist is not None:
            for k, f in (("q", "q_hist"), ("vel", "vel_hist"), ("u", "u_hist"), ("ca", "ca_hist"),
                         ("ctl", "ctl_hist"), ("P", "P_hist"), ("state", "state_hist")):
                setattr(a, f, hist[k].data_ptr())
        a.workspace = self.ws.data_ptr()
        a.cntrl, a.safety, a.tp = self.cntrl, self.safety, self.tp
        return a

    def run(self, steps, history=False, stream=None):
        """Advance every trial `steps` control periods. With history=True
        returns per-step device tensors q/vel/u [steps][B][n][3] (u: 0 for
        stopped controllers), ca/ctl [steps][B][n], P [steps][B][n] (int16),
        state [steps][B]; else None."""
        dev = self.q.device
        B, n = self.B, self.n
        hist = None
        if history:
            f64 = dict(dtype=torch.float64, device=dev)
            hist = {"q": torch.empty((steps, B, n, 3), **f64),
                    "vel": torch.empty((steps, B, n, 3), **f64),
                    "u": torch.empty((steps, B, n, 3), **f64),
                    "ca": torch.empty((steps, B, n), dtype=torch.uint8, device=dev),
                    "ctl": torch.empty((steps, B, n), dtype=torch.uint8, device=dev),
                    "P": torch.empty((steps, B, n), dtype=torch.int16, device=dev),
                    "state": torch.empty((steps, B), dtype=torch.int32, device=dev)}
        a = self._args(steps, hist)
        F = self.table.struct()
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        L.check(L.lib().acl_trial_batch(ct.byref(F), ct.byref(a), ct.c_void_p(stream)),
                "acl_trial_batch")
        self.step += steps
        return hist

    def status(self):
        """Per-trial supervisor state and counters, structured numpy [B]."""
        arr = np.ascontiguousarray(self.ts.cpu().numpy())
        return arr.view(L.TRIAL_STATUS_DTYPE).reshape(-1)

    def records(self):
        """The supervisor's per-trial record (the CSV row of complete(),
        supervisor.py:404-415) as numpy arrays: dist [B][n], time [B][K],
        time_avoidance [B][K], assignments [B][K], plus state / done_step."""
        st = self.status()
        return {"dist": self.dist.cpu().numpy(), "time": self.t_conv.cpu().numpy(),
                "time_avoidance": self.t_avoid.cpu().numpy(),
                "assignments": self.n_assign.cpu().numpy(),
                "state": st["state"].copy(), "last_state": st["last_state"].copy(),
                "done_step": st["done_step"].copy()}


def generate_formation_groups(seeds, n, fc, l, w, h, min_dist=2.0, max_candidates=0,
                              stream=None):
    """acl_generate_formation_groups: the reference's
    generate_formation_group (generate_random_formation.py:59-80) after
    np.random.seed(seed), for every seed at once on the device.

    seeds: [F] int tensor on the device (taken as uint32). Returns a dict of
    device tensors: points [F][2][n][3] f64, adj [F][n][n] u8, status [F]
    int32, drawn [F] int64 (32-bit outputs consumed)."""
    dev = seeds.device
    F = int(seeds.shape[0])
    s32 = (seeds.to(torch.int64) & 0xFFFFFFFF).to(torch.int32).contiguous()  # uint32 bits
    out = {
        "points": torch.empty((F, 2, n, 3), dtype=torch.float64, device=dev),
        "adj": torch.empty((F, n, n), dtype=torch.uint8, device=dev),
        "status": torch.empty(F, dtype=torch.int32, device=dev),
        "drawn": torch.empty(F, dtype=torch.int64, device=dev),
    }
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    L.check(L.lib().acl_generate_formation_groups(
        F, n, s32.data_ptr(), int(bool(fc)), float(l), float(w), float(h), float(min_dist),
        int(max_candidates), out["points"].data_ptr(), out["adj"].data_ptr(),
        out["status"].data_ptr(), out["drawn"].data_ptr(), ct.c_void_p(stream)),
        "acl_generate_formation_groups")
    return out
