"""Multi-GPU result gather (one process per GPU, torch.distributed).

Swarm instances are independent, so a solve exchanges nothing between GPUs
(SURVEY §8e). The only collective is the result gather of the north star:
the per-vehicle assignments and the 16-byte status records of every rank go
to rank 0 in one all_gather (RCCL over xGMI; gloo on CPU for tests), and the
convergence statistics -- flag counts, the fragile-margin count, a histogram
of the effective CBAA rounds -- are reduced with one all_reduce (plus one
for the maxima / minima).
"""
import torch
import torch.distributed as dist

# status record (include/aclswarm_amd.h acl_swarm_status_t):
# flags u32 | eff_rounds u16 | rounds u16 | n_invalid u16 | n_ca u16 | margin f32
STAT_KEYS = ("swarms", "valid", "agree", "changed", "nonfinite", "bad_input", "ca_active",
             "fragile", "invalid_vehicles", "ca_vehicles", "eff_rounds_sum")
FLAG_BITS = (0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40)
HIST_BINS = 64  # effective rounds 0..62, bin 63 = 63 or more


def swarm_stats(status_u8):
    """[B][16] uint8 status records -> (int64 counters [len(STAT_KEYS) +
    HIST_BINS]: the STAT_KEYS counts then the eff_rounds histogram;
    extrema f64 [2]: max eff_rounds, -(min margin)) on the device. GPU
    records: one launch of acl_swarm_stats; CPU records (the gloo tests):
    the same reduction in torch."""
    if status_u8.is_cuda:
        return _swarm_stats_native(status_u8)
    return swarm_stats_torch(status_u8)


def _swarm_stats_native(status_u8):
    from . import _lib
    st = status_u8.contiguous()
    dev = st.device
    counters = torch.empty(len(STAT_KEYS) + HIST_BINS, dtype=torch.int64, device=dev)
    ext = torch.empty(2, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rc = _lib.lib().acl_swarm_stats(st.data_ptr(), st.shape[0], counters.data_ptr(),
                                    ext.data_ptr(), stream)
    _lib.check(rc)
    return counters, ext


def swarm_stats_torch(status_u8):
    """The torch statement of acl_swarm_stats (CPU records, and the GPU
    test's reference)."""
    s = status_u8.to(torch.int64)
    flags = s[:, 0] | (s[:, 1] << 8) | (s[:, 2] << 16) | (s[:, 3] << 24)
    eff = s[:, 4] | (s[:, 5] << 8)
    ninv = s[:, 8] | (s[:, 9] << 8)
    nca = s[:, 10] | (s[:, 11] << 8)
    dev = s.device
    margin = (status_u8[:, 12:16].contiguous().view(torch.float32).reshape(-1)
              if status_u8.shape[0] else torch.empty(0, dtype=torch.float32, device=dev))
    c = [torch.tensor(s.shape[0], device=dev, dtype=torch.int64)]
    c += [((flags & bit) != 0).sum() for bit in FLAG_BITS]
    c += [ninv.sum(), nca.sum(), eff.sum()]
    # a fixed-size scatter (bincount sizes its output from the data: a host sync)
    hist = torch.zeros(HIST_BINS, dtype=torch.int64, device=dev)
    hist.scatter_add_(0, eff.clamp(max=HIST_BINS - 1), torch.ones_like(eff))
    counters = torch.cat([torch.stack(c), hist])
    if eff.numel():
        ext = torch.stack([eff.max().to(torch.float64), -margin.min().to(torch.float64)])
    else:
        ext = torch.tensor([0.0, -1.0], dtype=torch.float64, device=dev)
    return counters, ext


def gather_results(P_out, status_u8, group=None):
    """Gather P_out ([B][n] int16) and the status records of every rank to
    rank 0 and reduce the swarm statistics. Stays on the device (no host
    sync): returns (P_all, status_all -- None on non-zero ranks --, counters,
    extrema); turn the last two into a dict with stats_dict()."""
    counters, ext = swarm_stats(status_u8)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return P_out, status_u8, counters, ext
    world = dist.get_world_size(group)
    B = P_out.shape[0]
    # one all_gather of [B][2n + 16] bytes per rank (neither gloo nor RCCL
    # gathers int16 directly)
    src = torch.cat([P_out.contiguous().view(torch.uint8).reshape(B, -1),
                     status_u8.contiguous().reshape(B, 16)], 1)
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(ext, op=dist.ReduceOp.MAX, group=group)
    if dist.get_rank(group) != 0:
        return None, None, counters, ext
    allb = torch.cat(parts, 0)
    nb = 2 * P_out.shape[1]
    P_all = allb[:, :nb].contiguous().view(P_out.dtype).reshape(-1, P_out.shape[1])
    st_all = allb[:, nb:].contiguous()
    return P_all, st_all, counters, ext


def stats_dict(counters, ext):
    vals = counters.tolist()
    d = {k: int(v) for k, v in zip(STAT_KEYS, vals)}
    hist = vals[len(STAT_KEYS):]
    last = max((i for i, h in enumerate(hist) if h), default=0)
    d["eff_rounds_hist"] = [int(h) for h in hist[:last + 1]]
    e = ext.tolist()
    d["eff_rounds_max"] = int(e[0])
    d["margin_min"] = float(-e[1])
    return d
