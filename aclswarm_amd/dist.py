"""Multi-GPU result gather (one process per GPU, torch.distributed).

Swarm instances are independent, so a solve exchanges nothing between GPUs
(SURVEY §8e). The only collective is the result gather of the north star:
the per-vehicle assignments of every rank go to rank 0 (all_gather over RCCL
on xGMI; gloo on CPU for tests) and the convergence statistics are summed /
maxed with one all_reduce.
"""
import torch
import torch.distributed as dist

# status record: flags u32 | eff_rounds u16 | rounds u16 | n_invalid u16 | n_ca u16 | pad
STAT_KEYS = ("swarms", "valid", "agree", "changed", "nonfinite", "bad_input", "ca_active",
             "invalid_vehicles", "ca_vehicles", "eff_rounds_sum")


def swarm_stats(status_u8):
    """[B][16] uint8 status records -> int64 counter vector (device) and the
    max effective round count."""
    s = status_u8.to(torch.int64)
    flags = s[:, 0] | (s[:, 1] << 8) | (s[:, 2] << 16) | (s[:, 3] << 24)
    eff = s[:, 4] | (s[:, 5] << 8)
    ninv = s[:, 8] | (s[:, 9] << 8)
    nca = s[:, 10] | (s[:, 11] << 8)
    c = torch.stack([
        torch.tensor(s.shape[0], device=s.device, dtype=torch.int64),
        ((flags & 0x01) != 0).sum(), ((flags & 0x02) != 0).sum(),
        ((flags & 0x04) != 0).sum(), ((flags & 0x08) != 0).sum(),
        ((flags & 0x10) != 0).sum(), ((flags & 0x20) != 0).sum(),
        ninv.sum(), nca.sum(), eff.sum()])
    return c, eff.max() if eff.numel() else torch.zeros((), dtype=torch.int64, device=s.device)


def gather_results(P_out, status_u8, group=None):
    """Gather P_out ([B][n] int16) of every rank to rank 0 and reduce the
    swarm statistics. Stays on the device (no host sync): returns
    (P_all or None on non-zero ranks, counters, eff_max) as tensors; turn
    them into a dict with stats_dict()."""
    counters, eff_max = swarm_stats(status_u8)
    eff_max = eff_max.reshape(1).clone()
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return P_out, counters, eff_max
    world = dist.get_world_size(group)
    # as bytes: neither gloo nor RCCL reduces/gathers int16
    src = P_out.contiguous().view(torch.uint8)
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    parts = [x.view(P_out.dtype) for x in parts]
    dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(eff_max, op=dist.ReduceOp.MAX, group=group)
    P_all = torch.cat(parts, 0) if dist.get_rank(group) == 0 else None
    return P_all, counters, eff_max


def stats_dict(counters, eff_max):
    d = {k: int(v) for k, v in zip(STAT_KEYS, counters.tolist())}
    d["eff_rounds_max"] = int(eff_max.reshape(-1)[0].item())
    return d
