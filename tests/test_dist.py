"""Multi-process (world_size 2, gloo, CPU) coverage of the result gather used
by bench.py --gpus N: each rank owns a contiguous shard of swarms; rank 0
receives every rank's assignments and the summed statistics."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _status(B, rank):
    st = np.zeros(B, dtype=[("flags", "<u4"), ("eff_rounds", "<u2"), ("rounds", "<u2"),
                            ("n_invalid", "<u2"), ("n_ca", "<u2"), ("margin", "<f4")])
    st["flags"] = 0x03
    st["flags"][0] |= 0x04
    st["flags"][1] = 0x10 if rank == 1 else 0x03
    st["eff_rounds"] = np.arange(B) + 10 * rank
    st["rounds"] = 200
    st["n_ca"] = rank + 1
    st["margin"] = 0.5
    st["margin"][2] = 1e-7 if rank == 1 else 0.25   # one fragile swarm
    st["flags"][2] |= 0x40 if rank == 1 else 0
    return torch.from_numpy(st.view(np.uint8).reshape(B, 16).copy())


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from aclswarm_amd import dist as D
    B, n = 5, 7
    P = torch.full((B, n), rank, dtype=torch.int16)
    P_all, st_all, counters, em = D.gather_results(P, _status(B, rank))
    stats = D.stats_dict(counters, em)
    if rank == 0:
        q.put((P_all.numpy().tolist(), st_all.numpy().tolist(), stats))
    else:
        assert P_all is None and st_all is None
    dist.barrier()
    dist.destroy_process_group()


def test_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    P_all, st_all, stats = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    P_all = np.array(P_all)
    assert P_all.shape == (10, 7)
    assert (P_all[:5] == 0).all() and (P_all[5:] == 1).all()
    assert stats["swarms"] == 10
    assert stats["bad_input"] == 1
    assert stats["valid"] == 9
    assert stats["changed"] == 2
    assert stats["ca_vehicles"] == 5 * 1 + 5 * 2
    assert stats["eff_rounds_max"] == 14
    assert stats["eff_rounds_sum"] == sum(range(5)) + sum(range(10, 15))
    # the status records travel with the assignments, in rank order
    st = np.array(st_all, np.uint8).view(np.dtype([("flags", "<u4"), ("eff_rounds", "<u2"),
                                                    ("rounds", "<u2"), ("n_invalid", "<u2"),
                                                    ("n_ca", "<u2"), ("margin", "<f4")]))
    np.testing.assert_array_equal(st["eff_rounds"].ravel(), list(range(5)) + list(range(10, 15)))
    assert stats["fragile"] == 1
    assert abs(stats["margin_min"] - 1e-7) < 1e-12
    hist = stats["eff_rounds_hist"]
    assert sum(hist) == 10 and hist[0] == 1 and hist[14] == 1 and len(hist) == 15


def test_single_process_passthrough():
    from aclswarm_amd import dist as D
    P = torch.zeros((3, 4), dtype=torch.int16)
    P_all, st_all, c, em = D.gather_results(P, _status(3, 0))
    assert P_all is P
    assert D.stats_dict(c, em)["swarms"] == 3
