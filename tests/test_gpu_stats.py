"""acl_swarm_stats (the per-solve convergence counters of SURVEY §8e) on the
GPU against its torch statement in aclswarm_amd/dist.py, bit for bit: one
workgroup writing the outputs itself (B <= 16 384) and the multi-workgroup
atomics (B > 16 384)."""
import numpy as np
import pytest
import torch

from aclswarm_amd import dist as D

pytestmark = pytest.mark.gpu


def _records(rng, B):
    st = np.zeros((B, 16), np.uint8)
    flags = rng.randint(0, 128, size=B).astype(np.uint32)
    eff = rng.choice([0, 1, 5, 9, 14, 62, 63, 64, 200, 65535], size=B).astype(np.uint16)
    margin = rng.choice([0.0, 1.0, 3e-7, 0.25, 1e-3], size=B)
    margin = np.where(rng.rand(B) < 0.5, rng.rand(B), margin).astype(np.float32)
    st[:, 0:4] = flags.view(np.uint8).reshape(B, 4)
    st[:, 4:6] = eff.view(np.uint8).reshape(B, 2)
    st[:, 6:8] = np.full(B, 200, np.uint16).view(np.uint8).reshape(B, 2)
    st[:, 8:10] = rng.randint(0, 300, size=B).astype(np.uint16).view(np.uint8).reshape(B, 2)
    st[:, 10:12] = rng.randint(0, 300, size=B).astype(np.uint16).view(np.uint8).reshape(B, 2)
    st[:, 12:16] = margin.view(np.uint8).reshape(B, 4)
    return st


@pytest.mark.parametrize("B", [0, 1, 1000, 4096, 16384, 16385, 70001])
def test_stats_native_matches_torch(B):
    rng = np.random.RandomState(B)
    st = torch.from_numpy(_records(rng, B))
    c_ref, e_ref = D.swarm_stats_torch(st)
    c, e = D.swarm_stats(st.cuda())
    torch.cuda.synchronize()
    assert torch.equal(c.cpu(), c_ref)
    assert torch.equal(e.cpu(), e_ref)


def test_stats_of_a_solve():
    """The counters of a real batch (generator swarms, n = 20)."""
    from aclswarm_amd import engine, workload
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    w = workload.simform_workload(512, 20, gen, dev, L=15.0, complete=True)
    T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"], w["planes"])
    out = engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"])
    c, e = D.swarm_stats(out["status"])
    c_ref, e_ref = D.swarm_stats_torch(out["status"].cpu())
    assert torch.equal(c.cpu(), c_ref) and torch.equal(e.cpu(), e_ref)
    d = D.stats_dict(c, e)
    assert d["swarms"] == 512 and d["valid"] == 512
