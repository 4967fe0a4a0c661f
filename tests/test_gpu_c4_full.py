"""Config C4 at its per-GPU shard (simform500 noncomplete, L=90,
B = 16 384 over 8 GPUs = 2 048 swarms per GPU, a unique formation per swarm
from the reference generator reproduced on the device) -- `bench.py --config
c4`'s own workload. Every swarm is checked for what the path guarantees (a
valid permutation adopted by all vehicles, finite commands, counters
consistent); 16 swarms spread over the shard against the CPU restatement
(assignments, status, margin bit-exact; commands within 1e-5 relative)."""
import numpy as np
import pytest
import torch

from aclswarm_amd import dist as D
from aclswarm_amd import engine, workload
from test_gpu_c3_full import _sample_check

pytestmark = pytest.mark.gpu
B, N = 2048, 500


@pytest.fixture(scope="module")
def c4():
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(2024)
    w = workload.simform_workload(B, N, gen, dev, L=90.0, complete=False, planes=5, seed0=0)
    T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"], w["planes"])
    return w, T


def test_c4_full_shard(c4):
    w, T = c4
    out = engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"])
    torch.cuda.synchronize()
    P = out["P_out"].to(torch.int64)
    srt, _ = torch.sort(P, dim=1)
    assert torch.equal(srt, torch.arange(N, device=P.device).expand_as(srt))
    assert bool(torch.isfinite(out["u"]).all()) and bool(torch.isfinite(out["u_safe"]).all())
    d = D.stats_dict(*D.swarm_stats(out["status"]))
    assert d["swarms"] == B and d["bad_input"] == 0 and d["nonfinite"] == 0
    assert d["valid"] == B and d["agree"] == B
    # a second run of the whole shard is bit-identical
    again = engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"])
    torch.cuda.synchronize()
    for k in ("P_out", "status", "u", "u_safe", "ca_flag"):
        assert torch.equal(out[k], again[k]), k
    rng = np.random.RandomState(2048)
    idx = np.sort(np.concatenate([[0, B - 1], rng.choice(np.arange(1, B - 1), 14, replace=False)]))
    _sample_check(w, out, idx)
