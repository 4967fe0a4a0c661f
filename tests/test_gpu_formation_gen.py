"""GPU parity of the device formation-group generator
(acl_generate_formation_groups): bit-exact against the
reference generator's own outputs (tests/golden/simform*.npz) and against
the CPU restatement (oracle/formation_gen_oracle.py, itself pinned to numpy's
RandomState in tests/test_formation_gen.py), including the number of 32-bit
outputs each group consumed."""
import os

import numpy as np
import pytest

import formation_gen_oracle as G

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen(seeds, n, fc, l, w, h, md=2.0, maxc=0):
    import torch
    from aclswarm_amd import engine
    s = torch.tensor(np.asarray(seeds, np.int64), device="cuda:0")
    out = engine.generate_formation_groups(s, n, fc, l, w, h, md, maxc)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("name", ["simform20_fc", "simform20_nc", "simform100_nc", "simform500_nc"])
def test_generator_matches_reference_fixtures(cuda, name):
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    n, fc, L, h, md = int(d["n"]), bool(d["fc"]), float(d["L"]), float(d["h"]), float(d["min_dist"])
    r = _gen(d["seeds"], n, fc, L, L, h, md)
    assert (r["status"] == 0).all()
    assert (r["adj"] == d["adjmat"]).all()
    assert (r["points"] == d["points"]).all()


@pytest.mark.parametrize("n,fc,L,count", [(20, False, 15.0, 48), (20, True, 15.0, 16),
                                          (100, False, 40.0, 12), (5, False, 6.0, 16),
                                          (64, False, 30.0, 8)])
def test_generator_matches_cpu_restatement(cuda, n, fc, L, count):
    seeds = [int(x) for x in np.random.RandomState(n + count).randint(0, 2 ** 32 - 1, count,
                                                                       dtype=np.int64)]
    r = _gen(seeds, n, fc, L, L, 2.0)
    for g, s in enumerate(seeds):
        adj, forms, drawn = G.generate_formation_group(s, n, fc, L, L, 2.0, 2.0)
        assert r["status"][g] == 0
        assert (r["adj"][g] == np.array(adj, np.uint8)).all(), s
        for k in range(2):
            assert (r["points"][g, k] == np.array(forms[k])).all(), (s, k)
        assert r["drawn"][g] == drawn, s


def test_generator_reports_infeasible_groups(cuda):
    # 3 points at pairwise distance >= 2 cannot fit in a 1 x 1 box
    r = _gen([1, 2], 3, True, 1.0, 1.0, 1.0, 2.0, maxc=5000)
    assert (r["status"] == 1).all()
