"""CPU pins of the formation-group generator restatement
(oracle/formation_gen_oracle.py): numpy's legacy
RandomState stream semantics on the same seeds, and the reference
generator's own outputs committed as tests/golden/simform*.npz
(generate_random_formation.py:20-96 via tests/golden/make_fixtures.py)."""
import os

import numpy as np
import pytest

import formation_gen_oracle as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("seed", [0, 1, 7, 12345, 2 ** 32 - 1])
def test_mt19937_stream_matches_numpy_randomstate(seed):
    rs = np.random.RandomState(seed)
    mt = G.MT19937(seed)
    # uniform doubles across several twists, then bounded integers
    for k in range(1500):
        lo, hi = (-7.5, 7.5) if k % 3 == 0 else ((0.0, 2.0) if k % 3 == 1 else (-20.0, 20.0))
        assert mt.uniform(lo, hi) == rs.uniform(low=lo, high=hi)
    n = 100
    assert 1 + mt.bounded(n - 5) == rs.randint(1, n - 4 + 1)
    assert [mt.bounded(n - 1) for _ in range(37)] == list(rs.choice(n, size=(37,)))
    assert [mt.bounded(5) for _ in range(50)] == list(rs.randint(0, 6, size=50))
    assert mt.uniform(0.0, 1.0) == rs.uniform(0.0, 1.0)


@pytest.mark.parametrize("name", ["simform20_fc", "simform20_nc", "simform100_nc", "simform500_nc"])
def test_generator_reproduces_reference_fixtures(name):
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    n, fc, L, h, md = int(d["n"]), bool(d["fc"]), float(d["L"]), float(d["h"]), float(d["min_dist"])
    for g, s in enumerate(d["seeds"]):
        adj, forms, _ = G.generate_formation_group(int(s), n, fc, L, L, h, md)
        assert (np.array(adj, np.uint8) == d["adjmat"][g]).all(), (name, s)
        for k in range(2):
            assert (np.array(forms[k]) == d["points"][g, k]).all(), (name, s, k)
