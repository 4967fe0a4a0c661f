"""getPrice's float (auctioneer.cpp:546-549): the auction kernels' fast path
(acl_price, csrc/common.h: sqrt and reciprocal by Newton steps, IEEE
fallback near float rounding boundaries) vs the IEEE expression
(float)(1.0 / (sqrt(x) + 1e-8)), bit for bit, on the GPU: random squared
distances over the whole double range, the benchmark's range, and inputs
placed on float rounding midpoints."""
import ctypes as ct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sweep(x):
    import torch
    from aclswarm_amd import _lib as L
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(np.ascontiguousarray(x, np.float64)).to(dev)
    fast = torch.empty(len(x), dtype=torch.float32, device=dev)
    ieee = torch.empty(len(x), dtype=torch.float32, device=dev)
    rc = L.lib().acl_internal_price_sweep(ct.c_void_p(xd.data_ptr()), ct.c_void_p(fast.data_ptr()),
                                          ct.c_void_p(ieee.data_ptr()), len(x))
    assert rc == 0
    return fast.cpu().numpy().view(np.uint32), ieee.cpu().numpy().view(np.uint32)


def _midpoint_inputs(rng, m):
    """x whose price 1/(sqrt(x)+1e-8) lands on (or a few ulp around) the
    midpoint of two consecutive floats."""
    f = rng.uniform(1e-3, 1e3, m).astype(np.float32)
    mid = (f.astype(np.float64) + np.nextafter(f, np.float32(np.inf)).astype(np.float64)) / 2
    s = 1.0 / mid - 1e-8
    x = s * s
    out = [x]
    for k in (1, 2, 5, 40, 300):
        out += [x * (1 + k * 2.0 ** -52), x * (1 - k * 2.0 ** -52)]
    return np.concatenate(out)


def test_price_fast_path_bit_exact(cuda):
    rng = np.random.RandomState(7)
    xs = [
        10.0 ** rng.uniform(-320, 308, 1 << 21),            # the whole double range
        rng.uniform(0, 40.0, 1 << 21) ** 2,                  # distances of the bench (C3)
        10.0 ** rng.uniform(-9, -3, 1 << 18),                # around the fast path's 1e-6 cut
        np.nextafter(1e-6, np.array([0.0, np.inf])),
        _midpoint_inputs(rng, 1 << 17),
        np.array([0.0, -0.0, 1e-320, 5e-324, 1e-200, 1e60, 1e300, np.inf, -1.0, np.nan,
                  np.finfo(np.float64).max, 1e-16, 1e-17]),
    ]
    x = np.concatenate(xs)
    fast, ieee = _sweep(x)
    bad = np.nonzero(fast != ieee)[0]
    assert bad.size == 0, (bad.size, x[bad[:5]], fast[bad[:5]], ieee[bad[:5]])
