"""CPU checks of the gain kernel's fp64 atan (acl_atan_k32, csrc/common.h):
the 17-point range-reduction table read from the header equals tan / atan of
k pi / 32, and the fp32 interval estimate keeps |t| < 0.052 so the degree-9
odd polynomial stays within 2e-14 relative of atan over [0, 1e8] -- far inside
the 1e-5 relative parity bar of DistCntrl::compute (distcntrl.cpp:78-83, the
K1 atan(K2 e) terms). The GPU parity tests check the kernel itself."""
import math
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table():
    src = open(os.path.join(ROOT, "aclswarm_amd", "csrc", "common.h")).read()
    body = src[src.index("kAtan32Tab[17][5]"):]
    body = body[body.index("{") + 1: body.index("};")]
    rows = re.findall(r"\{([^{}]*)\}", body)
    return np.array([[float(x) for x in r.split(",")] for r in rows])


def test_table_is_tan_and_atan_of_k_pi_over_32():
    T = _table()
    assert T.shape == (17, 5)
    for k in range(1, 16):
        c = math.tan(k * math.pi / 32)
        assert T[k, 0] == 1.0 and T[k, 3] == 1.0
        assert abs(T[k, 2] - c) <= 2 * np.spacing(c) and T[k, 1] == -T[k, 2]
        assert abs(T[k, 4] - math.atan(T[k, 2])) <= 2 * np.spacing(T[k, 4])
    assert list(T[0]) == [1.0, 0.0, 0.0, 1.0, 0.0]
    assert list(T[16]) == [0.0, -1.0, 1.0, 0.0, math.pi / 2]


def test_reduction_and_polynomial_error_bound():
    T = _table()
    x = np.concatenate([np.linspace(0, 4, 400001), np.logspace(-12, 8, 400001)])
    xf = x.astype(np.float32)
    big = xf > 1
    with np.errstate(divide="ignore"):
        yf = np.where(big, np.float32(1) / xf, xf).astype(np.float32)
    f32 = np.float32
    t0 = yf * (f32(0.78539816) - (yf - f32(1)) * (f32(0.2447) + f32(0.0663) * yf))
    th = np.where(big, f32(1.57079633) - t0, t0).astype(np.float32)
    k = np.clip((th * f32(10.18591636) + f32(0.5)).astype(np.int32), 0, 16)
    num = T[k, 0] * x + T[k, 1]
    den = T[k, 2] * x + T[k, 3]
    t = num / den
    assert np.abs(t).max() < 0.052
    z = t * t
    p = ((z * (1 / 9) - 1 / 7) * z + 1 / 5) * z - 1 / 3
    r = T[k, 4] + (t + t * z * p)
    ref = np.arctan(x)
    rel = np.abs(r - ref) / np.maximum(ref, 1e-300)
    assert rel.max() < 2e-14


def _btable():
    src = open(os.path.join(ROOT, "aclswarm_amd", "csrc", "common.h")).read()
    body = src[src.index("kAtanBTab[34][5]"):]
    body = body[body.index("{") + 1: body.index("};")]
    rows = re.findall(r"\{([^{}]*)\}", body)
    return np.array([[float(x) for x in r.split(",")] for r in rows])


def test_binade_table():
    """acl_atan_b's rows: c = tan of the midpoint of each step's atan range."""
    T = _btable()
    assert T.shape == (34, 5)
    assert list(T[0]) == [1.0, 0.0, 0.0, 1.0, 0.0]
    assert list(T[33]) == [0.0, -1.0, 1.0, 0.0, math.pi / 2]
    for b in range(32):
        e, m = b // 4 - 4, b % 4
        lo, hi = 2.0 ** e * (1 + m / 4), 2.0 ** e * (1 + (m + 1) / 4)
        c = math.tan((math.atan(lo) + math.atan(hi)) / 2)
        row = T[b + 1]
        assert row[0] == 1.0 and row[3] == 1.0 and row[1] == -row[2]
        assert abs(row[2] - c) <= 2 * np.spacing(c)
        assert abs(row[4] - math.atan(row[2])) <= 2 * np.spacing(row[4])


def test_binade_reduction_error_bound():
    """The row index from the float bits of |x| ((bits >> 21) - 492 + 1,
    clamped to [0, 33]) keeps |t| <= 0.0625, and the degree-11 odd polynomial
    is within 1e-15 relative of atan over [0, 1e12]."""
    T = _btable()
    x = np.concatenate([np.linspace(0, 20, 400001), np.logspace(-12, 12, 400001)])
    bits = np.abs(x).astype(np.float32).view(np.uint32)
    k = np.clip((bits >> 21).astype(np.int64) - (123 << 2) + 1, 0, 33)
    t = (T[k, 0] * x + T[k, 1]) / (T[k, 2] * x + T[k, 3])
    assert np.abs(t).max() <= 0.0625 + 1e-12
    z = t * t
    p = (((z * (-1 / 11) + 1 / 9) * z - 1 / 7) * z + 1 / 5) * z - 1 / 3
    r = T[k, 4] + (t + t * z * p)
    ref = np.arctan(x)
    rel = np.abs(r - ref) / np.maximum(ref, 1e-300)
    assert rel.max() < 1e-15
