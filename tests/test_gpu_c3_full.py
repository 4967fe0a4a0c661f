"""Config C3 at its full size (simform100 noncomplete, B = 65 536,
a unique formation per swarm from the reference generator reproduced on the
device) -- the bench's own workload. Every swarm is checked for the
properties the path guarantees (a valid permutation adopted by all
vehicles, finite commands, flags consistent with the counters); a sample
spread over the batch is checked against the CPU restatement (assignments,
status, margin bit-exact; commands within 1e-5 relative). A crowded variant
of the same swarms (positions scaled so most vehicles are within the 1.5 m
avoidance radius) drives the collision-avoidance sector algebra at full
size, sampled the same way."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as O  # noqa: E402

from aclswarm_amd import dist as D  # noqa: E402
from aclswarm_amd import engine, workload  # noqa: E402

pytestmark = pytest.mark.gpu
U_RTOL = 1e-5
B, N = 65536, 100


@pytest.fixture(scope="module")
def c3():
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(2024)
    w = workload.simform_workload(B, N, gen, dev, L=40.0, complete=False, planes=5, seed0=0)
    T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"], w["planes"])
    return w, T


def _sample_check(w, out, idx, q=None):
    idx = torch.as_tensor(idx)
    fi = w["fidx"][idx].cpu().numpy()
    forms, inv = np.unique(fi, return_inverse=True)
    ft = torch.from_numpy(forms).to(w["p"].device)
    pts = w["p"][ft].cpu().numpy()
    adj = w["adj"][ft].cpu().numpy().astype(np.uint8)
    G = np.stack([workload.dense_gains_host(w, int(f)) for f in forms])
    qq = (w["q"] if q is None else q)[idx].cpu().numpy()
    vel = w["vel"][idx].cpu().numpy()
    Pin = w["P_in"][idx].cpu().numpy().view(np.uint16)
    ref, _ = O.solve_batch(inv.astype(np.int32), qq, vel, pts, adj, G, Pin, nthreads=8)
    st = engine.status_to_numpy(out["status"][idx.to(out["status"].device)])
    P_out = out["P_out"][idx].cpu().numpy().view(np.uint16)
    np.testing.assert_array_equal(P_out, ref["P_out"])
    for k in ("flags", "eff_rounds", "rounds", "n_invalid", "n_ca"):
        np.testing.assert_array_equal(st[k], ref["status"][k], err_msg=k)
    np.testing.assert_array_equal(st["margin"], ref["status"]["margin"])
    np.testing.assert_array_equal(out["ca_flag"][idx].cpu().numpy(), ref["ca"])
    for k in ("u", "u_safe"):
        g = out[k][idx].cpu().numpy()
        err = np.abs(g - ref[k]) / np.maximum(np.abs(ref[k]), 1.0)
        assert err.max() <= U_RTOL, (k, err.max())
    return ref


def _invariants(out):
    P = out["P_out"].to(torch.int64)
    # every swarm adopted a permutation of 0..n-1
    srt, _ = torch.sort(P, dim=1)
    assert torch.equal(srt, torch.arange(N, device=P.device).expand_as(srt))
    assert bool(torch.isfinite(out["u"]).all()) and bool(torch.isfinite(out["u_safe"]).all())
    d = D.stats_dict(*D.swarm_stats(out["status"]))
    assert d["swarms"] == B and d["bad_input"] == 0 and d["nonfinite"] == 0
    return d


def test_c3_full_batch(c3):
    w, T = c3
    out = engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"])
    torch.cuda.synchronize()
    d = _invariants(out)
    assert d["valid"] == B and d["agree"] == B
    # 96 swarms spread over the whole batch (every launch slot region)
    rng = np.random.RandomState(65536)
    idx = np.sort(np.concatenate([[0, 1, B - 1], rng.choice(B, 93, replace=False)]))
    _sample_check(w, out, idx)


def test_c3_full_batch_crowded(c3):
    """The same swarms with positions scaled by 0.3 about each swarm's centre:
    vehicles crowd within the avoidance radius (utils.h / safety.cpp:412-541
    sector algebra) for most of the batch."""
    w, T = c3
    q = w["q"].clone()
    c = q[:, :, :2].mean(dim=1, keepdim=True)
    q[:, :, :2] = c + 0.3 * (q[:, :, :2] - c)
    out = engine.solve(T, w["fidx"], q, w["vel"], w["P_in"])
    torch.cuda.synchronize()
    d = _invariants(out)
    assert d["ca_active"] > B // 2, d["ca_active"]
    rng = np.random.RandomState(3)
    idx = np.sort(np.concatenate([[0, B - 1], rng.choice(B, 46, replace=False)]))
    ref = _sample_check(w, out, idx, q=q)
    assert int(ref["ca"].sum()) > 0
