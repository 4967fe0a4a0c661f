"""How many C3 assignments depend on the Eigen version's umeyama rule.

The reference pins no Eigen ("3.2.2 or later", aclswarm/CMakeLists.txt:30-32);
Eigen::umeyama (auctioneer.cpp:397) decides the reflection sign by det(sigma)
with a rank-1 branch in 3.3.x and by det(U) det(V) in 3.4.
This engine (GPU and oracle/) follows 3.3.x. This script takes the bench's own
C3 workload (bench.py's seed and generator: n = 100, a generator formation per
swarm), runs the CPU restatement over the first S swarms once per rule
(orc_set_umeyama_variant 0 / 1, the full solve on all host threads) and
counts the swarms whose assignment, status flags or round count differ, and
how many of them the engine flags FRAGILE (decision margin < 1e-6, computed
under the 3.3 rule). The GPU output of the same swarms is checked against the
3.3 run. Test infrastructure: runs the oracle as the checker, on the box.

    python scripts/eigen_variant_risk.py [--S 16384] [--threads 16] > out.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=16384, help="swarms checked (first S of the batch)")
    ap.add_argument("--B", type=int, default=65536, help="the bench batch the workload is cut from")
    ap.add_argument("--seed", type=int, default=2024, help="bench.py --seed")
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "8")))
    args = ap.parse_args()
    import numpy as np
    import torch
    import pyoracle as O
    from aclswarm_amd import engine, workload

    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed)  # bench.py, rank 0
    w = workload.simform_workload(args.B, 100, gen, dev, L=40.0, complete=False, planes=5, seed0=0)
    T = engine.FormationTable(w["n"], w["p"], w["bits"], w["gains"], w["gain_off"], w["planes"])
    out = engine.solve(T, w["fidx"], w["q"], w["vel"], w["P_in"], margin=True)
    torch.cuda.synchronize()
    S = min(args.S, args.B)
    idx = torch.arange(S, device=dev)
    pts = w["p"][idx].cpu().numpy()
    adj = w["adj"][idx].cpu().numpy().astype(np.uint8)
    G = np.stack([workload.dense_gains_host(w, f) for f in range(S)])
    q = w["q"][:S].cpu().numpy()
    vel = w["vel"][:S].cpu().numpy()
    Pin = w["P_in"][:S].cpu().numpy().view(np.uint16)
    fidx = np.arange(S, dtype=np.int32)
    res = {}
    for var in (0, 1):
        O.lib().orc_set_umeyama_variant(var)
        t0 = time.time()
        r, _ = O.solve_batch(fidx, q, vel, pts, adj, G, Pin, nthreads=args.threads)
        res[var] = r
        print(f"[eigen_variant_risk] rule {var}: {S} swarms in {time.time() - t0:.1f} s",
              file=sys.stderr, flush=True)
    O.lib().orc_set_umeyama_variant(0)
    r0, r1 = res[0], res[1]
    dP = (r0["P_out"] != r1["P_out"]).any(axis=1)
    # (FRAGILE masked: the margin tracks the 3.3 rule's determinant test)
    keep = np.uint32(0xFFFFFFFF ^ 0x40)
    dF = (r0["status"]["flags"] & keep) != (r1["status"]["flags"] & keep)
    dR = r0["status"]["eff_rounds"] != r1["status"]["eff_rounds"]
    changed = dP | dF | dR
    fragile = (r0["status"]["flags"] & 0x40) != 0  # ACL_SWARM_FRAGILE
    gP = out["P_out"][:S].cpu().numpy().view(np.uint16)
    gst = engine.status_to_numpy(out["status"][:S])
    rep = {
        "what": "C3 swarms (bench workload, first S) solved by the CPU restatement under the "
                "Eigen 3.3.x umeyama rule (this engine's) and the 3.4 rule",
        "S": S, "threads": args.threads,
        "assignment_changed": int(dP.sum()), "flags_changed": int(dF.sum()),
        "eff_rounds_changed": int(dR.sum()), "any_changed": int(changed.sum()),
        "changed_and_fragile": int((changed & fragile).sum()),
        "fragile_total": int(fragile.sum()),
        "changed_swarms": [int(b) for b in np.nonzero(changed)[0][:64]],
        "min_margin_3_3": float(r0["status"]["margin"].min()),
        "gpu_equals_rule_3_3": bool((gP == r0["P_out"]).all()
                                    and (gst["flags"] == r0["status"]["flags"]).all()
                                    and (gst["eff_rounds"] == r0["status"]["eff_rounds"]).all()
                                    and (gst["margin"] == r0["status"]["margin"]).all()),
    }
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
