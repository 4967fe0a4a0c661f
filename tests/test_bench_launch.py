"""CPU suite: bench.py's multi-rank launch path. `bench.py --gpus N` started
directly spawns its N ranks (the torchrun environment contract) before any
GPU call; --dry-run runs the same launch + gather + max-over-ranks timing on
gloo with synthetic outputs, so the path the driver's SCALE run takes is
exercised without a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(stdout):
    return [json.loads(x) for x in stdout.splitlines() if x.startswith("{")]


def test_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1", "--B", "512"])
    assert r.returncode == 0, r.stderr
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout          # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["dry_run"] is True
    assert d["config"]["B_per_gpu"] == 512 and d["config"]["B_total"] == 1024
    assert d["gathered"] == {"swarms": 1024, "status_records": 1024}
    assert d["stats"]["swarms"] == 1024
    assert d["scaling"] == "weak"


def test_gpus4_c4_shard_sizes():
    r = _run(["--gpus", "4", "--dry-run", "--config", "c4", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr
    d = _json_lines(r.stdout)[0]
    assert d["n_gpus"] == 4 and d["config"]["n"] == 500
    assert d["config"]["B_total"] == 4 * 2048 == d["gathered"]["swarms"]


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "1", "--dry-run", "--steps", "1"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_graph_group_times_exactly_the_steps():
    """--graph-steps G: the timed K steps are K / G' replays of a graph of G'
    steps, G' the largest divisor of K not above G (so no step is dropped or
    added)."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.graph_group(10, 20) == 10
    assert bench.graph_group(10, 25) == 5
    assert bench.graph_group(10, 7) == 7
    assert bench.graph_group(10, 13) == 1
    assert bench.graph_group(1, 20) == 1
    assert bench.graph_group(0, 20) == 1
    for K in range(1, 60):
        for G in range(0, 15):
            g = bench.graph_group(G, K)
            assert K % g == 0 and 1 <= g <= max(1, G)
