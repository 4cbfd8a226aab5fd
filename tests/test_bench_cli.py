"""bench.py contract: `--gpus N` runs N ranks (spawned by bench.py itself when no
launcher set WORLD_SIZE), rank 0 prints ONE JSON line with n_gpus == N, and a
launcher world that disagrees with --gpus is an error (CPU / gloo here; the
driver runs the same code path over RCCL on an 8-GPU node)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--cpu", "--steps", "4", "--warmup", "1", "--train-rows", "3000", "--test-rows", "400"]


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    e["OMP_NUM_THREADS"] = "2"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=300, env=e, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_n_ranks(n):
    """Default topology for N >= 2 (BASELINE config 2/3, the north star): rank 0 is
    the server, ranks 1..N-1 the worker ranks (RCCL reduce + broadcast on GPUs)."""
    p, lines = _run(["--gpus", str(n)] + SMALL)
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert d["steps"] == 4 and d["warmup"] == 1
    assert d["config"]["workers"] == n - 1  # (one worker per rank on the CPU)
    assert d["config"]["parallelism"].startswith(f"ps-bsp 1 server rank + {n - 1} worker ranks")
    assert d["topology"]["server_rank"] == 0 and d["topology"]["worker_ranks"] == n - 1
    assert d["topology"]["schedule"] == "reduce_bcast"
    assert d["config"]["features"] == 1024 and d["config"]["window_rows_total"] == 1024 * (n - 1)
    assert "3000 train / 400 test" in d["data"]
    assert "time_to_f1_0.40_s" in d and d["best_test_f1"] is not None
    assert d["protocol"]["server_lr"] == d["protocol"]["reference_server_lr"]


def test_bench_colocated_server_variant():
    p, lines = _run(["--gpus", "2", "--colocated-server"] + SMALL)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["config"]["workers"] == 2 and d["config"]["parallelism"].startswith("ps-bsp dp2")
    assert d["topology"]["server_rank"] is None and d["topology"]["schedule"] == "allreduce"


def test_bench_dedicated_server_config2():
    p, lines = _run(["--gpus", "2", "--dedicated-server"] + SMALL)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["workers"] == 1
    assert "1 server rank + 1 worker ranks" in d["config"]["parallelism"]


def test_bench_world_mismatch_is_an_error():
    p, _ = _run(["--gpus", "2"] + SMALL, env={"WORLD_SIZE": "1", "RANK": "0", "MASTER_PORT": "29731"})
    assert p.returncode != 0
    assert "--gpus 2" in (p.stderr + p.stdout)


def test_bench_single_gpu_default():
    """One GPU: the server and 8 workers in one process -- one per XCD of the MI355X
    (all of the reference's workers share one process too, BaseKafkaApp.java:25,70),
    server step 1/N (ServerProcessor.java:36); --workers 4 is the reference's numWorkers."""
    p, lines = _run(SMALL)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["parallelism"].startswith("ps-bsp w8")
    assert d["config"]["workers"] == 8 and d["config"]["server_lr"] == 0.125
    assert d["config"]["workers_per_gpu"] == 8
    p, lines = _run(SMALL + ["--workers", "4"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["config"]["workers"] == 4 and d["config"]["server_lr"] == 0.25
    assert d["time_to_f1_0.40_s"] is None or d["time_to_f1_0.40_s"] > 0


@pytest.mark.parametrize("c", [2, -1])
def test_bench_async_two_runs_same_engine(c):
    """Warm-up run then timed run of the same engine (SSP / ASP with a dedicated
    server rank): the workers that finished the warm-up rejoin the timed run."""
    p, lines = _run(["--gpus", "3", "--consistency", str(c)] + SMALL)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["config"]["workers"] == 2
    assert d["value"] > 0


def test_bench_default_schedule_peer_sum_on_gpus():
    """Dense multi-GPU BSP with a dedicated server defaults to the peer_sum schedule
    (rank-level lane sums into the server GPU's inbox, no collective per round); CPU
    runs and the wide models keep reduce + broadcast / the key-range server, and the
    colocated variant the all-reduce."""
    sys.path.insert(0, ROOT)
    import bench

    a = bench.parse(["--gpus", "8"])
    assert a.schedule == "peer_sum" and a.psum_colocated  # the server kernel beside rank 0's 7 lanes
    a = bench.parse(["--gpus", "8", "--dedicated-server"])
    assert a.schedule == "peer_sum" and not a.psum_colocated and a.dedicated_server
    assert bench.parse(["--gpus", "2", "--cpu"]).schedule == "reduce_bcast"
    assert bench.parse(["--gpus", "2", "--consistency", "-1"]).schedule == "reduce_bcast"
    assert bench.parse(["--gpus", "8", "--model", "sparse1m"]).schedule == "reduce_bcast"
    assert bench.parse(["--gpus", "8", "--model", "sharded100m"]).schedule == "keyrange"
    assert bench.parse(["--gpus", "8", "--colocated-server"]).schedule == "allreduce"
    assert bench.parse(["--gpus", "8", "--schedule", "reduce_bcast"]).schedule == "reduce_bcast"


def test_peer_sum_needs_gpu_ranks():
    """--bsp_schedule peer_sum on a CPU rank is refused before any collective."""
    sys.path.insert(0, ROOT)
    from psx.parallel.dist import DistEngine
    from psx.runtime.config import PSConfig

    cfg = PSConfig(num_workers=2, bsp_schedule="peer_sum", server_colocated=False, workers_per_rank=2)
    with pytest.raises(ValueError, match="peer_sum"):
        DistEngine(cfg, 0, 2, "cpu")


def test_peer_sum_colocated_worker_layout():
    """peer_sum with the server colocated: rank 0 hosts 7 lanes beside the server kernel
    (its XCD 7), every other rank --workers lanes; worker ids are contiguous per rank and
    N (the server's lr = 1/N) counts them all.  A dedicated server rank hosts none."""
    sys.path.insert(0, ROOT)
    from psx.parallel.dist import rank_worker_layout
    from psx.runtime.config import PSConfig

    cfg = PSConfig(num_workers=1, bsp_schedule="peer_sum", server_colocated=True, workers_per_rank=8)
    lay = rank_worker_layout(cfg, 8)
    assert lay == [(0, 7)] + [(7 + 8 * (r - 1), 8) for r in range(1, 8)]
    assert sum(c for _, c in lay) == 63
    assert rank_worker_layout(cfg, 1) == [(0, 7)]
    cfg = PSConfig(num_workers=1, bsp_schedule="peer_sum", server_colocated=False, workers_per_rank=8)
    assert rank_worker_layout(cfg, 8) == [(0, 0)] + [(8 * (r - 1), 8) for r in range(1, 8)]
    cfg = PSConfig(num_workers=1, bsp_schedule="allreduce", server_colocated=True, workers_per_rank=4)
    assert rank_worker_layout(cfg, 3) == [(0, 4), (4, 4), (8, 4)]
    cfg = PSConfig(num_workers=1, consistency_model=-1, server_colocated=True, workers_per_rank=4)
    assert rank_worker_layout(cfg, 3) == [(0, 0), (0, 4), (4, 4)]  # SSP / ASP: always a dedicated server
