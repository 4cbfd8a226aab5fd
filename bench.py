"""Headline benchmark: parameter-server updates/s + test accuracy on MI355X.

Metric (BASELINE.json): "test-accuracy-vs-wallclock + SGD updates/sec, logistic
regression, 1/2/4/8 workers".  One *step* is one round of the parameter
server: under Sequential consistency (BSP) every worker ingests new stream
rows into its HBM ring, runs the local solve on its adaptive window (2 L-BFGS
iterations with strong-Wolfe line search on the standardised objective = the
reference's Spark ``setMaxIter(2)`` fit, LogisticRegressionTaskSpark.java:
170-184), evaluates its local model on the test set (the reference logs that
every iteration), pushes its delta; the server applies the aggregate
(lr = 1/N), evaluates the global model and all workers pull the new weights.
Under ASP a step is one worker iteration per worker (the server applies every
push on arrival).  Nothing is skipped inside the timed region.

--model dense  (default, BASELINE.json config 2/3 = the headline): multinomial
    LR, F = 1024 hashed features, labels 1..5 (+ phantom class 0: K = 6,
    P = 6150), buffer min/max/bc = 128/1024/0.3, fine-food-reviews-shaped
    synthetic data (90k train / 4,877 test rows), random-init weights, bf16
    features with fp32 master weights.  BSP; 8 workers per GPU by default, one per
    XCD (BASELINE's 8-worker configuration; --workers 4 = the reference's numWorkers),
    all solved in ONE launch per round (csrc/kernels/lanes_kernels.hip).
--model sparse1m  (config 4): 10M rows x 2^20 hashed sparse features, labels
    1..5, ASP with a dedicated server rank (world >= 2; one GPU: in-process).
--model sharded100m  (config 5): 10M rows x 10^8 hashed features, binary
    sigmoid model, P = 10^8 + 1 dense fp32 weights, BSP key-range sharded
    server: every rank stores only its key range; a round pulls / pushes only
    the ids the windows touch (psx/parallel/keyrange.py).

value = server-applied updates per second over ALL workers.
vs_baseline = value / reference updates/s (dense: 0.76 for 1 worker, 1.85 for
the best 4-worker run); null for the configs the reference never
ran.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--model M]
       N > 1: one rank per GPU over RCCL.  Under torch.distributed.run the
       ranks come from its environment; a plain ``python bench.py --gpus N``
       spawns the N ranks itself (before anything touches the GPU) and every
       rank checks that the world it joined has exactly N ranks.
       --dedicated-server (the default): BASELINE config 2/3 (1 server rank + N-1
       worker ranks; dense: the peer_sum schedule, no collective per round --
       --schedule reduce_bcast for RCCL reduce + broadcast); --consistency D>0 /
       -1: configs 3/4 (dedicated server rank, peer data plane / RCCL p2p).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REF_UPDATES_PER_S_1W = 0.76  # single worker, 804 updates / 1053 s
REF_UPDATES_PER_S_4W = 1.85  # best 4-worker run

MODELS = {
    "dense": dict(features=1024, train_rows=90000, test_rows=4877, consistency=0, schedule="allreduce"),
    "sparse1m": dict(features=1 << 20, train_rows=10_000_000, test_rows=20000, consistency=-1, schedule="allreduce"),
    "sharded100m": dict(features=100_000_000, train_rows=10_000_000, test_rows=20000, consistency=0,
                        schedule="keyrange"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: 2000 dense, 300 wide)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default: 200 dense, 30 wide)")
    ap.add_argument("--model", default="dense", choices=sorted(MODELS))
    ap.add_argument("--consistency", type=int, default=None)
    ap.add_argument("--rows-per-step", type=int, default=None,
                    help="new stream rows per worker per step (dense default: the whole window, as with the "
                         "reference's unthrottled producer every local solve sees fresh rows; wide default: 64)")
    ap.add_argument("--server-lr", type=float, default=None,
                    help="server step on each delta (default 1/N, N = all logical workers: the reference's "
                         "learningRate = 1/numWorkers, ServerProcessor.java:36,148-151)")
    ap.add_argument("--train-rows", type=int, default=None)
    ap.add_argument("--test-rows", type=int, default=None)
    ap.add_argument("--features", type=int, default=None)
    ap.add_argument("--buffer", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="dense model feature rows (fp32: row-parallel solver with hi+lo MFMA operands)")
    ap.add_argument("--workers", type=int, default=None,
                    help="logical workers per worker GPU, one XCD each in one launch per round (default 8: one "
                         "per XCD of the MI355X -- BASELINE's 8-worker configuration on one GPU; --workers 4 is the "
                         "reference's numWorkers = 4, all hosted in one process, BaseKafkaApp.java:25,70)")
    ap.add_argument("--schedule", default=None,
                    choices=["allreduce", "reduce_bcast", "sharded", "keyrange", "peer", "peer_sum"],
                    help="multi-GPU BSP (dense default with a dedicated server: peer_sum = each worker rank's "
                         "lane sum stored into the server GPU's inbox by the round kernel, summed and applied "
                         "slice-parallel by the server kernel, written back into every rank's receive slot over "
                         "xGMI -- no collective on the round's path); reduce_bcast = RCCL reduce + broadcast; "
                         "peer = the asynchronous loops with the sequential tracker (per-worker deltas)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--graph", action="store_true", help="replay each solve as one hipGraph (dense default: eager)")
    ap.add_argument("--persist", action="store_true",
                    help="dense: stats_prep + ONE persistent launch per local solve (the default for a lone GPU "
                         "worker in one process; forces it elsewhere)")
    ap.add_argument("--chain", action="store_true",
                    help="dense: the 8-launch chain per local solve instead of the persistent launch")
    ap.add_argument("--async-scheduler", default="auto", choices=["auto", "events", "threads"],
                    help="in-process SSP/ASP with --workers > 1: event polling (GPU default) or a thread per worker")
    ap.add_argument("--rccl-trace", action="store_true",
                    help="RCCL collective/p2p trace into ./rccl-trace.<host>.<pid>.log (multi-GPU runs)")
    ap.add_argument("--dedicated-server", action="store_true", default=None,
                    help="multi-GPU: rank 0 is a server GPU only, ranks 1..N-1 the worker ranks -- BASELINE config "
                         "2/3 topology (the default for SSP / ASP and --schedule reduce_bcast; dense BSP's default "
                         "peer_sum runs the server kernel on XCD 7 of rank 0 beside 7 workers of its own)")
    ap.add_argument("--colocated-server", dest="dedicated_server", action="store_false",
                    help="multi-GPU BSP: every rank hosts workers and a server replica, one RCCL all-reduce per "
                         "round (data-parallel variant)")
    ap.add_argument("--cpu", action="store_true", help="run on CPU (plumbing check only)")
    ap.add_argument("--no-accuracy-run", dest="accuracy_run", action="store_false",
                    help="with --steps < 2000: skip the untimed continuation to 2000 rounds that reports the "
                         "accuracy half of the metric (accuracy_run in the JSON; GPU runs only)")
    a = ap.parse_args(argv)
    m = MODELS[a.model]
    wide = a.model != "dense"
    for k in ("features", "train_rows", "test_rows", "consistency"):
        if getattr(a, k) is None:
            setattr(a, k, m[k])
    if a.schedule is None and m["schedule"] == "keyrange":
        a.schedule = "keyrange"
    if a.schedule == "sharded" and wide:
        a.schedule = "keyrange"  # the wide model's sharded server is the key-range one
    if a.rows_per_step is None:
        a.rows_per_step = 64 if wide else a.buffer
    if a.steps is None:
        a.steps = 300 if wide else 2000
    if a.warmup is None:
        a.warmup = 30 if wide else 200
    # peer_sum with the server kernel colocated on rank 0 (beside 7 of its lanes) unless
    # --dedicated-server asks for a server-only GPU
    a.psum_colocated = a.dedicated_server is None
    if a.schedule is None:
        # dense BSP: the peer_sum schedule (measured against RCCL reduce + broadcast in the
        # one-GPU rehearsals, profiles/r06/README.md); CPU / wide: RCCL or gloo
        if a.dedicated_server is not False:
            a.schedule = "peer_sum" if (not wide and not a.cpu and a.consistency == 0) else "reduce_bcast"
        else:
            a.schedule = "allreduce"
    if a.dedicated_server is None:
        a.dedicated_server = True
    if a.workers is None:  # the wide configs keep one worker per GPU; dense: one worker per XCD
        a.workers = 1 if wide else 8
    return a


def build_cfg(a, n_workers):
    from psx.ops.lr import SolverOptions
    from psx.runtime.config import PSConfig

    wide = a.model != "dense"
    return PSConfig(
        num_workers=n_workers,
        consistency_model=a.consistency,
        producer_time_per_event=0,
        stream_mode="per_iter",
        rows_per_iter=a.rows_per_step,
        epochs=1_000_000,
        min_buffer_size=128,
        max_buffer_size=a.buffer,
        buffer_size_coefficient=0.3,
        init="random",
        seed=0,
        model="wide" if wide else "dense",
        dtype=a.dtype,
        sigmoid=a.model == "sharded100m",
        solver=SolverOptions(iters=a.iters, use_graph=False if a.no_graph else (True if a.graph else None),
                             zero_const=not wide, persist=True if a.persist else (False if a.chain else None)),
        bsp_schedule=a.schedule,
        server_colocated=not a.dedicated_server,
        async_scheduler=a.async_scheduler,
        server_lr=a.server_lr,  # None: 1/N, the reference's update rule (ServerProcessor.java:36)
        workers_per_rank=1 if wide else a.workers,
    )


def make_data(a, device):
    """Synthetic train/test sets of the configured shape (generated on the device for the wide configs)."""
    from psx.utils.data import synth_finefood, synth_sparse

    if a.model == "dense":
        return (synth_finefood(a.train_rows, num_features=a.features, seed=0, dtype=a.dtype),
                synth_finefood(a.test_rows, num_features=a.features, seed=1))
    labels = "binary" if a.model == "sharded100m" else "finefood"
    kw = dict(num_features=a.features, labels=labels, nnz_mean=48, max_nnz=128, device=device)
    return synth_sparse(a.train_rows, seed=0, **kw), synth_sparse(a.test_rows, seed=1, **kw)


def _backend_label() -> str:
    """What carried the multi-rank traffic: RCCL, or gloo (CPU runs, PSX_GPU_OVERSUBSCRIBE)."""
    import torch.distributed as dist

    if not dist.is_initialized():
        return "RCCL"
    return "RCCL" if dist.get_backend() == "nccl" else dist.get_backend()


def describe(a, world, cfg, ups, dt, summ, tuples_seen=None, rccl_ranks=None, topo=None):
    async_mode = a.consistency != 0 or cfg.bsp_schedule == "peer"
    n_workers = cfg.num_workers
    wpr = max(1, int(cfg.workers_per_rank))
    if a.model == "dense":
        model = f"multinomial-logreg F={a.features} K=6 (P={6 * a.features + 6}), local solver L-BFGS x2 + strong-Wolfe"
        data = (f"synthetic (fine-food-reviews-shaped, {a.train_rows} train / {a.test_rows} test rows, "
                f"random-init weights)")
        ref = REF_UPDATES_PER_S_1W if n_workers == 1 else REF_UPDATES_PER_S_4W
        # the reference's buffer is -max 1024; larger windows are a new config
        vs = round(ups / ref, 1) if a.buffer == 1024 else None
        if a.buffer != 1024:
            model += f", window {a.buffer} rows/worker"
    else:
        kind = "binary sigmoid" if a.model == "sharded100m" else "multinomial K=6"
        model = f"sparse-input logreg F={a.features} {kind}, local solver L-BFGS x2 + strong-Wolfe (window subspace)"
        data = (f"synthetic sparse hashed bag-of-words ({a.train_rows} train / {a.test_rows} test rows, "
                f"~48 nnz/row, random-init weights)")
        vs = None  # the reference never ran this configuration
    mode = "asp" if a.consistency == -1 else ("ssp" if a.consistency > 0 else "bsp")
    backend = _backend_label()
    lanes = f"{wpr} workers/GPU, one XCD each" if wpr > 1 else "1 worker/GPU"
    if cfg.bsp_schedule == "keyrange":
        par = (f"ps-{mode} key-range sharded server x{world} (every rank: 1 worker + the shard of its key "
               f"range; pull/push of the window's ids over {backend if world > 1 else 'local copies'})")
    elif world == 1 and not getattr(a, "dist_world1", False):
        if a.model != "dense" and n_workers > 1:  # (the wide model's in-process workers: a stream each)
            lanes = f"{n_workers} workers/GPU, one HIP stream each"
        par = f"ps-{mode} w{n_workers} (server colocated, {lanes if n_workers > 1 else '1 worker'})"
    elif async_mode and wpr > 1:
        par = (f"ps-{mode} 1 server rank + {world - 1} worker ranks x {wpr} workers (peer data plane over xGMI: "
               f"lanes -> server inbox, server kernel -> receive slots)")
    elif async_mode:
        par = f"ps-{mode} 1 server rank + {n_workers} worker ranks ({backend} p2p{', sparse push' if a.model != 'dense' else ''})"
    elif cfg.bsp_schedule == "peer_sum" and cfg.server_colocated:
        more = f", {world - 1} more ranks x {wpr} workers" if world > 1 else " (one rank)"
        par = (f"ps-{mode} rank 0: server kernel (XCD 7) + {n_workers - (world - 1) * wpr} workers{more} "
               f"(peer_sum over xGMI: each rank's lane sum stored into "
               f"rank 0's inbox by its round kernel, summed + applied by the server kernel, weights written into "
               f"every rank's receive slot; no collective per round)")
    elif cfg.bsp_schedule == "peer_sum":
        par = (f"ps-{mode} 1 server rank + {world - 1} worker ranks x {wpr} workers (peer_sum over xGMI: each "
               f"rank's lane sum stored into the server GPU's inbox by its round kernel, summed + applied by the "
               f"server kernel, weights written into every rank's receive slot; no collective per round)")
    elif not cfg.server_colocated:
        par = (f"ps-{mode} 1 server rank + {world - 1} worker ranks x {wpr} workers "
               f"({backend} reduce + broadcast, {cfg.bsp_schedule})")
    else:
        par = f"ps-{mode} dp{world} x {wpr} workers ({cfg.bsp_schedule}, {backend})"
    res = {
        "metric": "server_updates_per_s (PS push/pull rounds, logistic regression; test accuracy reported alongside)",
        "value": round(ups, 2),
        "unit": "updates/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt * 1000.0 / a.steps, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": vs,
        "dtype": a.dtype,
        "data": data,
        "config": {
            "model": model,
            # a PS step has no batch / sequence: the per-step work is every worker's
            # sliding window (rows x features); seq_len does not apply
            "global_batch": a.buffer * n_workers,
            "seq_len": None,
            "window_rows_total": a.buffer * n_workers,
            "window_rows_per_worker": a.buffer,
            "features": a.features,
            "parallelism": par,
            "consistency": a.consistency,
            "workers": n_workers,
            "workers_per_gpu": wpr,
            "rows_per_step_per_worker": a.rows_per_step,
            "server_lr": cfg.lr,
            "bench_model": a.model,
        },
        # where the protocol differs from the reference's (ServerProcessor.java:36,
        # WorkerTrainingProcessor.java:63-98): the update rule is the reference's
        # w += (1/N) delta; the producer is unthrottled (-p 0) and every local solve
        # fits a whole fresh window
        "protocol": {"server_lr": cfg.lr, "reference_server_lr": 1.0 / n_workers,
                     "rows_per_step_per_worker": a.rows_per_step, "window_rows": a.buffer,
                     "producer": "unthrottled (-p 0), fresh rows every round"},
        "test_accuracy": summ.get("final_server_acc"),
        "test_f1": summ.get("final_server_f1"),
        "best_test_f1": summ.get("best_server_f1"),
    }
    if topo is not None:
        res["topology"] = topo
    if rccl_ranks is not None:
        res["rccl_ranks"] = rccl_ranks
    if tuples_seen is not None:
        res["tuples_seen"] = tuples_seen
    return res


def main(argv=None):
    a = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if a.gpus > 1 and world_env is None:
        # plain `python bench.py --gpus N`: start the N ranks here.  This process
        # never touches the GPU (no torch.cuda call before or after the spawn).
        return _spawn_ranks(a.gpus, sys.argv[1:] if argv is None else list(argv))
    if os.environ.get("PSX_HANG_DUMP_S"):  # debugging aid: dump every thread's stack, then exit
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["PSX_HANG_DUMP_S"]), exit=True)
    import torch

    world = int(world_env or "1")
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks")
    if world > 1 or os.environ.get("PSX_BENCH_DIST") == "1" or a.schedule == "keyrange":
        # PSX_BENCH_DIST=1 with one rank: the multi-rank code path (DistEngine, RCCL
        # communicator, all-reduce + update launch per round) rehearsed on one GPU
        return bench_distributed(a)

    device = "cpu" if a.cpu else "cuda:0"
    from psx.runtime.engine import LocalEngine

    train, test = make_data(a, device)
    cfg = build_cfg(a, a.workers)
    cfg.max_iters = a.warmup
    eng = LocalEngine(cfg, device, train=train, test=test)
    # ONE log sink for the whole run: the accuracy half's t = 0 is the run's first
    # server row, warm-up included
    if a.warmup > 0:
        eng.run(close_log=False)
    eng.cfg.max_iters = a.steps
    n_warm = len(eng.log.book.server) if eng.log.book is not None else 0
    u0 = eng.server.updates  # the server's counter includes the warmup rounds
    if device != "cpu":
        torch.cuda.synchronize()
    # timed region: exactly `steps` rounds, synchronised on both sides (their rows
    # logged inside it)
    t0 = time.perf_counter()
    out = eng.run(close_log=False, summary=False)  # (the log book's summary below, untimed)
    t_run = time.perf_counter()
    eng.log.drain(block=True)  # every row of the timed rounds finalised inside the region
    if device != "cpu":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    from psx.utils.logsink import summarize

    out.update(summarize(eng.log.book))
    ups = (eng.server.updates - u0) / dt
    res = describe(a, 1, cfg, ups, dt, out, eng.workers[0].tuples_seen)
    if out.get("wide_lanes"):  # the wide model's workers: every solve of a round in one launch
        nl = int(out["wide_lanes"])
        mode = res["config"]["parallelism"].split()[0]
        res["config"]["parallelism"] = (f"{mode} w{nl} (server colocated, {nl} workers/GPU: one solve launch per "
                                        f"round, {max(1, 8 // nl)} XCD(s) per worker)")
        res["config"]["workers_per_gpu"] = nl
    res["native"] = {"lanes": out.get("lanes"), "hand_off_scope": out.get("hand_off_scope"),
                     "host_us_per_round": round(getattr(eng, "native_host_us_per_round", 0.0), 2),
                     "host_phases_us": getattr(eng, "native_host_phases_us", None)}
    if getattr(eng, "native_host_busy_us_per_token", None) is not None:  # SSP / ASP: the host loop's share
        res["native"]["host_busy_us_per_token"] = round(eng.native_host_busy_us_per_token, 2)
    if "phases_ms" in out:  # where the timed region's wall clock went (host view)
        res["native"]["phases_ms"] = dict(out["phases_ms"], drain=round((t0 + dt - t_run) * 1e3, 3))
    rows = list(eng.log.book.server)
    res.update(_accuracy_fields(rows, timed_from=n_warm, start_ms=eng.train_start_ms))
    if a.steps < ACC_ROUNDS and a.accuracy_run and a.model == "dense" and not a.cpu:
        eng.cfg.max_iters = ACC_ROUNDS - a.steps
        eng.run(close_log=False)
        res["accuracy_run"] = _accuracy_run(list(eng.log.book.server), a.steps, n_warm, eng.train_start_ms)
    eng.log.close()
    print(json.dumps(res))
    return res


ACC_ROUNDS = 2000  # the default --steps: the accuracy half of the metric is quoted at this many rounds


def _accuracy_run(rows, steps, n_warm, start_ms=None):
    """Accuracy half of the metric when the timed region is shorter than
    ACC_ROUNDS (the driver's short runs): the same engine keeps training, UNTIMED,
    until ACC_ROUNDS rounds past the warm-up; the curve covers every server row of
    the run (t = 0 at the first warm-up row).  updates/s is never taken from the
    continuation."""
    out = {"rounds_after_warmup": ACC_ROUNDS, "timed_rounds": steps, "untimed_continuation_rounds": ACC_ROUNDS - steps}
    out.update(_accuracy_fields(rows, timed_from=n_warm, start_ms=start_ms))
    if rows:
        out["best_test_f1"] = round(max(r[2] for r in rows), 4)
        out["test_f1"] = round(rows[-1][2], 4)
        out["test_accuracy"] = round(rows[-1][3], 4)
        out["wallclock_s"] = round((rows[-1][0] - rows[0][0]) / 1000.0, 6)
    return out


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_ranks(n: int, argv) -> int:
    """One child process per GPU with torchrun's environment (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_*); rank 0 prints the JSON line.  A failed rank takes the
    others down (their collectives would never complete)."""
    import subprocess

    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, TORCHELASTIC_RUN_ID=f"psxbench{port}")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        pending = set(range(n))
        while pending:
            for r in sorted(pending):
                code = procs[r].poll()
                if code is None:
                    continue
                pending.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:
                        if q.poll() is None:
                            q.terminate()
            time.sleep(0.05)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    if rc != 0:
        sys.exit(rc if rc > 0 else 1)
    return 0


def bench_distributed(a):
    """N > 1 GPUs: one rank per GPU (torchrun or _spawn_ranks), RCCL over xGMI.
    Default topology (BASELINE config 2/3): rank 0 is the server, ranks 1..N-1 are
    worker ranks with --workers workers each; every round the worker ranks' lane
    sums are reduced to the server (push), updated there, and broadcast (pull)."""
    import torch
    import torch.distributed as dist

    from psx.ops.lr import is_gpu
    from psx.parallel.dist import DistEngine, init_from_env, rccl_trace_env
    from psx.utils.logsink import summarize

    if a.rccl_trace:
        os.environ.update(rccl_trace_env("."))
    rank, world, device = init_from_env(cpu=a.cpu)
    a.dist_world1 = world == 1  # (the multi-rank body with one rank: labelled as such)
    if dist.get_world_size() != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the process group has {dist.get_world_size()} ranks")
    peer_bsp = a.consistency == 0 and a.schedule == "peer"
    peer_sum = a.consistency == 0 and a.schedule == "peer_sum"
    async_mode = a.consistency != 0 or peer_bsp  # (peer BSP: the asynchronous loops, sequential tracker)
    keyrange = a.schedule == "keyrange"
    # (key-range: every rank holds a shard; peer_sum: rank 0 runs the server kernel -- beside 7
    # lanes of its own unless --dedicated-server)
    psum_colo = peer_sum and a.psum_colocated
    dedicated = (async_mode or a.dedicated_server or peer_sum) and not keyrange and not psum_colo
    # workers per worker rank: --workers lanes, one XCD each (SSP / ASP / peer BSP: the lanes of one
    # persistent launch; the peer data plane runs no transfer kernel beside it, so all 8 XCDs)
    wpr = 1 if (a.model != "dense" or a.cpu) else a.workers
    worker_ranks = world - 1 if dedicated else world
    cfg = build_cfg(a, worker_ranks * wpr)  # (DistEngine fixes num_workers: rank 0's lanes under psum_colo)
    cfg.workers_per_rank = wpr
    cfg.server_colocated = not dedicated
    if peer_bsp:
        cfg.bsp_schedule = "peer"
    elif not async_mode:
        cfg.bsp_schedule = a.schedule if a.schedule != "reduce_bcast" or dedicated else "allreduce"
        if dedicated and cfg.bsp_schedule == "allreduce":
            cfg.bsp_schedule = "reduce_bcast"
    if keyrange:
        cfg.bsp_schedule = "keyrange"
    train, test = make_data(a, device)
    cfg.max_iters = a.warmup
    eng = DistEngine(cfg, rank, world, device, train=train, test=test)
    run = eng._run_async if async_mode else eng._run_bsp
    eng.mark_start()
    if a.warmup:
        run()
    n_warm = len(eng.log.book.server) if (rank == 0 and eng.log is not None and eng.log.book is not None) else 0
    cfg.max_iters = a.steps
    dist.barrier()
    if is_gpu(device):
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    out = run()
    if eng.log is not None:
        eng.log.drain(block=True)
    dist.barrier()
    if is_gpu(device):
        torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    comm = getattr(eng, "comm", None)
    # ranks of the RCCL communicator that carried the traffic: the native one (BSP
    # collectives) or torch.distributed's (nccl backend = RCCL); None on gloo
    rccl = comm.c.size if comm is not None else (dist.get_world_size() if dist.get_backend() == "nccl" else None)
    res = None
    topo = {"server_rank": 0 if (dedicated or psum_colo) else None, "worker_ranks": worker_ranks, "workers_per_rank": wpr,
            "workers": cfg.num_workers,
            "schedule": cfg.bsp_schedule if not async_mode else ("peer" if wpr > 1 else "p2p"),
            "native_lanes_loop": getattr(eng, "_lanes", None) is not None}
    # where each rank's call went (untimed: after the measurement)
    phases = [None] * world
    dist.all_gather_object(phases, getattr(eng, "_phases", None))
    if rank == 0:
        book = eng.log.book
        summ = summarize(book)
        ups = a.steps * cfg.num_workers / dt
        res = describe(a, world, cfg, ups, dt, summ, rccl_ranks=rccl, topo=topo)
        res["max_vc_gap"] = out.get("max_vc_gap")
        if any(p is not None for p in phases):
            res["rank_phases"] = phases
        if "keyrange" in out:
            k = out["keyrange"]
            res["keyrange"] = dict(k, model_bytes_per_round=round(k["model_bytes"] / max(1, a.steps + a.warmup), 1),
                                   dense_vector_bytes=(a.features + 1) * 4)
        res.update(_accuracy_fields(list(book.server), timed_from=n_warm, start_ms=eng.train_start_ms))
        if rccl is not None and rccl != world:
            raise SystemExit(f"bench.py: RCCL communicator has {rccl} ranks, world is {world}")
    if a.steps < ACC_ROUNDS and a.accuracy_run and a.model == "dense" and not async_mode and not a.cpu:
        # untimed continuation for the accuracy half (see _accuracy_run); every rank runs it
        cfg.max_iters = ACC_ROUNDS - a.steps
        eng._run_bsp()
        if rank == 0:
            res["accuracy_run"] = _accuracy_run(list(eng.log.book.server), a.steps, n_warm, eng.train_start_ms)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if eng.log is not None:
        eng.log.close()
    eng.close()
    dist.barrier()
    dist.destroy_process_group()
    return res


def _accuracy_fields(server_rows, threshold=0.40, timed_from=0, start_ms=None):
    """Accuracy half of the metric (global model on the test set, ServerProcessor.java:
    154-165): the curve, the best weighted F1 and the time to reach F1 >= threshold.
    Row timestamps are taken when each evaluation completed (us resolution).
    time_to_f1_0.40_s counts from the moment training began (start_ms: the first
    round's launch, warm-up included); ..._from_first_row_s from the run's first
    server row (the reference's t = 0, SURVEY.md section 6 -- 0 when the very first
    update already reaches the threshold)."""
    out = {"accuracy_vs_wallclock": _curve(server_rows)}
    if server_rows:
        ts0 = server_rows[0][0]
        hit = next((r for r in server_rows if r[2] >= threshold), None)
        t0 = start_ms if start_ms is not None else ts0
        out["time_to_f1_0.40_s"] = round((hit[0] - t0) / 1000.0, 6) if hit is not None else None
        out["time_to_f1_0.40_from_first_row_s"] = round((hit[0] - ts0) / 1000.0, 6) if hit is not None else None
        out["time_to_f1_0.40_rounds"] = (server_rows.index(hit) + 1) if hit is not None else None
        out["server_rows"] = len(server_rows)
        out["timed_server_rows"] = len(server_rows) - timed_from
        out["best_test_f1_all_rows"] = round(max(r[2] for r in server_rows), 4)
        # robust accuracy: the median weighted F1 / accuracy over the last 10 % of the server
        # rows (the global model's F1 swings from round to round: see README "Accuracy")
        tail = server_rows[-max(1, len(server_rows) // 10):]
        f1s, accs = sorted(r[2] for r in tail), sorted(r[3] for r in tail)
        out["f1_last10pct_median"] = round(f1s[len(f1s) // 2], 4)
        out["acc_last10pct_median"] = round(accs[len(accs) // 2], 4)
    return out


def _curve(server_rows, points=10):
    """[(seconds since the run's first server row, test accuracy, weighted F1)] samples."""
    if not server_rows:
        return []
    ts0 = server_rows[0][0]
    idx = sorted({int(i * (len(server_rows) - 1) / max(1, points - 1)) for i in range(points)})
    return [(round((server_rows[i][0] - ts0) / 1000.0, 6), round(server_rows[i][3], 4), round(server_rows[i][2], 4))
            for i in idx]


def _fresh_log(eng):
    from psx.utils.logsink import LogSink

    eng.log.close()
    return LogSink(eng.spec.eval_classes, eng.device)


if __name__ == "__main__":
    main()
