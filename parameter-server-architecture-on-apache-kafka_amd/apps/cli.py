"""Command-line front ends with the reference's flags and exit codes.

Reference CLIs (commons-cli, both ``-x`` and ``--long`` forms):
  ServerAppRunner.java:19-26  -training -test -c -p -v -h -r -l
  WorkerAppRunner.java:17-24  -test -min -max -bc -v -h -r -l
``-h`` prints the help and exits 0; stray positional arguments print the help
and exit 2 (ServerAppRunner.java:42-54).  New flags make the reference's
hard-coded constants configurable.
"""
from __future__ import annotations

import argparse
import sys

from ..ops.lr import SolverOptions
from ..runtime.config import PSConfig
from ..runtime.faults import parse_worker_map


class _Parser(argparse.ArgumentParser):
    """argparse with the reference's help/exit behaviour."""

    def error(self, message):  # bad option -> help + exit 2 (commons-cli ParseException path)
        self.print_help(sys.stderr)
        sys.stderr.write(f"\nerror: {message}\n")
        sys.exit(2)


def _common(ap: argparse.ArgumentParser):
    ap.add_argument("-v", "--verbose", action="store_true", help="If enabled, prints the parameter that are used")
    ap.add_argument("-h", "--help", action="store_true", help="Show list of possible parameter")
    ap.add_argument("-r", "--remote", action="store_true",
                    help="Rendezvous with the remote host $PSX_REMOTE_HOST instead of 127.0.0.1 "
                         "(reference: remote Kafka broker)")
    ap.add_argument("-l", "--logging", action="store_true",
                    help="If enabled, writes performance logs into ./logs-{server,worker}.csv")
    ap.add_argument("--num_workers", type=int, default=4, help="number of workers (reference: 4, hard-coded)")
    ap.add_argument("--device", default=None, help="cpu | cuda | cuda:N (default: cuda if available)")
    ap.add_argument("--log_dir", default=".")
    ap.add_argument("--master_port", type=int, default=None, help="rendezvous port (default $MASTER_PORT or 29500)")
    ap.add_argument("--trace", default=None, help="write a Chrome trace of host + device phases to this path")
    ap.add_argument("--perf_log", action="store_true",
                    help="write logs-perf.csv (per-round device phase times, updates/s) next to the CSV logs")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--rccl_trace", action="store_true",
                    help="RCCL collective/p2p trace into <log_dir>/rccl-trace.<host>.<pid>.log (multi-rank runs)")


def server_parser() -> argparse.ArgumentParser:
    ap = _Parser(prog="ServerAppRunner", add_help=False)
    ap.add_argument("-training", "--training_data_file_path", default="./data/train.csv",
                    help="The path to an csv file that is used as training data.")
    ap.add_argument("-test", "--test_data_file_path", default="./data/test.csv",
                    help="The path to an csv file that is used as test data (to compute statistics)")
    ap.add_argument("-c", "--consistency_model", type=int, default=0,
                    help="0 = sequential, -1 = eventual, D > 0 = bounded delay D (see README)")
    ap.add_argument("-p", "--producer_time_per_event", type=float, default=200.0,
                    help="ms per produced event: ~1000/p rows/s after a burst of N*128 rows; 0 = unthrottled")
    _common(ap)
    g = ap.add_argument_group("model / solver")
    g.add_argument("--num_features", type=int, default=None, help="expected feature count (default: from CSV)")
    g.add_argument("--num_classes", type=int, default=None, help="logits incl. phantom class 0 (default: max label+1)")
    g.add_argument("--label_col", type=int, default=-1)
    g.add_argument("--header", default="auto", choices=["auto", "yes", "no"])
    g.add_argument("--local_iters", type=int, default=2, help="local solver iterations (reference: 2)")
    g.add_argument("--local_solver", default="lbfgs", choices=["lbfgs", "gd"])
    g.add_argument("--gd_lr", type=float, default=1.0)
    g.add_argument("--lbfgs_history", type=int, default=10)
    g.add_argument("--ls_max", type=int, default=4, help="line-search evaluations per iteration")
    g.add_argument("--no_center", action="store_true", help="disable multinomial centring")
    g.add_argument("--keep_constant_features", action="store_true",
                   help="keep w_old for zero-variance features instead of Spark's zeroing")
    g.add_argument("--server_lr", type=float, default=None, help="server step (default 1/num_workers)")
    g.add_argument("--init", default="zeros", choices=["zeros", "random"])
    g.add_argument("--model", default="auto", choices=["auto", "dense", "wide"],
                   help="dense: <= 2048 features (MFMA tiles); wide: sparse rows up to ~1e8 hashed features "
                        "(LIBSVM input); auto: wide for .svm/.libsvm inputs or > 2048 features")
    g.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                   help="dense model feature rows: bf16 (default) or fp32 (row-parallel solver, hi+lo MFMA operands)")
    g.add_argument("--sigmoid", action="store_true", help="wide model: binary sigmoid (one logit, labels 0/1)")
    g.add_argument("--ring_nz", type=int, default=0, help="wide model: non-zeros per buffered row (0 = from data)")
    g.add_argument("--no_standardize", action="store_true",
                   help="wide model: skip Spark's 1/std feature scaling over the buffer")
    g.add_argument("--dense_push", action="store_true",
                   help="wide model, -c != 0: push the dense delta instead of (feature ids, values)")
    g.add_argument("--dense_pull", action="store_true",
                   help="wide model, -c != 0: pull the dense weights instead of the deltas applied since the last pull")
    g = ap.add_argument_group("run control")
    g.add_argument("--max_iters", type=int, default=0, help="iterations per worker (0 = until data exhausted)")
    g.add_argument("--max_wallclock_s", type=float, default=0.0)
    g.add_argument("--idle_exit_s", type=float, default=2.0)
    g.add_argument("--epochs", type=int, default=1)
    g.add_argument("--stream_mode", default="schedule", choices=["schedule", "per_iter"])
    g.add_argument("--rows_per_iter", type=int, default=0)
    g.add_argument("--iter_new_rows", type=int, default=0,
                   help="a worker iterates only after this many new tuples reached its buffer (0: continuously, "
                        "the reference's behaviour)")
    g.add_argument("--iter_new_frac", type=float, default=0.5,
                   help="a worker iterates once this fraction of its current buffer is new tuples (default 0.5: "
                        "every tuple is in at most ~2 local solves -- the pacing the reference's ~1 s Spark fit "
                        "imposes on its workers, which saw ~55 new rows per update at 10 tps; an engine 100x "
                        "faster that re-solves an unchanged window only over-fits it, evaluation/README.md "
                        "section 2); 0: iterate continuously")
    g.add_argument("--iter_new_cap", type=int, default=128,
                   help="cap of the new tuples --iter_new_frac waits for (0: none): a 1024-row window at 10 tps "
                        "would otherwise update every ~50 s")
    g.add_argument("--iter_new_ramp", type=int, default=0,
                   help="a worker's first local solves wait for at most R, 2R, 4R, ... new tuples (0: off): "
                        "at a low producer rate the frac / cap rule alone holds the first update back for tens "
                        "of seconds (evaluation/README.md section 5)")
    g.add_argument("--inprocess", action="store_true",
                   help="run server + all workers in this process on one device (single-GPU / CPU mode)")
    g.add_argument("--async_scheduler", default="auto", choices=["auto", "events", "threads"],
                   help="--inprocess SSP/ASP: one host thread polling the workers' HIP events, or a thread "
                        "per worker (auto: events on a GPU unless a delay is injected)")
    g.add_argument("--bsp_schedule", default="reduce_bcast",
                   choices=["allreduce", "reduce_bcast", "sharded", "keyrange", "peer", "peer_sum"],
                   help="multi-rank Sequential consistency: RCCL all-reduce / reduce + broadcast / reduce-scatter + "
                        "all-gather, the key-range server, peer = the asynchronous loops with the sequential "
                        "tracker, or peer_sum = each worker rank's round kernel stores its lane sum into the "
                        "server GPU's inbox and the server kernel writes the new weights into every rank's receive "
                        "slot over xGMI (dense, every rank on a GPU; no collective per round)")
    g.add_argument("--workers_per_rank", type=int, default=1,
                   help="multi-rank BSP on GPUs: logical workers per worker rank, one XCD each in one launch per "
                        "round (the native lanes loop)")
    g.add_argument("--async_plane", default="auto", choices=["auto", "peer", "host"],
                   help="SSP/ASP with --workers_per_rank > 1: peer = deltas / weights written GPU to GPU by the "
                        "kernels over xGMI (IPC-mapped fine-grained memory), host = shared-memory staging")
    g.add_argument("--checkpoint_dir", default=None)
    g.add_argument("--checkpoint_every", type=int, default=0)
    g.add_argument("--resume", action="store_true")
    g.add_argument("--inject_worker_delay", action="append", default=[], metavar="K:MS",
                   help="fault injection: worker K sleeps MS ms per iteration (straggler)")
    g.add_argument("--inject_worker_crash", action="append", default=[], metavar="K:ITER",
                   help="fault injection: worker K fails at its ITER-th iteration")
    g.add_argument("--inject_worker_stop", action="append", default=[], metavar="K:ITER",
                   help="worker K leaves the run cleanly (final push) after ITER iterations")
    g.add_argument("--worker_timeout", type=float, default=600.0,
                   help="watchdog: a worker busy and silent this many seconds has failed")
    g.add_argument("--idle_wait", type=float, default=600.0,
                   help="how long a run may wait for a worker's rows or release while nothing is in flight "
                        "(a row-starved stream; never below --worker_timeout)")
    g.add_argument("--on_worker_failure", default="auto", choices=["auto", "drop", "fail"],
                   help="drop the failed worker and continue, or abort (auto: drop under -c -1)")
    return ap


def worker_parser() -> argparse.ArgumentParser:
    ap = _Parser(prog="WorkerAppRunner", add_help=False)
    ap.add_argument("-test", "--test_data_file_path", default="./data/test.csv",
                    help="The path to an csv file that is used as test data (to compute statistics)")
    ap.add_argument("-min", "--min_buffer_size", type=int, default=128, help="min buffer size")
    ap.add_argument("-max", "--max_buffer_size", type=int, default=1024, help="max buffer size")
    ap.add_argument("-bc", "--buffer_size_coefficient", type=float, default=0.3,
                    help="target buffer = bc * events per minute")
    _common(ap)
    ap.add_argument("--first_gpu", type=int, default=1, help="GPU of worker 0 (server uses GPU 0)")
    return ap


def parse_or_exit(ap: argparse.ArgumentParser, argv):
    args, rest = ap.parse_known_args(argv)
    if args.help:
        ap.print_help()
        sys.exit(0)
    if rest:  # stray arguments -> help + exit 2 (ServerAppRunner.java:49-54)
        ap.print_help()
        sys.exit(2)
    return args


def parse_delays(items) -> dict:
    return parse_worker_map(items)


def server_config(a) -> PSConfig:
    if a.consistency_model < -1:
        # reference quirk Q4: c <= -2 matches no branch and stalls forever -> reject
        print("error: consistency_model must be -1 (eventual), 0 (sequential) or D > 0 (bounded delay)",
              file=sys.stderr)
        sys.exit(2)
    solver = SolverOptions(iters=a.local_iters, hist=a.lbfgs_history, ls_max=a.ls_max, mode=a.local_solver,
                           gd_lr=a.gd_lr, center=not a.no_center, zero_const=not a.keep_constant_features,
                           standardize=not a.no_standardize)
    return PSConfig(
        train_path=a.training_data_file_path, test_path=a.test_data_file_path, header=a.header,
        label_col=a.label_col, num_features=a.num_features, num_classes=a.num_classes,
        num_workers=a.num_workers, consistency_model=a.consistency_model,
        producer_time_per_event=a.producer_time_per_event, stream_mode=a.stream_mode,
        rows_per_iter=a.rows_per_iter, iter_new_rows=a.iter_new_rows, iter_new_frac=a.iter_new_frac, iter_new_cap=a.iter_new_cap, iter_new_ramp=a.iter_new_ramp, epochs=a.epochs, init=a.init, seed=a.seed, server_lr=a.server_lr,
        solver=solver, max_iters=a.max_iters, max_wallclock_s=a.max_wallclock_s, idle_exit_s=a.idle_exit_s,
        logging=a.logging, log_dir=a.log_dir, verbose=a.verbose, bsp_schedule=a.bsp_schedule,
        server_colocated=False, checkpoint_dir=a.checkpoint_dir, checkpoint_every=a.checkpoint_every,
        resume=a.resume, inject_worker_delay_ms=parse_delays(a.inject_worker_delay), trace_path=a.trace,
        perf_log=a.perf_log, async_scheduler=a.async_scheduler, workers_per_rank=a.workers_per_rank, async_plane=a.async_plane,
        model=a.model, dtype=a.dtype, sigmoid=a.sigmoid, ring_nz=a.ring_nz, sparse_push=not a.dense_push, sparse_pull=not a.dense_pull,
        inject_worker_crash={k: int(v) for k, v in parse_worker_map(a.inject_worker_crash).items()},
        inject_worker_stop={k: int(v) for k, v in parse_worker_map(a.inject_worker_stop).items()},
        worker_timeout_s=a.worker_timeout, idle_wait_s=a.idle_wait, on_worker_failure=a.on_worker_failure)


def print_params(title: str, items: dict):
    print()
    print("Used parameter:")
    for k, v in items.items():
        print(f"    {k}: {v}")
    print()
