"""Run configuration shared by the CLIs, the engines and bench.py.

Defaults equal the reference's constants: numWorkers=4
(BaseKafkaApp.java:25), min/max buffer 128/1024 and bc 0.3
(WorkerAppRunner.java:56-58), -p 200 and -c 0 (ServerAppRunner.java:59-60),
numMaxIter=2 (LogisticRegressionTaskSpark.java:35), server lr = 1/numWorkers
(ServerProcessor.java:36).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field

from ..ops.lr import SolverOptions


@dataclass
class PSConfig:
    # data
    train_path: str = "./data/train.csv"
    test_path: str = "./data/test.csv"
    header: str = "auto"
    label_col: int = -1
    num_features: int | None = None  # inferred from the CSV
    num_classes: int | None = None  # inferred: max label + 1 (incl. phantom class 0)
    # model: "dense" (<= 2048 features, MFMA tiles), "wide" (sparse rows, up to
    # ~10^8 features; BASELINE.json configs 4/5) or "auto" (wide for LIBSVM
    # inputs / sparse datasets / more than 2048 features)
    model: str = "auto"
    dtype: str = "bf16"  # feature rows of the dense model: bf16 or fp32 (the reference fits in fp64)
    sigmoid: bool = False  # wide model: one logit + sigmoid (binary labels)
    log_workers: bool = True  # worker rows (the reference logs one per local iteration)
    ring_nz: int = 0  # wide model: non-zeros per ring row (0 = from the data)
    wide_dense_delta: bool = False  # wide model: also produce a dense delta (collective pushes)
    sparse_push: bool = True  # wide model, SSP/ASP across ranks: push (ids, values) instead of a dense delta
    sparse_pull: bool = True  # ... and pull the log entries since the last pull instead of the dense weights
    # topology / consistency
    num_workers: int = 4
    consistency_model: int = 0  # 0 sequential, -1 eventual, D>0 bounded delay
    # producer
    producer_time_per_event: float = 200.0  # -p (ms per event; 0 = unthrottled)
    stream_mode: str = "schedule"  # or "per_iter"
    rows_per_iter: int = 0
    epochs: int = 1
    iter_new_rows: int = 0  # a worker iterates once this many new tuples arrived (0: continuously)
    # ... or once this fraction of its current window is new (0: off).  At matched
    # producer rates a fast worker otherwise re-fits an almost unchanged window
    # many times over, which over-fits it (evaluation/README.md)
    iter_new_frac: float = 0.0
    iter_new_cap: int = 128  # ... but never more than this many new tuples per iteration (0: no cap)
    # ... and a worker's first local solves wait for at most ramp, 2 ramp, 4 ramp, ... new
    # tuples (0: off): at a low producer rate the frac / cap rule alone would hold the
    # first update back for tens of seconds (evaluation/README.md section 5)
    iter_new_ramp: int = 0
    # buffer
    min_buffer_size: int = 128
    max_buffer_size: int = 1024
    buffer_size_coefficient: float = 0.3
    # model / solver
    init: str = "zeros"
    seed: int = 0
    server_lr: float | None = None  # default 1/num_workers
    solver: SolverOptions = field(default_factory=SolverOptions)
    # run control
    max_iters: int = 0  # per worker; 0 = until data exhausted + drained
    max_wallclock_s: float = 0.0
    idle_exit_s: float = 2.0  # stop when the stream is exhausted and this much time passed
    # logging
    logging: bool = False
    log_dir: str = "."
    verbose: bool = False
    # distributed
    # allreduce | reduce_bcast | sharded | keyrange (wide: sharded == keyrange) | peer (dense, several
    # workers per rank: the sequential tracker over the peer data plane, csrc/comm/peer_bus.h) |
    # peer_sum (dense, GPUs: rank-level lane sums into the server GPU's inbox, the server kernel's
    # update written into every rank's receive slot; psx/parallel/dist.py)
    bsp_schedule: str = "allreduce"
    server_colocated: bool = True
    # logical workers per worker rank (one XCD each: the multi-lane round loop);
    # the reference hosts all of its workers in one process (BaseKafkaApp.java:25,70)
    workers_per_rank: int = 1
    # SSP / ASP data plane of worker ranks with several lanes: "peer" = the lanes push
    # their deltas into the server GPU's inbox and the server kernel writes the weights
    # into the workers' receive slots over xGMI (csrc/comm/peer_bus.h; every rank on a
    # GPU); "host" = the host shared-memory transport HostP2P; "auto" = peer when possible
    async_plane: str = "auto"
    # checkpoint
    checkpoint_dir: str | None = None
    checkpoint_every: int = 0
    resume: bool = False
    # fault injection / tracing
    inject_worker_delay_ms: dict = field(default_factory=dict)  # worker -> ms per iteration
    inject_worker_crash: dict = field(default_factory=dict)  # worker -> iteration at which it fails
    inject_worker_stop: dict = field(default_factory=dict)  # worker -> iterations after which it leaves cleanly
    worker_timeout_s: float = 600.0  # watchdog: a busy worker silent this long has failed
    # idle waits (a row-starved stream, a lane waiting for its release) are bounded by this,
    # never by the watchdog above: a short --worker_timeout must not end a healthy idle run
    idle_wait_s: float = 600.0
    on_worker_failure: str = "auto"  # drop | fail | auto (drop under eventual consistency)
    trace_path: str | None = None
    pair_eval: bool = True
    concurrent_workers: bool = True  # in-process BSP on a GPU: one HIP stream per worker
    # in-process SSP/ASP: "events" (one host thread launches the released workers'
    # solves on their HIP streams and polls completion events), "threads" (a thread
    # per worker; needed for injected delays) or "auto" (events on a GPU)
    async_scheduler: str = "auto"
    perf_log: bool = False  # write {log_dir}/logs-perf.csv (per-round device phase times)

    @property
    def lr(self) -> float:
        return self.server_lr if self.server_lr is not None else 1.0 / self.num_workers

    def to_dict(self) -> dict:
        return asdict(self)


def cadence_free(c: "PSConfig") -> bool:
    """True when the tuple-driven cadence (iter_new_rows / iter_new_frac) never
    holds a worker back: no cadence, or per-round deliveries (stream_mode
    per_iter) that always bring at least the required new tuples -- the native
    round loops (which solve every round) then run the same schedule."""
    import math

    if not c.iter_new_rows and not c.iter_new_frac:
        return True
    if c.stream_mode != "per_iter" or c.rows_per_iter <= 0:
        return False
    return c.rows_per_iter >= new_tuples_needed(c, c.max_buffer_size)


def new_tuples_needed(c: "PSConfig", window: int, updates: int | None = None) -> int:
    """New tuples a worker with a `window`-row buffer waits for before its next
    local solve: iter_new_rows, or the iter_new_frac share of the window capped at
    iter_new_cap (a large window at a high rate would otherwise wait for hundreds
    of tuples between updates).  With iter_new_ramp R and the worker's completed
    local solves `updates`, the share is also capped at R * 2^updates (the first
    updates of a slow stream come early; None: no ramp)."""
    import math

    k = math.ceil(c.iter_new_frac * int(window))
    if c.iter_new_cap > 0:
        k = min(k, c.iter_new_cap)
    ramp = int(getattr(c, "iter_new_ramp", 0) or 0)
    if ramp > 0 and updates is not None and updates < 30:
        k = min(k, ramp << max(0, int(updates)))
    return max(c.iter_new_rows, k)

