"""Multi-process parameter server over torch.distributed (RCCL on MI355X, gloo on CPU).

One process per GPU.  The reference's Kafka bus (BaseKafkaApp.java:27-33:
INPUT_DATA / WEIGHTS_TOPIC / GRADIENTS_TOPIC) becomes:

* data        -> every rank holds the dataset in its own HBM and takes its
                 round-robin shard (no cross-GPU traffic at all);
* push / pull -> RCCL collectives (BSP) or point-to-point send/recv plus a
                 shared-memory token queue (SSP/ASP), see below.

Sequential (BSP, c = 0) schedules, chosen with ``--bsp_schedule``:
  allreduce     every rank is a worker and holds a replica of the server
                state: ncclAllReduce(delta) then every replica applies the same
                w += lr * sum(delta) (deterministic, bitwise identical), rank 0
                evaluates and logs.  ONE collective per round -- the cheapest
                schedule on point-to-point xGMI (ring, per-link bound).
  reduce_bcast  the textbook PS: ncclReduce(delta -> server) then
                ncclBroadcast(w <- server).  Works with a dedicated server rank
                (contributes zeros) or a colocated one.
  sharded       dense model: every rank owns P/world of the master weights;
                ncclReduceScatter(delta) -> shard update -> ncclAllGather(w).
                Wide model (or ``keyrange``): the key-range sharded server of
                keyrange.py -- each rank stores ONLY its key range and a round moves
                the window's ids and values (pull / push by owner), never P floats.
  peer_sum      dense, several workers per worker rank, every rank on a GPU (the
                bench.py default for N > 1 GPUs) and NO collective.  The server is
                rank 0's persistent kernel: on XCD 7 beside 7 lanes of rank 0's own
                (server_colocated, bench.py's default: every GPU trains), or on a
                dedicated server GPU.  The last lane to finish a slice on a worker rank stores
                the rank's lane sum straight into that rank's slot of the server
                GPU's inbox (IPC-mapped fine-grained memory, xGMI) and tags it; the
                server's persistent kernel sums the W ranks' slices in rank order,
                applies w += lr * sum slice-parallel and writes the new slice into
                every rank's receive slot with the round's tag; the next round's
                launch -- already dispatched behind the current one -- starts its
                solve once its slices' tags arrive.  No host, no kernel boundary and
                no collective sits between a round's push and the next round's pull
                (csrc/comm/peer_bus.h, LanesArgs::push, server_persist.h kSrvBspSum).
On GPUs the BSP collectives are issued through a native RCCL communicator
(psx.parallel.comm, csrc/comm/rccl_comm.h): a few us of host time per call
instead of ~30 us through torch.distributed, which otherwise bounds the round.

Bounded-delay (SSP, c = D > 0) and eventual (ASP, c = -1) need a dedicated
server rank 0 (workers are ranks 1..N).  A worker pushes a (worker, vc) token
into the shm control queue and sends its delta; the ONE server loop -- the native
AsyncServer (csrc/runtime/async_server.h) -- pops tokens in arrival order (= the
single GRADIENTS_TOPIC partition), receives from that worker, applies, and sends
the new weights to every worker the tracker releases.  The data plane is RCCL
point-to-point over xGMI (one rank per GPU) or, for ranks without an RCCL
communicator (CPU / gloo runs) and for worker ranks that host several workers as
lanes of one persistent launch (whose CUs an RCCL kernel could not share), the
host shared-memory transport HostP2P with the same per-peer message order.  A worker always posts its recv right after
its send and the server only receives from workers whose token it has seen, so
the send/recv graph is acyclic (deadlock free).
"""
from __future__ import annotations

import json
import os
import time

import torch
import torch.distributed as dist

from .. import _native
from ..models.logreg import ModelSpec
from ..ops.lr import is_gpu
from ..runtime.config import PSConfig, cadence_free
from ..runtime.engine import load_datasets
from ..runtime.faults import WorkerFailure, drop_on_failure
from ..ops.sparse import SparseDelta, nz_capacity
from .comm import make_comm, oversubscribed
from ..runtime.roles import EvalPair, ServerRole, WorkerRole, is_wide, make_evalset
from ..utils.checkpoint import flush_checkpoints, maybe_checkpoint, maybe_resume
from ..utils.logsink import LogSink, summarize
from ..utils.trace import Tracer

# peer_sum with the server colocated: rank 0's lanes take XCDs 0..6, its server kernel XCD 7
PSUM_RANK0_LANES = 7
kSrvXcdColocated = 7


def rank_worker_layout(cfg: PSConfig, world: int) -> list:
    """(first worker id, workers) of every rank: a dedicated server rank 0 (SSP / ASP, or
    server_colocated False) hosts none and ranks 1.. host workers_per_rank each; colocated,
    every rank hosts workers_per_rank -- rank 0 at most PSUM_RANK0_LANES under peer_sum,
    whose server kernel takes its last XCD."""
    wpr = max(1, int(cfg.workers_per_rank))
    async_mode = cfg.consistency_model != 0 or cfg.bsp_schedule == "peer"
    if async_mode or not cfg.server_colocated:
        return [(0, 0)] + [((r - 1) * wpr, wpr) for r in range(1, world)]
    wpr0 = min(wpr, PSUM_RANK0_LANES) if (cfg.consistency_model == 0 and cfg.bsp_schedule == "peer_sum") else wpr
    return [(0, wpr0)] + [(wpr0 + (r - 1) * wpr, wpr) for r in range(1, world)]

KIND_DELTA, KIND_FINAL, KIND_ERROR = 0, 1, 2


def rccl_trace_env(log_dir: str = ".") -> dict:
    """Environment that turns on RCCL's own collective / p2p trace (SURVEY.md §5.1:
    the analogue of the reference's Confluent monitoring interceptors,
    BaseKafkaApp.java:73-78).  RCCL reads it at communicator creation, so it must
    be in the environment before :func:`init_from_env`; one file per host and
    process under ``log_dir``."""
    return {
        "NCCL_DEBUG": "INFO",
        "NCCL_DEBUG_SUBSYS": "INIT,COLL,P2P",
        "NCCL_DEBUG_FILE": os.path.join(os.path.abspath(log_dir), "rccl-trace.%h.%p.log"),
    }


def init_from_env(cpu: bool = False):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if cpu or not torch.cuda.is_available():
        device = torch.device("cpu")
        backend = "gloo"
    else:
        # PSX_GPU_OVERSUBSCRIBE=1 (tests only): every rank on GPU 0 over gloo, so the
        # multi-rank GPU schedules can be exercised on a one-GPU machine (RCCL
        # refuses two ranks on one device)
        over = os.environ.get("PSX_GPU_OVERSUBSCRIBE") == "1"
        idx = 0 if over else local
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
        backend = "gloo" if over else "nccl"
    if not dist.is_initialized():
        kw = {"device_id": device} if backend == "nccl" else {}
        timeout = float(os.environ.get("PSX_PG_TIMEOUT_S", "0") or 0)
        if timeout > 0:
            import datetime

            kw["timeout"] = datetime.timedelta(seconds=timeout)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, device


def ctrl_queue_name() -> str:
    return f"/psx_ctrl_{os.environ.get('MASTER_PORT', '29500')}_{os.environ.get('TORCHELASTIC_RUN_ID', 'x')}"[:250]


class StopVote:
    """Run-stop agreement of the BSP ranks without a host synchronisation per round.

    A rank that wants to stop (its stream is exhausted, or its wall-clock budget
    is spent) writes 1 into a device word that the round's collective sums over
    the ranks: the allreduce schedule carries it as one extra element of the
    delta payload (no extra traffic), the other schedules all-reduce it beside
    their collectives.  The reduced word is copied stream-ordered into pinned
    host memory and read ``LAG`` rounds later, when that copy has long landed,
    so every rank stops before the same round without waiting for the device.
    Replaces a per-round all_reduce + .item() (a full device sync per round)."""

    LAG = 2
    _RING = 4

    def __init__(self, device, word: torch.Tensor, first_round: int):
        self.gpu = is_gpu(device)
        self.word = word  # one float32 element on the device, reduced each round
        self.first = first_round
        self.voted = False
        self._cpu = {}
        self._ring = _native.hip().pinned_alloc(4 * self._RING) if self.gpu else 0

    def vote(self):
        if not self.voted:
            self.word.fill_(1.0)  # stream-ordered before this round's collective
            self.voted = True

    def _slot(self, r: int):
        import ctypes

        return ctypes.c_float.from_address(self._ring + 4 * (r % self._RING))

    def post(self, r: int, stream: int):
        """After the collective of round r (on ``stream``)."""
        if self.gpu:
            self._slot(r).value = -1.0
            _native.hip().memcpy_d2h_async(self._ring + 4 * (r % self._RING), self.word.data_ptr(), 4, stream)
        else:
            self._cpu[r] = float(self.word.item())  # gloo collectives complete on return

    def decided(self, r: int) -> bool:
        """Before round r: did the vote of round r - LAG pass?"""
        k = r - self.LAG
        if k < self.first:
            return False
        if not self.gpu:
            return self._cpu.pop(k, 0.0) > 0.0
        slot = self._slot(k)
        t0 = time.time()
        while slot.value < 0.0:  # the copy was enqueued LAG rounds ago: normally already landed
            if time.time() - t0 > 600.0:
                raise TimeoutError("BSP stop vote: the device copy never landed")
        return slot.value > 0.0

    def close(self):
        if self._ring:
            _native.hip().pinned_free(self._ring)
            self._ring = 0


def pull_log_capacity(umax: int) -> int:
    """Ids the pull log keeps: ~16 pushes of the largest window subspace."""
    return 16 * (int(umax) + 1)


def uses_keyrange(cfg: PSConfig) -> bool:
    """The wide model's sharded schedule is the key-range server (keyrange.py):
    each rank stores only its key range and moves only the window's ids / values."""
    return cfg.bsp_schedule == "keyrange" or (cfg.bsp_schedule == "sharded" and cfg.model == "wide")


class DistEngine:
    def __new__(cls, cfg: PSConfig, *args, **kwargs):
        if cls is DistEngine and uses_keyrange(cfg):
            from .keyrange import KeyRangeEngine

            return KeyRangeEngine(cfg, *args, **kwargs)
        return super().__new__(cls)

    def __init__(self, cfg: PSConfig, rank: int, world: int, device, train=None, test=None):
        self.cfg, self.rank, self.world, self.device = cfg, rank, world, torch.device(device)
        # bsp_schedule "peer": sequential consistency through the asynchronous loops of the
        # peer data plane -- the server applies each delta on arrival (ServerProcessor.java:
        # 148-151) and the sequential tracker (MessageTracker.java:111-120 semantics) answers
        # every worker once the round is complete; no collective, so nothing serialises the
        # worker ranks' persistent launches behind a reduce / broadcast
        self.peer_bsp = cfg.consistency_model == 0 and cfg.bsp_schedule == "peer"
        self.async_mode = cfg.consistency_model != 0 or self.peer_bsp
        # bsp_schedule "peer_sum": rank-level lane sums into the server GPU's inbox, the
        # server kernel's slice-parallel sum + update into every rank's receive slot
        self.peer_sum = cfg.consistency_model == 0 and cfg.bsp_schedule == "peer_sum"
        if self.peer_sum and torch.device(device).type != "cuda":
            raise ValueError("--bsp_schedule peer_sum: every rank (the server too) on a GPU")
        # (peer_sum with server_colocated: rank 0 runs the server kernel on XCD 7 AND up to 7
        # lanes on XCDs 0-6 -- every GPU trains; otherwise rank 0 is a dedicated server GPU)
        self.dedicated = self.async_mode or not cfg.server_colocated
        self.psum_colocated = self.peer_sum and not self.dedicated
        wpr = max(1, int(cfg.workers_per_rank))
        n_worker_ranks = world - 1 if self.dedicated else world
        self._rank_workers = rank_worker_layout(cfg, world)  # per rank: (first worker id, count)
        n_workers = sum(c for _, c in self._rank_workers)
        if self.psum_colocated and world > 1 and oversubscribed() and os.environ.get("PSX_PSUM_REHEARSE_MULTI") != "1":
            # (PSX_PSUM_REHEARSE_MULTI=1: a short one-off rehearsal of the rank indexing; two
            # processes' lanes on one GPU can deadlock on each other's CUs, section 2 of
            # profiles/r06/README.md)
            raise ValueError("--bsp_schedule peer_sum with the server colocated: one rank per GPU (a shared GPU "
                             "would host two processes' lanes); the one-GPU rehearsal is world 1")
        if n_worker_ranks < 1:
            raise ValueError("need at least one worker rank (world size >= 2 with a dedicated server)")
        hosts_workers = not (self.dedicated and rank == 0)  # (a dedicated server rank hosts none)
        if wpr > 1 and ((not self.async_mode and cfg.bsp_schedule == "sharded")
                        or (hosts_workers and torch.device(device).type != "cuda")):
            raise ValueError("several workers per rank: BSP (allreduce / reduce_bcast) or SSP / ASP on GPUs only "
                             "(the multi-lane loops, csrc/runtime/lanes_loop.h)")
        self.wpr = wpr
        if cfg.num_workers != n_workers:
            cfg.num_workers = n_workers
        if cfg.solver.persist and not (dist.is_initialized() and dist.get_backend() == "nccl"):
            # the persistent solve needs its workgroups co-resident on the rank's GPU:
            # one rank per GPU (the nccl = RCCL backend refuses two ranks on a device;
            # gloo runs may share one)
            import dataclasses

            cfg.solver = dataclasses.replace(cfg.solver, persist=False)
        if (cfg.solver.persist is None and not self.async_mode and not self.dedicated and cfg.bsp_schedule == "allreduce"
                and dist.is_initialized() and dist.get_backend() == "nccl"):
            # every rank is one worker whose round is solve -> all-reduce -> update on ONE
            # stream: nothing else runs on the GPU beside the solve, so the persistent
            # solve (one XCD, profiles/r02_v5) is safe and faster.  The asynchronous and
            # dedicated-server schedules overlap RCCL kernels of other streams with the
            # solve and keep the launch chain.
            import dataclasses

            cfg.solver = dataclasses.replace(cfg.solver, persist=True)
        self.spec, train, test = load_datasets(cfg, train, test)
        if int(train.rows) < cfg.num_workers:
            # worker k's round-robin shard (rows k, k + N, ...) would be empty: its rank's
            # native loop would stop on its own while the peers enter the round's
            # collectives.  Every rank holds the same data, so every rank raises here.
            raise ValueError(f"{int(train.rows)} training rows for {cfg.num_workers} workers: "
                             "every worker needs a non-empty round-robin shard")
        self.wide = is_wide(self.spec)
        # wide model: collectives and dense p2p pushes need the dense delta;
        # SSP/ASP with sparse_push send (feature ids, values) instead
        self.sparse_push = self.wide and self.async_mode and cfg.sparse_push
        # ... and released workers pull the log entries since their last pull (the native
        # server's ring log, csrc/runtime/async_server.h)
        self.sparse_pull = self.sparse_push and cfg.sparse_pull
        if self.wide and not self.sparse_push:
            cfg.wide_dense_delta = True
        self._umax = 0
        if self.wide:
            nz = cfg.ring_nz or nz_capacity(train.max_nnz)
            self._umax = min(self.spec.F, cfg.max_buffer_size * nz)
        self.is_server = rank == 0
        self.worker_id = (rank - 1) if self.dedicated else rank
        self.is_worker = self.worker_id >= 0
        self.evalset = make_evalset(self.spec, test, self.device)
        wp = sp = None
        append = False
        if cfg.logging:
            # rank 0 creates both files (with the reference headers); worker ranks
            # then append whole lines to the shared logs-worker.csv
            wpath = f"{cfg.log_dir}/logs-worker.csv"
            if rank == 0:
                sp = f"{cfg.log_dir}/logs-server.csv"
                if self.is_worker:
                    wp = wpath
                else:
                    with open(wpath, "w") as fh:
                        fh.write("timestamp;partition;vectorClock;loss;fMeasure;accuracy;numTuplesSeen\n")
            elif self.is_worker:
                wp, append = wpath, True
        # every rank evaluates (workers log their local model each iteration, as the
        # reference does); only files requested with -l are written.  Rank 0 creates
        # the files (headers written at once) before the others open them to append.
        mk = lambda: LogSink(self.spec.eval_classes, self.device, wp, sp, keep_records=(rank == 0),
                             worker_append=append)
        self.log = mk() if rank == 0 else None
        if cfg.logging:
            dist.barrier()
        if self.log is None:
            self.log = mk()
        self.tracer = Tracer(cfg.trace_path.replace(".json", f".rank{rank}.json") if cfg.trace_path else None, rank,
                             self.device, f"{cfg.log_dir}/logs-perf.rank{rank}.csv" if cfg.perf_log else None)
        w0 = self.spec.init(cfg.init, seed=cfg.seed, device=self.device)
        # every rank keeps a server replica in the allreduce schedule; otherwise only rank 0
        replicated = (not self.async_mode) and cfg.bsp_schedule in ("allreduce", "sharded")
        self.server = ServerRole(self.spec, cfg, self.device, self.evalset, w0) if (self.is_server or replicated) else None
        self.t0 = time.time()
        self.worker = None
        self.workers = []
        if self.is_worker:
            tr = train.to(self.device)
            k0, nloc = self._rank_workers[rank]
            self.workers = [WorkerRole(k0 + l, self.spec, cfg, self.device, tr, self.evalset,
                                       t0=self.t0) for l in range(nloc)]
            self.worker = self.workers[0]
        self.rounds = 0
        self._ctrl = None
        self._next_vc = 0
        if (not self.async_mode and not self.peer_sum and cfg.pair_eval and (self.is_server or cfg.bsp_schedule == "allreduce")
                and self.server is not None and self.worker is not None):
            # rank 0: worker row + previous server row + the update in one launch; the other
            # allreduce ranks: worker row + their replica's update in one launch
            EvalPair(self.server, self.worker)
        # resume: rank 0 restores the server, every worker rank its own worker file;
        # BSP continues at the server's round (agreed over a collective)
        resumed = maybe_resume(cfg, self.server if self.is_server else None,
                               [self.worker] if self.worker is not None else [])
        if resumed and self.server is not None and self.is_server:
            self.rounds = int(self.server.tracker.min_clock())
        if cfg.resume and cfg.checkpoint_dir and not self.async_mode:
            t = torch.tensor([self.rounds], dtype=torch.int64, device=self.device)
            dist.broadcast(t, src=0)
            self.rounds = int(t.item())
            if self.worker is not None:
                self._next_vc = self.rounds
        elif resumed and self.worker is not None:
            self._next_vc = self.worker.vc + 1

    # ------------------------------------------------------------------
    def run(self) -> dict:
        self.mark_start()
        try:
            out = self._run_async() if self.async_mode else self._run_bsp()
        except BaseException:
            comm, self.comm = getattr(self, "comm", None), None
            if comm is not None:
                comm.c.abort()  # peers may be gone: no collective teardown
            raise
        self.close()
        flush_checkpoints(self.cfg)
        if self.worker is not None and not out.get("failed"):
            self.worker.check_device_health()
        if self.log is not None:
            self.log.close()
            if self.log.book is not None:
                out.update(summarize(self.log.book))
        self.tracer.close()
        return out

    def mark_start(self):
        if getattr(self, "train_start_ms", None) is None:  # epoch ms when training first began
            self.train_start_ms = time.time() * 1000.0

    def close(self):
        """Release the native communicator (collective: every rank calls it)."""
        self._close_async()
        comm = getattr(self, "comm", None)
        self.comm = None
        if comm is not None:
            comm.close()

    def _all_ready(self) -> bool:
        flag = torch.tensor([1 if (self.worker is None or self.worker.ready()) else 0], dtype=torch.int32,
                            device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())

    # ------------------------------------------------------------------
    def _run_bsp(self) -> dict:
        cfg, spec = self.cfg, self.spec
        sched = cfg.bsp_schedule
        srv, wk = self.server, self.worker
        P = spec.P
        zeros = torch.zeros(P, dtype=torch.float32, device=self.device)
        if wk is not None and srv is not None and wk.w is not srv.w:
            # colocated server replica: the worker's pulled weights ARE the replica
            # (BSP: every solve of a round precedes the update in stream order)
            wk.w = srv.w
            if getattr(wk.solver, "_bound", None) is not None:
                wk.solver._bound = None
        if wk is not None and srv is None:
            wk.w.zero_()
        if srv is not None and srv.pair is not None:
            # the deferred evaluation rows ride in the next solve's launches (the
            # update is a plain launch: it applies the reduced sum, not this delta)
            srv.pair.set_ride(True, fuse_update=False)
        if self.peer_sum:  # (its receive slots carry the weights: seeded once, then every round's update)
            return self._run_bsp_peer_sum()
        # bootstrap pull (vc 0): everybody starts from rank 0's weights
        boot = srv.w if srv is not None else (wk.w if wk is not None else zeros)
        dist.broadcast(boot, src=0)
        if srv is not None and srv.frag is not None:
            srv.frag.refresh(srv.w)
        if wk is not None:
            wk.w.copy_(boot)
        if not hasattr(self, "comm"):  # created once per engine (init is ~0.1-0.5 s), closed by close()
            # None: torch.distributed collectives; ranks sharing one GPU get the IPC
            # transport when the lanes loop will carry the rounds
            self.comm = make_comm(self.rank, self.world, self.device, ipc=self._lanes_cfg_ok(sched))
        comm = self.comm
        lanes = self._lanes_ok(sched, comm)
        # wait until every worker has data (the multi-lane loop waits for its lanes itself)
        while not lanes:
            if wk is not None:
                wk.ingest()
            if self._all_ready():
                break
            time.sleep(0.001)
        shard = (P + self.world - 1) // self.world
        if sched == "sharded":
            wfull, pad, myd = self._sharded_buffers(shard)
        overlap = os.environ.get("PSX_COMM_OVERLAP", "0") == "1"
        N = cfg.num_workers
        lr = cfg.lr
        t_start = time.time()
        r = self.rounds
        vote = None
        if not cfg.max_iters and not lanes:  # run until the data / the wall clock says stop: agreed without host syncs
            if sched == "allreduce" and wk is not None:
                payload = self._vote_payload()
                vote = StopVote(self.device, payload[P:], r)
            else:
                vote = StopVote(self.device, torch.zeros(1, dtype=torch.float32, device=self.device), r)
        ingested_ahead = False
        if lanes:
            # every round of this rank in the multi-lane loop: its workers' solves on their
            # XCDs (one launch), the lane sum reduced to the server over RCCL, the update,
            # the weights broadcast back (or all-reduced into every replica); an unbounded
            # run stops by a collective vote between chunks of rounds
            n = self._run_bsp_lanes(comm, cfg.max_iters)
            r += n
            if srv is not None:
                srv.updates += N * n
            for w in self.workers:
                w.vc = r
        elif len(self.workers) > 1:
            raise RuntimeError("several workers per rank need the multi-lane loop (bounded BSP over RCCL)")
        elif vote is None and self._native_bsp_ok(sched, comm):
            # every round of this rank enqueued by the native loop: solve (with the
            # previous rows riding in it) -> RCCL all-reduce -> update, no Python per round
            n = self._run_bsp_native(comm, cfg.max_iters)
            r += n  # (rank 0's tracker advanced natively)
            srv.updates += N * n
            wk.vc = r
        while not lanes:
            if cfg.max_iters and r - self.rounds >= cfg.max_iters:
                break
            if vote is not None:
                if vote.decided(r):
                    break
                if (cfg.max_wallclock_s and time.time() - t_start >= cfg.max_wallclock_s) or (
                        not cfg.max_wallclock_s and wk is not None and wk.source.exhausted):
                    vote.vote()
            self.tracer.round_begin()
            with self.tracer.span("ingest"):
                if wk is not None and not ingested_ahead:
                    wk.ingest()
            ingested_ahead = False
            logged = False
            if sched == "allreduce":
                # solve -> allreduce launched on the RCCL stream -> the evaluation rows
                # (this round's worker row and, on rank 0, the previous round's server
                # row: one paired pass) run on the compute stream WHILE the collective
                # is in flight -> update
                with self.tracer.span("solve"):
                    delta = wk.solve() if wk is not None else zeros
                with self.tracer.span("comm", schedule=sched):
                    # the stop vote rides in the payload's extra element (allreduce schedule)
                    payload = self._payload if (vote is not None and wk is not None) else delta
                    row_first = comm is None and wk is not None
                    if row_first:
                        # torch.distributed (gloo): the worker row before the push, the
                        # reference's order (WorkerTrainingProcessor.java:86-97) -- a row logged
                        # after launching an asynchronous all-reduce can land after a faster
                        # rank's next row, and the log-derived BSP gap would read 2
                        wk.log_eval(self.log)
                    if comm is not None:
                        # in stream order; PSX_COMM_OVERLAP=1 runs it on the communicator's side
                        # stream beside the evaluations instead (the fork/join event pairs cost
                        # ~20 us of host time, more than the overlap saves for a 24 KB delta)
                        if overlap:
                            comm.fork()
                        comm.all_reduce(payload, side=overlap)
                        work = comm
                    else:
                        work = dist.all_reduce(payload, op=dist.ReduceOp.SUM, async_op=True)
                    if wk is not None:
                        if not row_first:
                            wk.log_eval(self.log)
                        # the next round's stream rows land in the ring while the collective
                        # is in flight (they overwrite only slots this round's solve has read)
                        if not (cfg.max_iters and r + 1 - self.rounds >= cfg.max_iters):
                            wk.ingest()
                            ingested_ahead = True
                    if comm is not None:
                        if overlap:
                            comm.join()
                    else:
                        work.wait()
                    srv.apply(delta, lr)
                    if self.rank == 0:
                        srv.log_eval(r, self.log)  # deferred into the next round's paired pass
                    logged = True
                    new_w = srv.w
            else:
                with self.tracer.span("solve"):
                    delta = wk.compute(self.log) if wk is not None else zeros
            with self.tracer.span("comm", schedule=sched):
                if sched == "reduce_bcast":
                    if comm is not None:
                        comm.reduce(delta, 0)
                    else:
                        dist.reduce(delta, dst=0, op=dist.ReduceOp.SUM)
                    if srv is not None:
                        srv.apply_and_log(delta, r, self.log, lr)
                        logged = True
                        new_w = srv.w
                    else:
                        new_w = wk.w
                    if comm is not None:
                        comm.broadcast(new_w, 0)
                    else:
                        dist.broadcast(new_w, src=0)
                elif sched == "sharded":  # key-range shards of the master weights (KeyRange.java:11-49)
                    srv.before_update()  # srv.w / fragments are rewritten below
                    if delta.data_ptr() != pad.data_ptr():  # the solver writes into pad[:P] directly
                        pad[:P].copy_(delta)
                    lo = self.rank * shard
                    mine = wfull[lo:lo + shard]
                    if comm is not None:
                        comm.reduce_scatter(myd, pad)
                        # this rank's key range of the master weights (KeyRange.java:11-49):
                        # w[lo:lo+shard] += lr * sum(delta) on the psx update kernel
                        _native.hip().axpy(mine.data_ptr(), myd.data_ptr(), float(lr), int(shard),
                                           torch.cuda.current_stream(self.device).cuda_stream)
                        comm.all_gather(wfull, mine)  # in place: srv.w is a view of wfull
                    else:
                        dist.reduce_scatter_tensor(myd, pad, op=dist.ReduceOp.SUM)
                        mine.add_(myd, alpha=lr)
                        dist.all_gather_into_tensor(wfull, mine)
                    if srv.frag is not None:
                        srv.frag.refresh(srv.w)
                    new_w = srv.w
            if vote is not None:
                if sched != "allreduce" or wk is None:  # the vote word travels on its own
                    if comm is not None:
                        comm.all_reduce(vote.word)
                    else:
                        dist.all_reduce(vote.word, op=dist.ReduceOp.SUM)
                vote.post(r, torch.cuda.current_stream(self.device).cuda_stream if is_gpu(self.device) else 0)
            if srv is not None:
                if self.rank == 0:
                    srv.tracker.bsp_round(r)  # received(k, r) + sent(k, r + 1) for every worker
                    if not logged:
                        srv.log_eval(r, self.log)
                srv.updates += N
            if wk is not None:
                if new_w is not wk.w:
                    wk.w.copy_(new_w)
                wk.vc = r + 1
            # every rank writes its own worker file at the same round; rank 0 also the server
            maybe_checkpoint(cfg, srv if self.rank == 0 else None, r + 1, [wk] if wk is not None else [])
            self.tracer.round_end(r, (r + 1 - self.rounds) * N)
            r += 1
            if self.log is not None:
                self.log.drain()
        if srv is not None:
            srv.flush_deferred(self.log)  # the last round's server row (rank 0)
            if srv.pair is not None:
                srv.pair.set_ride(False)
        if is_gpu(self.device):
            torch.cuda.synchronize(self.device)
        if vote is not None:
            vote.close()
        elapsed = time.time() - t_start
        self.rounds = r
        return {"rounds": r, "updates": r * N, "elapsed_s": elapsed,
                "updates_per_s": r * N / elapsed if elapsed > 0 else 0.0,
                "max_vc_gap": int(srv.tracker.max_gap) if (srv is not None and self.rank == 0) else 0}

    def _lanes_ok(self, sched: str, comm) -> bool:
        """The multi-lane round loop runs this rank's BSP rounds.  Decided from the
        configuration alone, so every rank (the dedicated server has no workers)
        reaches the same answer."""
        return comm is not None and self._lanes_cfg_ok(sched)

    def _lanes_cfg_ok(self, sched: str) -> bool:
        c = self.cfg
        if os.environ.get("PSX_NATIVE_LANES", "1") == "0" or not is_gpu(self.device):
            return False
        if sched not in ("reduce_bcast", "allreduce", "peer_sum") or self.wide or self.evalset is None \
                or self.tracer.enabled:
            return False
        if c.checkpoint_dir:
            return False
        if c.inject_worker_delay_ms or c.inject_worker_crash or c.inject_worker_stop or c.dtype != "bf16":
            return False
        if c.stream_mode == "per_iter" and c.rows_per_iter <= 0 or (c.stream_mode != "per_iter"
                                                                    and not c.producer_time_per_event > 0):
            return False
        o = c.solver
        if o.nslots >= 64 or o.hist > 16:
            return False
        cap = -(-int(c.max_buffer_size) // 32) * 32
        return bool(_native.hip().lanes_supported(self.spec.Fp, self.spec.K, cap))

    def _run_bsp_lanes(self, comm, rounds: int, build_only: bool = False) -> int:
        from ..ops.lr import Fragments

        cfg, srv, sp, W = self.cfg, self.server, self.spec, self.workers
        # (peer_sum: the lanes pull the server kernel's weights from their receive slot; on
        # the colocated rank 0 the server's own w is the server kernel's, not the lanes')
        lsrv = None if self.peer_sum else srv
        w_main = lsrv.w if lsrv is not None else W[0].w
        for w in W:
            w.w = w_main
            w.ring.flush()
        if srv is not None and srv.pair is not None:
            srv.pair.flush(self.log)
        lp = getattr(self, "_lanes", None)
        if lp is None:
            h = _native.hip()
            o = cfg.solver
            sc = h.SolverCfg()
            sc.K, sc.F, sc.Fp, sc.P, sc.cap = sp.K, sp.F, sp.Fp, sp.P, -(-int(cfg.max_buffer_size) // 32) * 32
            sc.iters, sc.hist, sc.ls_max = o.iters, o.hist, o.ls_max
            sc.mode = 1 if o.mode == "gd" else 0
            sc.center, sc.zero_const = int(o.center), int(o.zero_const)
            sc.nslots, sc.gd_lr, sc.tol = o.nslots, o.gd_lr, o.tol
            d = dict(scfg=sc, N=int(cfg.num_workers), per_iter_rows=cfg.rows_per_iter if cfg.stream_mode == "per_iter"
                     else 0, p_ms=float(cfg.producer_time_per_event), epochs=int(cfg.epochs), t0_ms=self.t0 * 1000.0,
                     k=[w.k for w in W], X=[w.ring.X.data_ptr() for w in W], y=[w.ring.y.data_ptr() for w in W],
                     window=[w.window.handle for w in W], w=w_main.data_ptr(), lr=float(cfg.lr),
                     api=_native.host.capi(), server_rank=0, allreduce=int(cfg.bsp_schedule == "allreduce"),
                     log_server=int(self.rank == 0 and lsrv is not None), log_workers=int(bool(W) and cfg.log_workers),
                     # ranks sharing one GPU (IPC transport): worker rank i's lanes on XCDs
                     # i*wpr .. i*wpr + wpr - 1, so no two ranks' lanes share an XCD
                     xcd0=self._rank_workers[self.rank][0] if (W and (getattr(comm, "kind", "rccl") == "ipc" or (
                         comm is None and oversubscribed()))) else 0,
                     sink=self.log.native.handle if self.log is not None else 0,
                     tracker=lsrv.tracker.handle if (lsrv is not None and self.rank == 0) else 0,
                     new_rows=int(cfg.iter_new_rows), new_frac=float(cfg.iter_new_frac), new_cap=int(cfg.iter_new_cap), new_ramp=int(cfg.iter_new_ramp))
            if W:
                ds = W[0].source.ds
                d.update(dsX=ds.X.data_ptr(), dsy=ds.y.data_ptr(), ds_rows=int(ds.rows))
            if lsrv is not None:
                self._lane_frags = [Fragments(sp, self.device) for _ in range(3)]  # (3: overlapped rounds)
                d.update(shi=[f.hi.data_ptr() for f in self._lane_frags], slo=[f.lo.data_ptr() for f in self._lane_frags],
                         sb=[f.b.data_ptr() for f in self._lane_frags])
            ev = self.evalset
            d.update(Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=ev.T)
            lp = h.LanesLoop(d, comm.c if comm is not None else None)
            if os.environ.get("PSX_LANES_TRACE_OUT"):  # (tools: the device phase stamps of every round)
                lp.set_trace(8192)
            self._lanes = lp
        elif self.log is not None:
            lp.set_sink(self.log.native.handle)
        if build_only:
            return 0
        for i, w in enumerate(W):
            lp.set_next_local(i, int(w.source.next_local))
            lp.set_seen_at_solve(i, int(w._seen_at_solve))
        stream = comm.compute_stream() if comm is not None else torch.cuda.current_stream(self.device).cuda_stream
        try:
            n = self._lanes_chunks(lp, comm, stream, int(rounds), W)
            lp.flush(stream)
            torch.cuda.synchronize(self.device)
            lp.poll_errors()
        except RuntimeError as e:
            if "cross-workgroup wait timed out" in str(e):
                raise WorkerFailure(W[0].k if W else -1, str(e)) from e
            raise
        for i, w in enumerate(W):
            w.source.next_local = int(lp.next_local(i))
            w.iters += n
            w._seen_at_solve = int(lp.seen_at_solve(i))
            if w.ring.XT is not None:
                w.ring.xt_stale = True
        if os.environ.get("PSX_LANES_TRACE_OUT"):  # one JSON line per call: the rounds' device stamps
            with open(f"{os.environ['PSX_LANES_TRACE_OUT']}.rank{self.rank}", "a") as fh:
                fh.write(json.dumps({"rank": self.rank, "rows": [list(r) for r in lp.trace_take(stream)]}) + "\n")
        if W:
            lp.copy_out_all([w.solver.loss.data_ptr() for w in W], [w.solver.delta.data_ptr() for w in W], stream)
        if srv is not None and srv.frag is not None:
            srv.frag.refresh(srv.w)
        self.native_host_us_per_round = float(lp.host_us_per_round)
        return n

    def _run_bsp_peer_sum(self) -> dict:
        """BSP rounds over the peer data plane with rank-level sums (bsp_schedule
        peer_sum; see the module docstring): the worker ranks run their native lanes
        loop with the push / pull in the round kernel (LanesLoop.set_peer_sum), the
        server rank runs the same rounds as commands of its persistent server kernel
        (PeerServer.run_bsp: the ranks' sums applied in rank order, the weights written
        into every rank's receive slot, the global model's server row per round).  No
        collective per round; an unbounded run stops by a vote between chunks."""
        cfg, srv, W = self.cfg, self.server, self.workers
        if not self._lanes_cfg_ok("peer_sum"):
            raise ValueError("--bsp_schedule peer_sum: dense bf16 windows of <= 8192 rows on GPUs, no tracing, "
                             "checkpoints or injected faults (the native lanes loop)")
        if not hasattr(self, "_psum_region"):
            self._peer_sum_setup()
        N = cfg.num_workers
        t_start = time.time()
        t0 = time.perf_counter()
        if self.is_server and not W:
            n = self._lanes_chunks(None, None, None, int(cfg.max_iters), [])
            t1 = time.perf_counter()
            if srv.frag is not None:
                srv.frag.refresh(srv.w)
            srv.updates += N * n
            self.native_host_us_per_round = float(self._pserver.host_us_per_round)
            if os.environ.get("PSX_LANES_TRACE_OUT"):
                with open(f"{os.environ['PSX_LANES_TRACE_OUT']}.rank0", "a") as fh:
                    fh.write(json.dumps({"rank": 0, "server": [list(r) for r in self._pserver.trace_take()]}) + "\n")
            torch.cuda.synchronize(self.device)
        else:  # a worker rank, or the colocated rank 0 (its lanes + the server kernel's rounds)
            n = self._run_bsp_lanes(None, int(cfg.max_iters))
            t1 = time.perf_counter()
            if os.environ.get("PSX_PSUM_DIAG"):  # (diagnostics: receive / push slice tags; a synchronisation)
                self._psum_tags = list(self._lanes.peer_sum_tags())
            if self.is_server:
                if srv.frag is not None:
                    srv.frag.refresh(srv.w)
                srv.updates += N * n
                self.native_server_host_us_per_round = float(self._pserver.host_us_per_round)
                if os.environ.get("PSX_LANES_TRACE_OUT"):
                    with open(f"{os.environ['PSX_LANES_TRACE_OUT']}.rank0", "a") as fh:
                        fh.write(json.dumps({"rank": 0, "server": [list(r) for r in self._pserver.trace_take()]}) + "\n")
        # (where a call's wall clock went: the rounds, then the tail -- bench.py gathers these)
        self._phases = {"rounds_ms": round((t1 - t0) * 1e3, 3),
                        "tail_ms": round((time.perf_counter() - t1) * 1e3, 3)}
        self.rounds += n
        for w in W:
            w.vc = self.rounds
        if self.log is not None:
            self.log.drain()
        elapsed = time.time() - t_start
        return {"rounds": self.rounds, "updates": self.rounds * N, "elapsed_s": elapsed,
                "updates_per_s": n * N / elapsed if elapsed > 0 else 0.0,
                "max_vc_gap": int(srv.tracker.max_gap) if srv is not None else 0, "data_plane": "peer_sum",
                "lanes": len(W)}

    def _peer_sum_setup(self):
        """peer_sum bring-up (collective, once per engine): the server exports its inbox
        (one slot per worker RANK), every worker rank a receive slot, in fine-grained
        device memory; the handles are exchanged and mapped, the server seeds every
        receive slot with the current weights (round 0's pull) and drains one empty
        launch of its kernel; each worker rank builds its lanes loop with the push / pull
        addresses.  On one shared GPU (the rehearsals) the worker ranks' launches skip the
        other ranks' and the server kernel's XCDs."""
        cfg, sp = self.cfg, self.spec
        h = _native.hip()
        colo = self.psum_colocated
        # worker ranks = inbox slots (colocated: rank r's slot is r, rank 0's local)
        NS, Wr = sp.Fp // 32, (self.world if colo else self.world - 1)
        slot = self.rank if colo else self.rank - 1
        dev = self.device.index or 0
        reg = h.PeerRegion(sp.P, NS, Wr if self.is_server else 1, dev)
        handles = [None] * self.world
        dist.all_gather_object(handles, reg.handle())
        self._psum_region = reg
        wait_s = max(float(cfg.worker_timeout_s), float(cfg.idle_wait_s))
        n_lanes = sum(c for _, c in self._rank_workers)
        if oversubscribed() and n_lanes >= 8:
            raise ValueError("one shared GPU: the worker ranks' lanes leave no XCD for the server kernel")
        if oversubscribed() and Wr > 1 and not colo and os.environ.get("PSX_PSUM_REHEARSE_MULTI") != "1":
            # Each worker rank's per-round launch places workgroups on every XCD (blockIdx % 8),
            # those on another rank's XCDs leave at once -- once a CU there is free.  With two
            # worker ranks whose next launches' lanes spin on their receive tags (and whose
            # riders spin on the previous launch), each can hold the CUs the other's leaving
            # workgroups need: measured stalls of 50-900 us and a 20-s timeout
            # (profiles/r06/README.md).  On the node every rank owns its GPU; the one-GPU
            # rehearsal is the GPU server + ONE worker rank
            raise ValueError("--bsp_schedule peer_sum on one shared GPU: one worker rank (the rehearsal form)")
        # the server kernel's XCD: after the lanes on a shared GPU (n_lanes <= 7); on the
        # colocated rank 0 the last one (its lanes take XCDs 0..6)
        sxcd = n_lanes if oversubscribed() else (kSrvXcdColocated if colo else 0)
        if self.is_server:
            maps = [h.PeerMapping(handles[r], sp.P, NS, 1) for r in range(1, self.world)]
            self._peer_maps = maps
            rx, rx_tag = [m.data(0) for m in maps], [m.tags(0) for m in maps]
            if colo:  # rank 0's own receive slot (local memory), ahead of the other ranks'
                self._psum_rx0 = h.PeerRegion(sp.P, NS, 1, dev)
                rx, rx_tag = [self._psum_rx0.data(0)] + rx, [self._psum_rx0.tags(0)] + rx_tag
            d = dict(nworkers=Wr, lr=float(cfg.lr), K=sp.K, F=sp.F, FP=sp.Fp, P=int(sp.P),
                     w=self.server.w.data_ptr(), inbox=reg.base, rx=rx, rx_tag=rx_tag,
                     api=_native.host.capi(), tracker=self.server.tracker.handle,
                     bsp=1, tag_wait_s=wait_s, worker_timeout_s=float(cfg.worker_timeout_s), sxcd=sxcd,
                     # a GPU whose other launches place workgroups on the server's XCD (a shared
                     # GPU's other ranks, the colocated rank 0's own lanes launch: its workgroups
                     # of that XCD retire at once) keeps half of that XCD's CUs free for them
                     nwg=int(os.environ.get("PSX_PSUM_NWG", 16 if (oversubscribed() or colo) else 32)),
                     # colocated: the server rows' sink slots, written ahead, leave the lanes' rows room
                     ahead=16 if colo else 0)
            ev = self.evalset
            if self.log is not None and ev is not None and os.environ.get("PSX_PSUM_NO_SERVER_ROWS") != "1":
                d.update(sink=self.log.native.handle, Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=int(ev.T))
            self._pserver = h.PeerServer(d)
            self._pserver.warm_up()
            self._pserver.seed_rx()
            if os.environ.get("PSX_LANES_TRACE_OUT"):  # (tools: the server kernel's per-round stamps)
                self._pserver.set_trace(8192)
        if self.workers:
            if self.is_server:  # colocated rank 0: push into its own inbox slot, pull from its local slot
                push, push_tag = reg.data(0), reg.tags(0)
                rx_reg = self._psum_rx0
            else:
                m = h.PeerMapping(handles[0], sp.P, NS, Wr)
                self._peer_maps = [m]
                push, push_tag = m.data(slot), m.tags(slot)
                rx_reg = reg
            self._run_bsp_lanes(None, 0, build_only=True)
            lp = self._lanes
            lp.set_peer_sum(rx_reg.data(0), rx_reg.tags(0), push, push_tag, wait_s)
            if oversubscribed():  # only this rank's lanes' XCDs: no rider spins on another process's CUs
                k0, nloc = self._rank_workers[self.rank]
                mine = ((1 << nloc) - 1) << k0
                lp.set_xcd_skip(0xff & ~mine)
            elif colo and self.is_server:  # the server kernel's XCD: its workgroups leave at once
                lp.set_xcd_skip(1 << sxcd)
        torch.cuda.synchronize(self.device)
        dist.barrier()

    def _lanes_chunks(self, lp, comm, stream, rounds: int, W) -> int:
        """Rounds of the native lanes loop: a bounded run in one call; an unbounded
        one (max_iters 0: ServerAppRunner's default) in chunks of 256 rounds with a
        collective stop vote after each -- stop when any rank's wall clock is up or
        every worker rank's stream has been exhausted for idle_exit_s (the dedicated
        server rank has no say on data).  Rounds paced by the stream (the producer
        clock or a tuple cadence: a rank's round waits for its lanes' tuples) run in
        chunks of 4 rounds, so the wall-clock stop lands within a few rounds; every
        rank runs the same rounds per chunk (no deadline inside a chunk: the ranks'
        collectives must pair up)."""
        cfg = self.cfg
        idle = float(cfg.idle_wait_s)
        if lp is None:  # (peer_sum server rank: the persistent server kernel runs its rounds)
            run = lambda k, r0: int(self._pserver.run_bsp(k, r0))
        elif self.peer_sum and self.is_server:  # colocated rank 0: the server's rounds beside its lanes'
            run = lambda k, r0: self._psum_colocated_rounds(lp, k, r0, stream, idle)
        else:
            run = lambda k, r0: int(lp.run(k, r0, stream, idle))
        if rounds:
            return run(rounds, int(self.rounds))
        t_start = time.time()
        exhausted_since = None
        # (no communicator -- peer_sum: the vote over torch.distributed, on the device for nccl)
        vdev = self.device if (comm is not None or dist.get_backend() == "nccl") else torch.device("cpu")
        flag = torch.zeros(2, dtype=torch.float32, device=vdev)
        paced = cfg.stream_mode != "per_iter" or not cadence_free(cfg)
        chunk = 4 if paced else 256
        n = 0
        while True:
            n += run(chunk, int(self.rounds) + n)
            now = time.time()
            if lp is not None and W and all(lp.exhausted(i) for i in range(len(W))):
                exhausted_since = exhausted_since or now
            done_data = not W or (exhausted_since is not None and now - exhausted_since >= cfg.idle_exit_s)
            flag[0] = 1.0 if (cfg.max_wallclock_s and now - t_start >= cfg.max_wallclock_s) else 0.0
            flag[1] = 0.0 if done_data else 1.0
            if comm is not None:
                comm.all_reduce(flag)
            else:
                dist.all_reduce(flag)
            f = flag.tolist()
            if f[0] > 0 or f[1] == 0:
                return n

    def _psum_colocated_rounds(self, lp, k: int, r0: int, stream, idle: float) -> int:
        """k peer_sum rounds on the colocated rank 0: the server kernel's commands written by
        a host thread of PeerServer (run_bsp_async) while this thread runs the rank's lanes
        loop; both end when the server kernel has applied the k rounds."""
        ps = self._pserver
        ps.run_bsp_async(k, r0)
        try:
            n = int(lp.run(k, r0, stream, idle))
        finally:
            ns = int(ps.run_bsp_join())
        if n != ns:
            raise RuntimeError(f"peer_sum: rank 0's lanes ran {n} rounds, its server kernel {ns}")
        return n

    def _native_bsp_ok(self, sched: str, comm) -> bool:
        """The native BSP loop (csrc/runtime/bsp_loop.h) runs this rank: allreduce
        schedule over the native RCCL communicator, a colocated replica whose rows
        ride in the solves, a bounded run and nothing that needs Python per round."""
        c, wk, srv = self.cfg, self.worker, self.server
        if os.environ.get("PSX_NATIVE_BSP", "1") == "0" or sched != "allreduce" or comm is None:
            return False
        if getattr(comm, "kind", "rccl") != "rccl":  # the one-worker native loop is bound to RCCL
            return False
        if wk is None or srv is None or srv.pair is None or not srv.pair.ride_ok or not srv.pair.shared:
            return False
        if wk.wide or wk.evalset is None or self.tracer.enabled or not c.max_iters or c.max_wallclock_s:
            return False
        if not cadence_free(c) or c.checkpoint_dir or c.inject_worker_delay_ms or c.inject_worker_crash \
                or c.inject_worker_stop:
            return False
        src = wk.source
        if (src.mode == "per_iter" and src.rows_per_iter <= 0) or (src.mode != "per_iter" and not src.p_ms > 0):
            return False
        ring = wk.ring
        if ring.f32 or ring.XT is None or src.ds.X.dtype != torch.bfloat16:
            return False
        return wk.solver.can_ride(ring, srv.w)

    def _run_bsp_native(self, comm, rounds: int) -> int:
        cfg, wk, srv, sp = self.cfg, self.worker, self.server, self.spec
        wk.ring.flush()
        srv.pair.flush(self.log)
        src, ring, ev = wk.source, wk.ring, wk.evalset
        d = dict(dsX=src.ds.X.data_ptr(), dsy=src.ds.y.data_ptr(), ds_rows=int(src.ds.rows), k=wk.k, N=src.N,
                 per_iter_rows=src.rows_per_iter if src.mode == "per_iter" else 0, p_ms=float(src.p_ms),
                 epochs=int(src.epochs), t0_ms=float(src.t0) * 1000.0, X=ring.X.data_ptr(), XT=ring.XT.data_ptr(),
                 y=ring.y.data_ptr(), cap=ring.cap, Fp=sp.Fp, K=sp.K, F=sp.F, window=wk.window.handle,
                 whi=wk.solver.frag.hi.data_ptr(), wlo=wk.solver.frag.lo.data_ptr(), wb=wk.solver.frag.b.data_ptr(),
                 loss=wk.solver.loss.data_ptr(), delta=wk.solver.delta.data_ptr(), w=srv.w.data_ptr(),
                 shi=srv.frag.hi.data_ptr(), slo=srv.frag.lo.data_ptr(), sb=srv.frag.b.data_ptr(),
                 scoff=srv.frag.coff, lr=float(cfg.lr), tracker=srv.tracker.handle if self.rank == 0 else 0,
                 Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=ev.T, acc=wk.scratch.acc.data_ptr(),
                 ticket=wk.scratch.ticket.data_ptr(), sink=self.log.native.handle if self.log is not None else 0,
                 log_server=1 if self.rank == 0 else 0, api=_native.host.capi())
        loop = _native.hip().BspLoop(wk.solver._native, comm.c, d)
        loop.next_local = int(src.next_local)
        stream = comm.compute_stream()
        n = int(loop.run(int(rounds), int(self.rounds), stream))
        loop.flush(stream)
        src.next_local = int(loop.next_local)
        wk.iters += n
        wk._seen_at_solve = wk.tuples_seen
        self.native_host_us_per_round = float(loop.host_us_per_round)
        return n

    def _vote_payload(self) -> torch.Tensor:
        """[P + 1] all-reduce payload: the solver writes its delta into the first P
        entries in place, entry P is the stop vote (StopVote)."""
        P, wk = self.spec.P, self.worker
        pl = getattr(self, "_payload", None)
        if pl is None or pl.numel() != P + 1:
            pl = torch.zeros(P + 1, dtype=torch.float32, device=self.device)
            self._payload = pl
        else:
            pl[P:].zero_()
        if wk.solver.delta.data_ptr() != pl.data_ptr():
            wk.solver.delta = pl[:P]  # bound by the native solver at its next run
            if getattr(wk.solver, "_bound", None) is not None:
                wk.solver._bound = None
        return pl

    def _sharded_buffers(self, shard: int):
        """Padded full weight vector whose first P entries ARE the server
        replica (srv.w is re-pointed to a view of it) and a padded delta whose
        first P entries ARE the solver's output: the only passes per round
        are the collectives themselves and the shard update."""
        if getattr(self, "_shard_bufs", None) is not None and self._shard_bufs[0].numel() == shard * self.world:
            return self._shard_bufs
        srv, wk, P = self.server, self.worker, self.spec.P
        wfull = torch.zeros(shard * self.world, dtype=torch.float32, device=self.device)
        wfull[:P].copy_(srv.w)
        srv.w = wfull[:P]
        pad = torch.zeros(shard * self.world, dtype=torch.float32, device=self.device)
        if wk is not None:
            wk.w = srv.w
            wk.solver.delta = pad[:P]  # bound lazily by the native solver at its first run
            if getattr(wk.solver, "_bound", None) is not None:
                wk.solver._bound = None
        myd = torch.zeros(shard, dtype=torch.float32, device=self.device)
        self._shard_bufs = (wfull, pad, myd)
        return self._shard_bufs

    # ------------------------------------------------------------------
    def _open_ctrl(self, host_p2p: bool):
        """The control plane (token queue, sparse-pull reply queues) and, for ranks
        without an RCCL communicator (CPU / gloo), the host shared-memory data
        plane (HostP2P): rank 0 creates, the workers attach after the barrier."""
        name = ctrl_queue_name()
        N = self.cfg.num_workers
        h = _native.hip()
        gpu = is_gpu(self.device)
        self._hp2p = None
        lanes = self.wpr > 1  # several workers per rank: the asynchronous lanes loop
        peers = self.world - 1 if lanes else N  # p2p peers: worker ranks (one worker each, or lanes)
        if self.rank == 0:
            self._ctrl = _native.host.CtrlQueue(name, 1024, True)
            # sparse pull: one reply queue per worker tells it what its next pull carries;
            # lanes: one per worker rank, shared by its workers (which lane the weights are for)
            if lanes:
                self._replies = [_native.host.CtrlQueue(f"{name}_r{r}"[:250], 256, True) for r in range(peers)]
            else:
                self._replies = ([_native.host.CtrlQueue(f"{name}_r{j}"[:250], 64, True) for j in range(N)]
                                 if self.sparse_pull else [])
            if host_p2p:
                self._hp2p = h.HostP2P(f"{name}_p2p"[:250], peers, 0, True, gpu, self._p2p_cap())
        dist.barrier()
        if self.rank != 0:
            self._ctrl = _native.host.CtrlQueue(name, 1024, False)
            self._reply = (_native.host.CtrlQueue(f"{name}_r{self.worker_id}"[:250], 256 if lanes else 64, False)
                           if (self.sparse_pull or lanes) else None)
            if host_p2p:
                self._hp2p = h.HostP2P(f"{name}_p2p"[:250], peers, self.rank, False, gpu, self._p2p_cap())
        dist.barrier()

    def _p2p_cap(self) -> int:
        """Bytes per HostP2P direction: a few of the largest messages (dense weights)."""
        return max(1 << 20, 4 * 4 * int(self.spec.P))

    def _peer_plane(self) -> bool:
        """SSP / ASP with several workers per worker rank (the asynchronous lanes loop):
        the peer data plane (csrc/comm/peer_bus.h) when every rank is on a GPU -- the
        lanes write their deltas into the server GPU's inbox and the server kernel
        writes the weights into their receive slots over xGMI.  Agreed collectively."""
        if not (self.async_mode and self.wpr > 1) or self.wide or self.cfg.async_plane == "host":
            if self.peer_bsp:
                raise ValueError("--bsp_schedule peer: several dense workers per worker rank on GPUs")
            return False
        flags = [None] * self.world
        dist.all_gather_object(flags, bool(is_gpu(self.device)))
        ok = all(flags)
        if (self.cfg.async_plane == "peer" or self.peer_bsp) and not ok:
            raise ValueError("--async_plane peer: every rank (the server too) must be on a GPU")
        return ok

    def _run_async(self) -> dict:
        if not hasattr(self, "comm"):  # collective: every rank creates it (None on gloo / CPU)
            self.comm = make_comm(self.rank, self.world, self.device)
        # several workers per worker rank (the asynchronous lanes loop): its persistent
        # launch holds every CU of the lanes' XCDs, so no RCCL p2p kernel could run
        # beside it.  The pushes / pulls go either through the peer data plane (the
        # kernels themselves store into IPC-mapped fine-grained memory of the other
        # GPU: no transfer kernel, no host staging) or, with a CPU rank, through the
        # host shared-memory transport HostP2P
        # the control plane (and the data plane's regions) are set up once per engine and
        # kept across runs (the warm-up and timed runs of bench.py): the native server
        # loops hold their queues' handles
        if not hasattr(self, "_peer"):
            self._peer = self._peer_plane()
        if self._ctrl is None:
            self._open_ctrl(host_p2p=(self.comm is None or self.wpr > 1) and not self._peer)
            if self._peer:
                self._peer_setup()
        try:
            if self.is_server:  # ONE server loop: the native one (peer plane, RCCL p2p or HostP2P)
                return self._server_loop_native()
            if self.wpr > 1:
                return self._worker_loop_lanes()
            return self._worker_loop()
        finally:
            dist.barrier()

    def _ctrl_diag(self) -> str:
        """(failure reports) the control plane as this rank sees it: tokens pushed /
        popped and the shared-memory segment of each queue."""
        out = []
        for tag, q in [("ctrl", getattr(self, "_ctrl", None)), ("reply", getattr(self, "_reply", None))] + \
                [(f"reply{i}", q) for i, q in enumerate(getattr(self, "_replies", None) or [])]:
            if q is not None:
                e, d, ino = q.state()
                out.append(f"{tag} {q.name} pushed {e} popped {d} inode {ino}")
        return "control plane: " + ", ".join(out)

    def _close_async(self):
        """Tear down the asynchronous control / data planes (after the last run)."""
        ps = getattr(self, "_pserver", None)
        if ps is not None:  # (the object stays for its counters: host_us_per_update, arrivals)
            ps.stop()
        for m in getattr(self, "_peer_maps", []):
            m.close()
        self._peer_maps = []
        if hasattr(self, "_psum_region"):  # peer_sum: a later run sets the plane up afresh (tags from 0)
            del self._psum_region
            self._lanes = None
            self._pserver = None
        if getattr(self, "_ctrl", None) is not None:
            if self.rank == 0:
                self._ctrl.unlink()
                for q in getattr(self, "_replies", []):
                    q.unlink()
            self._ctrl = None
        if getattr(self, "_hp2p", None) is not None:
            self._hp2p.unlink()
            self._hp2p = None

    def _peer_setup(self):
        """Peer data plane bring-up (collective): every rank exports one region of
        fine-grained device memory -- the server its inbox (one delta slot per worker),
        a worker rank its receive slots (one per lane) -- the handles are exchanged, each
        side maps the other's, and the loops are built with EVERY allocation and fill
        done now, and each loop's first launch too (an empty one, drained here): on a GPU
        shared by several ranks (the one-GPU rehearsal) a fill kernel or a first launch's
        one-time device work enqueued after another rank's persistent launch could wait
        for its CUs -- seen as a worker rank whose host loop stalled 20 s in its first
        launch while the server's watchdog fired."""
        cfg, sp = self.cfg, self.spec
        h = _native.hip()
        N, NS = cfg.num_workers, sp.Fp // 32
        dev = self.device.index or 0
        reg = h.PeerRegion(sp.P, NS, N if self.is_server else self.wpr, dev)
        handles = [None] * self.world
        dist.all_gather_object(handles, reg.handle())
        self._peer_region = reg
        if self.is_server:
            maps, rx, rxt = {}, [], []
            for k in range(N):
                r, l = 1 + k // self.wpr, k % self.wpr
                if r not in maps:
                    maps[r] = h.PeerMapping(handles[r], sp.P, NS, self.wpr)
                rx.append(maps[r].data(l))
                rxt.append(maps[r].tags(l))
            self._peer_maps = list(maps.values())
            n_lanes = (self.world - 1) * self.wpr
            if oversubscribed() and n_lanes >= 8:
                raise ValueError("one shared GPU: the worker ranks' lanes leave no XCD for the server kernel")
            ev = self.evalset
            d = dict(nworkers=N, lr=float(cfg.lr), K=sp.K, F=sp.F, FP=sp.Fp, P=int(sp.P),
                     w=self.server.w.data_ptr(), inbox=reg.base, rx=rx, rx_tag=rxt, api=_native.host.capi(),
                     tracker=self.server.tracker.handle, ctrl=self._ctrl.handle,
                     replies=[self._replies[k // self.wpr].handle for k in range(N)],
                     worker_timeout_s=float(cfg.worker_timeout_s),
                     # one GPU shared by every rank: the XCD after the worker ranks' lanes
                     sxcd=n_lanes if oversubscribed() else 0)
            if self.log is not None and ev is not None:
                d.update(sink=self.log.native.handle, Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=int(ev.T))
            self._pserver = h.PeerServer(d)
            self._pserver.warm_up()
        else:
            m = h.PeerMapping(handles[0], sp.P, NS, N)
            self._peer_maps = [m]
            lp = self._alanes_build()
            ks = [w.k for w in self.workers]
            lp.set_peer(reg.data(0), reg.tags(0), reg.stride, [m.data(k) for k in ks], [m.tags(k) for k in ks])
            lp.prepare_async()  # (with one empty launch: see LanesLoop::prepare_async)
        torch.cuda.synchronize(self.device)
        dist.barrier()

    def _native_server(self):
        """The C++ server loop (csrc/runtime/async_server.h) bound to this engine's
        tensors, token queue, tracker and metrics sink (created once per engine)."""
        a = getattr(self, "_aserver", None)
        if a is not None and getattr(self, "_aserver_p2p", None) is (self._hp2p or self.comm):
            return a
        cfg, srv, spec = self.cfg, self.server, self.spec
        h = _native.hip()
        gpu = is_gpu(self.device)
        d = dict(nworkers=cfg.num_workers, lr=float(cfg.lr), P=int(spec.P), w=srv.w.data_ptr(),
                 api=_native.host.capi(), tracker=srv.tracker.handle, ctrl=self._ctrl.handle,
                 worker_timeout_s=float(cfg.worker_timeout_s), cpu=0 if gpu else 1)
        keep = []
        if self.wide:
            d.update(KP=spec.KP, K=spec.K, Fw=int(spec.F))
            if self.sparse_push:
                KP = spec.KP
                ubuf = torch.zeros(max(1, self._umax), dtype=torch.int32, device=self.device)
                dbuf = torch.zeros(KP + self._umax * KP, dtype=torch.float32, device=self.device)
                keep += [ubuf, dbuf]
                d.update(model=1, umax=int(self._umax), ubuf=ubuf.data_ptr(), dbuf=dbuf.data_ptr())
                if self.sparse_pull:
                    cap = pull_log_capacity(self._umax)
                    lids = torch.zeros(cap, dtype=torch.int32, device=self.device)
                    lvals = torch.zeros(cap * KP, dtype=torch.float32, device=self.device)
                    keep += [lids, lvals]
                    d.update(sparse_pull=1, lids=lids.data_ptr(), lvals=lvals.data_ptr(), logcap=cap,
                             replies=[q.handle for q in self._replies])
            else:
                buf = torch.zeros(spec.P, dtype=torch.float32, device=self.device)
                keep.append(buf)
                d.update(model=2, buf=buf.data_ptr())
        else:
            buf = torch.zeros(spec.P, dtype=torch.float32, device=self.device)
            keep.append(buf)
            d.update(model=0, buf=buf.data_ptr(), K=spec.K, F=spec.F, FP=spec.Fp)
            fr = srv.frag
            if fr is not None:  # (GPU: the evaluation reads the model's MFMA fragments)
                d.update(coff=fr.coff, fhi=fr.hi.data_ptr(), flo=fr.lo.data_ptr(), fb=fr.b.data_ptr())
        ev = self.evalset
        if self.log is not None and ev is not None:
            d.update(sink=self.log.native.handle, acc=srv.scratch.acc.data_ptr(), ticket=srv.scratch.ticket.data_ptr(),
                     T=int(ev.T))
            if self.wide:
                ds = ev.ds
                d.update(t_indptr=ds.indptr.data_ptr(), t_idx=ds.idx.data_ptr(), t_val=ds.val.data_ptr(),
                         t_y=ds.y.data_ptr())
            else:
                d.update(Xt=ev.X.data_ptr(), yt=ev.y.data_ptr())
        if self.wpr > 1:  # worker k on rank 1 + k // wpr; that rank's reply queue says whose weights come
            d.update(peer=[1 + k // self.wpr for k in range(cfg.num_workers)],
                     replies=[self._replies[k // self.wpr].handle for k in range(cfg.num_workers)])
        p2p = self._hp2p if self._hp2p is not None else h.RcclP2P(self.comm.c)
        a = h.AsyncServer(p2p, d, torch.cuda.current_stream(self.device).cuda_stream if gpu else 0)
        self._aserver, self._aserver_keep, self._aserver_p2p = a, keep + [p2p], (self._hp2p or self.comm)
        return a

    def _server_loop_native(self) -> dict:
        """SSP / ASP server over native RCCL p2p: the C++ loop pops tokens, enqueues
        recv -> update (-> evaluation row) -> grouped sends of the new weights on
        this rank's stream and never synchronises with the device; Python only
        handles checkpoints and failed workers (ServerProcessor.java:143-183)."""
        cfg, srv = self.cfg, self.server
        h = _native.hip()
        peer = getattr(self, "_peer", False)
        a = self._pserver if peer else self._native_server()
        if self.log is not None and not peer:
            # rows logged natively go to the sink bound at creation: rebind if swapped
            if getattr(self, "_aserver_sink", None) not in (None, self.log.native.handle):
                self._aserver = None
                a = self._native_server()
            self._aserver_sink = self.log.native.handle
        gpu = is_gpu(self.device)
        a.set_stream(torch.cuda.current_stream(self.device).cuda_stream if gpu else 0)
        a.updates = srv.updates
        t_start = time.time()
        u0 = srv.updates
        a.begin()
        while True:
            try:
                code, k, upd = a.run(int(cfg.checkpoint_every or 0) if cfg.checkpoint_dir else 0)
            except RuntimeError as e:
                raise RuntimeError(f"{e}; {self._ctrl_diag()}") from None
            srv.updates = int(upd)
            if code == h.ASYNC_DONE:
                break
            if code == h.ASYNC_CHECKPOINT:
                maybe_checkpoint(cfg, srv, srv.updates)
                continue
            reason = "reported an error" if code == h.ASYNC_ERROR_TOKEN else "busy and silent (watchdog)"
            if not drop_on_failure(cfg):
                raise WorkerFailure(int(k), reason + "; " + self._ctrl_diag())
            print(f"psx server: worker {k} failed ({reason}); continuing without it", flush=True)
            a.fail(int(k))
        if gpu:
            torch.cuda.synchronize(self.device)
        elapsed = time.time() - t_start
        n = srv.updates - u0
        return {"rounds": int(srv.tracker.min_clock()), "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": n / elapsed if elapsed > 0 else 0.0, "max_vc_gap": int(srv.tracker.max_gap),
                "failed_workers": list(a.failed), "host_us_per_update": a.host_us_per_update, "native_server": True,
                "sparse_pulls": int(a.sparse_pulls), "dense_pulls": int(a.dense_pulls),
                "data_plane": "peer" if peer else ("rccl" if self._hp2p is None else "host")}

    def _worker_loop_lanes(self) -> dict:
        """This rank's workers as lanes of ONE persistent launch (LanesLoop.run_async_remote,
        csrc/kernels/lanes_async.hip in remote mode): each worker solves on its own XCD
        when its weights arrive, and the host loop pushes its delta to the server (p2p
        peer 0) with its token, receives the weights of every release the server
        announces on this rank's reply queue, and logs the worker rows the lanes
        evaluate (WorkerTrainingProcessor.java:63-98, ServerProcessor.java:143-183)."""
        cfg, W = self.cfg, self.workers
        h = _native.hip()
        lp = getattr(self, "_alanes", None)
        if lp is None:
            lp = self._alanes_build()
        else:
            lp.set_sink(self.log.native.handle)
        for i, w in enumerate(W):
            lp.set_next_local(i, int(w.source.next_local))
            lp.set_seen_at_solve(i, int(w._seen_at_solve))
        peer = getattr(self, "_peer", False)
        p2p = None if peer else (self._hp2p if self._hp2p is not None else h.RcclP2P(self.comm.c))
        if not hasattr(self, "_comm_stream"):
            self._comm_stream = torch.cuda.Stream(self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        t_start = time.time()
        deadline_ms = (t_start + cfg.max_wallclock_s) * 1000.0 if cfg.max_wallclock_s else 0.0
        iters = int(cfg.max_iters) if cfg.max_iters else 1 << 40
        try:
            n = int(lp.run_async_remote(p2p, self._ctrl.handle, self._reply.handle, iters, stream,
                                        self._comm_stream.cuda_stream, float(cfg.worker_timeout_s), deadline_ms))
        except RuntimeError as e:
            raise RuntimeError(f"{e}; {self._ctrl_diag()}") from None
        torch.cuda.synchronize(self.device)
        lp.poll_errors()
        for i, w in enumerate(W):
            w.source.next_local = int(lp.next_local(i))
            w._seen_at_solve = int(lp.seen_at_solve(i))
            if w.ring.XT is not None:
                w.ring.xt_stale = True
        if self.log is not None:
            self.log.drain()
        elapsed = time.time() - t_start
        return {"rounds": n // max(1, len(W)), "updates": n, "elapsed_s": elapsed, "async_lanes": True,
                "data_plane": "peer" if peer else "host", "host_us_per_update": float(lp.host_us_per_update)}

    def _alanes_build(self):
        """This rank's asynchronous lanes loop (created once): every worker of the rank
        a lane of one persistent launch, on consecutive XCDs."""
        lp = getattr(self, "_alanes", None)
        if lp is None:
            cfg, W, sp = self.cfg, self.workers, self.spec
            h = _native.hip()
            from ..ops.lr import Fragments

            o = cfg.solver
            sc = h.SolverCfg()
            sc.K, sc.F, sc.Fp, sc.P, sc.cap = sp.K, sp.F, sp.Fp, sp.P, W[0].ring.cap
            sc.iters, sc.hist, sc.ls_max = o.iters, o.hist, o.ls_max
            sc.mode = 1 if o.mode == "gd" else 0
            sc.center, sc.zero_const = int(o.center), int(o.zero_const)
            sc.nslots, sc.gd_lr, sc.tol = o.nslots, o.gd_lr, o.tol
            ds, ev = W[0].source.ds, self.evalset
            self._alanes_frags = [Fragments(sp, self.device), Fragments(sp, self.device)]
            d = dict(scfg=sc, dsX=ds.X.data_ptr(), dsy=ds.y.data_ptr(), ds_rows=int(ds.rows), N=int(cfg.num_workers),
                     per_iter_rows=cfg.rows_per_iter if cfg.stream_mode == "per_iter" else 0,
                     p_ms=float(cfg.producer_time_per_event), epochs=int(cfg.epochs), t0_ms=self.t0 * 1000.0,
                     k=[w.k for w in W], X=[w.ring.X.data_ptr() for w in W], y=[w.ring.y.data_ptr() for w in W],
                     window=[w.window.handle for w in W], w=W[0].w.data_ptr(), lr=float(cfg.lr),
                     shi=[f.hi.data_ptr() for f in self._alanes_frags], slo=[f.lo.data_ptr() for f in self._alanes_frags],
                     sb=[f.b.data_ptr() for f in self._alanes_frags], Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=ev.T,
                     sink=self.log.native.handle, api=_native.host.capi(), log_server=0,
                     log_workers=int(cfg.log_workers), new_rows=int(cfg.iter_new_rows),
                     new_frac=float(cfg.iter_new_frac), new_cap=int(cfg.iter_new_cap), new_ramp=int(cfg.iter_new_ramp), log_worker=-1,
                     delay_us=[int(round(float(cfg.inject_worker_delay_ms.get(w.k, 0.0)) * 1000.0)) for w in W],
                     # ranks sharing one GPU (the one-GPU rehearsals): worker rank i's lanes on XCDs
                     # i*wpr ..; on its own GPU a rank's lanes start at XCD 0 and may take all 8 (no
                     # transfer kernel runs beside the persistent launch: the pushes / pulls are the
                     # lanes' own stores (peer plane) or host staging by the DMA engines)
                     xcd0=(self.worker_id * len(W)) if oversubscribed() else 0)
            d.update(ev.ell_args())
            lp = h.LanesLoop(d, None)
            lp.set_idle_wait(float(cfg.idle_wait_s))
            self._alanes = lp
        return lp

    def _worker_loop(self) -> dict:
        cfg, wk = self.cfg, self.worker
        tok = _native.host.CtrlToken()
        tok.worker = wk.k
        comm = self.comm
        gpu = is_gpu(self.device)
        done = torch.cuda.Event() if gpu else None

        hp = self._hp2p  # no RCCL communicator: the host shared-memory data plane

        def _stream():
            return torch.cuda.current_stream(self.device).cuda_stream if gpu else 0

        def send(t):
            if comm is not None:
                comm.send(t, 0)
            else:
                hp.send(t.data_ptr(), t.numel(), _p2p_dtype(t), 0, _stream())

        def recv(t):
            if comm is not None:
                comm.recv(t, 0)
            else:
                hp.recv(t.data_ptr(), t.numel(), _p2p_dtype(t), 0, _stream())

        KP = self.spec.KP if self.wide else 0
        if self.sparse_pull:  # receive buffers of the largest pull the log can send
            cap = pull_log_capacity(self._umax)
            pids = torch.zeros(cap, dtype=torch.int32, device=self.device)
            pvals = torch.zeros(cap * KP, dtype=torch.float32, device=self.device)

        def pull():
            """The weights of the next clock: dense, or (sparse pull) the log entries
            since the last pull applied to this worker's replica (w += lr * delta)."""
            if not self.sparse_pull:
                recv(wk.w)
                return
            r = self._reply.pop(600.0)
            if r is None:
                raise TimeoutError(f"worker {wk.k}: no release from the server for 600 s")
            if r.kind == 0:
                recv(wk.w)
                return
            n, l1 = int(r.n), int(r.aux)
            if l1:
                recv(pids[:l1])
                recv(pvals[: l1 * KP])
            if n > l1:
                recv(pids[l1:n])
                recv(pvals[l1 * KP: n * KP])
            if gpu:
                _native.hip().log_apply(wk.w.data_ptr(), pids.data_ptr(), pvals.data_ptr(), n, KP, float(cfg.lr),
                                        torch.cuda.current_stream(self.device).cuda_stream)
            else:
                idx = (pids[:n].long() * KP).unsqueeze(1) + torch.arange(KP).unsqueeze(0)
                wk.w.index_add_(0, idx.reshape(-1), pvals[: n * KP] * cfg.lr)

        pull()
        if gpu and not wk.wide:
            from ..runtime.roles import SideStream

            wk.side = SideStream(self.device, force=True)
        wk.vc = self._next_vc  # 0, or the server's clock for this worker on a later run
        max_iters = cfg.inject_worker_stop.get(wk.k) or cfg.max_iters or 1 << 62
        t_start = time.time()
        it = 0
        while True:
            wk.ingest()
            while not wk.ready():
                time.sleep(0.001)
                wk.ingest()
            try:
                delta = wk.solve()
            except WorkerFailure as e:  # report, then leave the protocol (the server retires or aborts)
                tok.kind, tok.vc, tok.n = KIND_ERROR, wk.vc, 0
                self._ctrl.push(tok, 600.0)
                print(f"psx worker {wk.k}: {e}", flush=True)
                return {"rounds": it, "updates": it, "failed": True}
            if gpu:
                done.record(torch.cuda.current_stream(self.device))  # the delta is complete here
            early = comm is not None and not self.sparse_push
            if early:  # stream-ordered RCCL send, enqueued now: it moves as soon as the server posts the recv
                send(delta)
            # the local model's row (LogisticRegressionTaskSpark.java:186) on the side
            # stream: it overlaps the push/pull instead of delaying them
            wk.log_eval(self.log)
            it += 1
            final = it >= max_iters or (cfg.max_wallclock_s and time.time() - t_start >= cfg.max_wallclock_s) or (
                not cfg.max_iters and not cfg.max_wallclock_s and wk.source.exhausted)
            tok.vc = wk.vc
            tok.kind = KIND_FINAL if final else KIND_DELTA
            tok.aux = wk.tuples_seen
            if gpu:
                # the token says "my delta is complete": the server serves tokens in
                # arrival order, so it must not wait on a delta still being computed.
                # Poll this solve's completion event (no full stream synchronisation:
                # the evaluation row enqueued behind it keeps running)
                while not done.query():
                    pass
            U = wk.solver.host_count() if self.sparse_push else 0
            tok.n = U
            if not self._ctrl.push(tok, 600.0):
                raise TimeoutError("worker: control queue full for 600 s")
            if self.sparse_push:  # (ids, values) of the window's features only
                KP = self.spec.KP
                if U:
                    send(delta.uniq[:U])
                send(delta.dloc[: KP + U * KP])
            elif not early:  # (host transport: written after the token, read when the server serves it)
                send(delta)
            if final:
                break
            pull()  # stream-ordered: the next solve enqueued below waits for it on the device
            wk.vc += 1
            if self.log is not None:
                self.log.drain()
        self._next_vc = wk.vc + 1
        if is_gpu(self.device):
            torch.cuda.synchronize(self.device)
        elapsed = time.time() - t_start
        return {"rounds": it, "updates": it, "elapsed_s": elapsed}


def _p2p_dtype(t: torch.Tensor) -> int:
    from .comm import _dtype

    return _dtype(t)


def run_distributed(cfg: PSConfig, cpu: bool = False, train=None, test=None) -> dict:
    rank, world, device = init_from_env(cpu)
    try:
        eng = DistEngine(cfg, rank, world, device, train=train, test=test)
        return eng.run()
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
