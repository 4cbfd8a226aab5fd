"""In-process parameter-server engine: server + N workers on ONE device.

This is the degenerate case of the multi-GPU RCCL schedules (psx.parallel.dist):
push/pull become device-local copies, ordering comes from HIP streams and
events.  It is what a single MI355X (or the CPU, for tests / the plumbing
config) runs, and it exercises exactly the same roles, tracker, buffer, solver
and logging code as the distributed engine.

* BSP (c = 0): lock-step rounds on one stream -- every worker solves, the server
  applies the summed deltas (lr = 1/N), evaluates, and broadcasts.
* SSP (c = D > 0) / ASP (c = -1): one HIP stream per worker; the server applies
  deltas in completion order -- the analogue of the single-partition
  GRADIENTS_TOPIC (ServerApp.java:36-38) -- and releases workers per the
  vector-clock tracker.  On a GPU one host thread launches every worker's solve
  and polls completion events (_run_async_events); with injected stragglers, or
  on the CPU, each worker runs on its own host thread (_run_async).
"""
from __future__ import annotations

import dataclasses
import json
import os
import queue
import threading
import time

import torch

from .. import _native
from ..models.logreg import ModelSpec
from ..models.wide import WideSpec
from ..ops.lr import is_gpu, stream_handle
from ..utils import data as data_mod
from ..utils.checkpoint import flush_checkpoints, maybe_checkpoint, maybe_resume
from ..utils.logsink import LogSink, summarize
from ..utils.trace import Tracer
from .config import PSConfig, cadence_free
from .faults import WorkerFailure, drop_on_failure
from .roles import EvalPair, ServerRole, WorkerRole, make_evalset


def _wants_wide(cfg: PSConfig, train) -> bool:
    if cfg.model in ("dense", "wide"):
        return cfg.model == "wide"
    if train is not None:
        return not hasattr(train, "X")  # a SparseDataset
    if data_mod.is_libsvm_path(cfg.train_path):
        return True
    return cfg.num_features is not None and cfg.num_features > 2048


def load_datasets(cfg: PSConfig, train=None, test=None):
    """Datasets + model spec: dense CSV/binary rows -> ModelSpec, sparse
    (LIBSVM / SparseDataset) rows -> WideSpec."""
    if _wants_wide(cfg, train):
        if cfg.dtype != "bf16":
            raise ValueError("--dtype fp32 applies to the dense model (the wide model's values are bf16)")
        if train is None:
            train = data_mod.load_libsvm(cfg.train_path, num_features=cfg.num_features)
        if test is None and cfg.test_path:
            test = data_mod.load_libsvm(cfg.test_path, num_features=cfg.num_features)
        F = max(train.num_features, test.num_features if test is not None else 0)
        if cfg.num_features is not None:
            F = int(cfg.num_features)
        train.num_features = F  # hashed width: the larger of the two files' index ranges
        if test is not None:
            test.num_features = F
        if cfg.sigmoid:
            K = 1
        elif cfg.num_classes is not None:
            K = int(cfg.num_classes)
        else:
            mx = int(train.y.max())
            if test is not None:
                mx = max(mx, int(test.y.max()))
            K = max(2, mx + 1)
        return WideSpec(F, K), train, test
    if train is None:
        train = data_mod.load_any(cfg.train_path, header=cfg.header, label_col=cfg.label_col,
                                  num_features=cfg.num_features, dtype=cfg.dtype)
    if test is None and cfg.test_path:
        test = data_mod.load_any(cfg.test_path, header=cfg.header, label_col=cfg.label_col,
                                 num_features=train.num_features)
    train = train.as_dtype(cfg.dtype)  # the training rows in the run's feature dtype (test rows: bf16)
    if cfg.num_classes is not None:
        K = int(cfg.num_classes)
    else:
        mx = int(train.y.max())
        if test is not None:
            mx = max(mx, int(test.y.max()))
        K = max(2, mx + 1)
    spec = ModelSpec(train.num_features, K)
    return spec, train, test


class LocalEngine:
    def __init__(self, cfg: PSConfig, device="cpu", train=None, test=None, log: LogSink | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.spec, train, test = load_datasets(cfg, train, test)
        self.train = train.to(self.device)
        self.evalset = make_evalset(self.spec, test, self.device)
        if log is None:
            wp = f"{cfg.log_dir}/logs-worker.csv" if cfg.logging else None
            sp = f"{cfg.log_dir}/logs-server.csv" if cfg.logging else None
            log = LogSink(self.spec.eval_classes, self.device, wp, sp, to_stdout=not cfg.logging and cfg.verbose)
        self.log = log
        self.tracer = Tracer(cfg.trace_path, 0, self.device,
                             f"{cfg.log_dir}/logs-perf.csv" if cfg.perf_log else None)
        if cfg.solver.persist and cfg.num_workers > 1:
            # the persistent solve needs its workgroups co-resident: one worker only.
            # Measured: two workers' persistent launches on their own XCDs deadlock (each
            # launch's gap / riding workgroups wait for CUs of the other's XCD, and the
            # dispatcher places a launch's workgroups in order) -- profiles/r02_v5
            cfg.solver = dataclasses.replace(cfg.solver, persist=False)
        if cfg.solver.persist is None and cfg.num_workers == 1 and is_gpu(self.device):
            # a lone worker has the GPU to itself: the persistent solve (one XCD) is the
            # fastest small-window solve on MI355X (profiles/r02_v5); unsupported shapes
            # (rows mode, fp32 rows, > 1024 features) keep the chain inside the solver
            cfg.solver = dataclasses.replace(cfg.solver, persist=True)
        if cfg.num_workers > 4 and is_gpu(self.device) and cfg.solver.tail:
            # many concurrent workers' solves share the CUs: no launch may wait for
            # workgroups of its own that other workers' launches keep from being placed
            # (8 workers' tail launches, 33 one-CU workgroups each, did -- fresh windows
            # need many line-search retries).  Up to 4 workers (132 tail workgroups) keep
            # the tail: 14.4k / 20.2k updates/s with it against 9.2k / 15.2k without
            # (profiles/r02_v5/workers_*.jsonl)
            cfg.solver = dataclasses.replace(cfg.solver, tail=False)
        if cfg.solver.use_graph is None and cfg.num_workers > 2:
            # many in-process workers share this process's launch thread: one graph
            # replay per solve beats 8 eager launches there (bench.py --workers 8:
            # 17.7k vs 13.4k updates/s); a lone worker is GPU-bound and runs eagerly
            cfg.solver = dataclasses.replace(cfg.solver, use_graph=True)
        w0 = self.spec.init(cfg.init, seed=cfg.seed, device=self.device)
        self.server = ServerRole(self.spec, cfg, self.device, self.evalset, w0)
        self.t0 = time.time()
        # one worker: its solve's cooperating workgroups on XCD 0 (in-L2 hand-offs); several
        # concurrent workers: spread over the XCDs (a one-XCD launch's gap workgroups would
        # wait for CUs the other workers' solves hold -- the ASP runs timed out that way)
        xcd = 0 if cfg.num_workers == 1 else -1
        self.workers = [WorkerRole(k, self.spec, cfg, self.device, self.train, self.evalset, t0=self.t0, xcd=xcd)
                        for k in range(cfg.num_workers)]
        self.rounds = 0
        # worker 0's rows and the server rows: one eval pass (sequential consistency,
        # or one worker, which every model runs lock-step)
        if (cfg.consistency_model == 0 or cfg.num_workers == 1) and cfg.pair_eval:
            EvalPair(self.server, self.workers[0])
        self.failed: set[int] = set()
        self.left: set[int] = set()  # workers that left cleanly (--inject_worker_stop)
        self._trace_cap = 1024  # device trace ring of the lanes loops (rounds / tickets between takes)
        if maybe_resume(cfg, self.server, self.workers):
            self.rounds = int(self.server.tracker.min_clock())
            self.failed = {k for k in range(cfg.num_workers) if not self.server.tracker.is_live(k)}

    # ------------------------------------------------------------------
    def _stop(self, iters_done: int, t_start: float, exhausted_since: float | None) -> bool:
        c = self.cfg
        if c.max_iters and iters_done >= c.max_iters:
            return True
        if c.max_wallclock_s and time.time() - t_start >= c.max_wallclock_s:
            return True
        if not c.max_iters and exhausted_since is not None and time.time() - exhausted_since >= c.idle_exit_s:
            return True
        return False

    def run(self, close_log: bool = True, summary: bool = True) -> dict:
        """Run until the configured stop (max_iters / wall clock / data).  close_log
        False: the log sink stays open for a later run (its rows are flushed).
        summary False: no headline numbers from the log book (a scan of every row
        logged so far: bench.py computes them outside its timed region)."""
        t_entry = time.time()
        if getattr(self, "train_start_ms", None) is None:  # epoch ms when training first began
            self.train_start_ms = time.time() * 1000.0
        live = [w for w in self.workers if w.k not in self.failed]
        if self.cfg.consistency_model == 0 or len(live) == 1:
            # with a single worker every consistency model releases that worker right
            # after its delta is applied (tracker: BSP, SSP(D) and ASP coincide), so the
            # lock-step loop runs it without the thread / queue / event hand-offs
            out = self._run_bsp()
        elif self._async_lanes_ok():
            out = self._run_async_lanes()
        elif self._wide_lanes_ok():  # the wide model's workers: one solve launch per round
            out = self._run_wide_lanes()
        # the Python SSP / ASP schedulers: the runs the native lanes loop cannot take --
        # CPU runs, the wide model, fp32 rings, windows over 8,192 rows, shards shorter than
        # a ring.  Their dense-GPU branch stays exercised by tests/test_gpu_engine.py
        # (PSX_ASYNC_LANES=0: the crash-retirement test on the event scheduler)
        elif self._event_scheduler():
            out = self._run_async_events()
        else:
            out = self._run_async()
        flush_checkpoints(self.cfg)
        if not out.get("lanes"):  # (the multi-lane loop raises on a device error itself)
            for w in self.workers:
                if w.k not in self.failed:
                    w.check_device_health()
        if close_log:
            self.log.close()
            self.tracer.close()
        t_sum = time.time()
        if summary and self.log.book is not None:
            out.update(summarize(self.log.book))
        if "phases_ms" in out:
            ph = out["phases_ms"]
            ph["summary"] = round((time.time() - t_sum) * 1e3, 3)
            # the whole call less its loop phases: the Python around the native loop
            ph["python"] = round((time.time() - t_entry) * 1e3 - ph.get("rounds", 0.0) - ph.get("tail", 0.0)
                                 - ph.get("sync", 0.0) - ph["summary"], 3)
        out["max_vc_gap"] = int(self.server.tracker.max_gap)
        out["failed_workers"] = sorted(self.failed)
        if self.left:
            out["left_workers"] = sorted(self.left)
        return out

    def _worker_failed(self, e: Exception, k: int):
        """Policy on a failed worker: retire it (drop) or abort the run (fail)."""
        if not drop_on_failure(self.cfg):
            raise e if isinstance(e, WorkerFailure) else WorkerFailure(k, repr(e))
        self.failed.add(k)
        released = self.server.tracker.retire(k)
        print(f"psx: worker {k} failed ({e}); continuing with {self.server.tracker.num_live} workers", flush=True)
        return released

    # ------------------------------------------------------------------
    def _native_bsp_ok(self) -> bool:
        """The native round loop (csrc/runtime/bsp_loop.h) runs this BSP run: one
        dense GPU worker whose rows ride in its solves, a bounded run, and nothing
        that needs Python between rounds (tracing, checkpoints, injected faults,
        a wall-clock or stream-driven cadence)."""
        c = self.cfg
        if os.environ.get("PSX_NATIVE_BSP", "1") == "0" or not is_gpu(self.device):
            return False
        if len(self.workers) != 1 or self.failed or self.server.pair is None or not self.server.pair.ride_ok:
            return False
        wk, srv = self.workers[0], self.server
        if wk.wide or not srv.pair.shared or wk.evalset is None or self.tracer.enabled:
            return False
        if not c.max_iters or c.max_wallclock_s or not cadence_free(c) or c.checkpoint_dir or c.inject_worker_delay_ms \
                or c.inject_worker_crash or c.inject_worker_stop:
            return False
        if c.stream_mode == "per_iter":
            if wk.source.rows_per_iter <= 0:
                return False
        elif not wk.source.p_ms > 0:
            return False
        ring = wk.ring
        if ring.f32 or ring.XT is None or wk.source.ds.X.dtype != torch.bfloat16:
            return False
        return wk.solver.can_ride(ring, srv.w)

    def _lanes_ok(self) -> bool:
        """The multi-lane round loop (csrc/runtime/lanes_loop.h) runs this BSP run:
        1..8 dense GPU workers with bf16 rings of <= 8192 rows, ONE launch per round
        (every worker's solve on its own XCD, the update, the previous round's
        evaluation rows).  Runs that need Python between rounds (tracing, injected
        faults) use the loops below.  The tuple-driven cadence (--iter_new_*) and
        the producer clock run natively: a round waits until every lane saw its
        new tuples.  Injected stragglers sleep on the device (LaneRound.delay_us);
        an injected crash ends a chunk of rounds at its iteration (_run_bsp_lanes)."""
        return self._lanes_shape_ok()

    def _async_lanes_ok(self) -> bool:
        """SSP / ASP in the native asynchronous lanes loop (LanesLoop.run_async: ONE
        persistent launch, every worker released by the C++ tracker, updates serial
        in arrival order on the device): the lanes loop's shapes, plus every
        worker's shard at least its ring (a release's pending rows span at most one
        epoch wrap).  Injected straggler delays run on the device, injected crashes /
        clean leaves in the host loop (LanesLoop.set_injection); tracing keeps the
        Python schedulers."""
        if os.environ.get("PSX_ASYNC_LANES", "1") == "0" or not self._lanes_shape_ok():
            return False
        W = [w for w in self.workers if w.k not in self.failed]
        return all(w.source.ds.rows // max(1, self.cfg.num_workers) >= w.ring.cap for w in W)

    def _lanes_shape_ok(self) -> bool:
        # (cached per engine: its workers' rings, sources and solver options are fixed at
        # construction -- 16 us of Python per call otherwise, in every bench.py step
        # window; profiles/r05/README.md section 10)
        key = (tuple(sorted(self.failed)), os.environ.get("PSX_NATIVE_LANES", "1"), self.evalset is None,
               self.cfg.stream_mode, self.cfg.rows_per_iter, self.cfg.producer_time_per_event)
        hit = getattr(self, "_shape_ok", None)
        if hit is not None and hit[0] == key:
            return hit[1]
        ok = self._lanes_shape_check()
        self._shape_ok = (key, ok)
        return ok

    def _lanes_shape_check(self) -> bool:
        c = self.cfg
        if os.environ.get("PSX_NATIVE_LANES", "1") == "0" or not is_gpu(self.device):
            return False
        W = [w for w in self.workers if w.k not in self.failed]
        if not W or len(W) > 8 or self.evalset is None:
            return False
        sp = self.spec
        for w in W:
            if w.wide or w.ring.f32 or w.source.ds.X.dtype != torch.bfloat16:
                return False
            if (w.source.mode == "per_iter" and w.source.rows_per_iter <= 0) or (
                    w.source.mode != "per_iter" and not w.source.p_ms > 0):
                return False
        if w.solver.opts.nslots >= 64 or w.solver.opts.hist > 16:
            return False
        return bool(_native.hip().lanes_supported(sp.Fp, sp.K, W[0].ring.cap))

    def _lanes_loop(self, W):
        """The native loop bound to this engine's rings / windows / server (built
        once per set of workers; the metrics sink is rebound per run)."""
        key = tuple(w.k for w in W)
        lp = getattr(self, "_lanes", None)
        if lp is not None and self._lanes_key == key:
            bound = (self.log.native.handle, float(self.cfg.lr))
            if bound != getattr(self, "_lanes_bound", None):  # (rebound only when they change)
                lp.set_sink(bound[0])
                lp.set_lr(bound[1])
                self._lanes_bound = bound
            return lp
        from ..ops.lr import Fragments

        h, sp, cfg, srv = _native.hip(), self.spec, self.cfg, self.server
        o = W[0].solver.opts
        sc = h.SolverCfg()
        sc.K, sc.F, sc.Fp, sc.P, sc.cap = sp.K, sp.F, sp.Fp, sp.P, W[0].ring.cap
        sc.iters, sc.hist, sc.ls_max = o.iters, o.hist, o.ls_max
        sc.mode = 1 if o.mode == "gd" else 0
        sc.center, sc.zero_const = int(o.center), int(o.zero_const)
        sc.nslots, sc.gd_lr, sc.tol = o.nslots, o.gd_lr, o.tol
        self._lane_frags = [Fragments(sp, self.device) for _ in range(3)]  # (3: overlapped rounds)
        src0, ev = W[0].source, self.evalset
        d = dict(scfg=sc, dsX=src0.ds.X.data_ptr(), dsy=src0.ds.y.data_ptr(), ds_rows=int(src0.ds.rows),
                 N=int(cfg.num_workers), per_iter_rows=src0.rows_per_iter if src0.mode == "per_iter" else 0,
                 p_ms=float(src0.p_ms), epochs=int(src0.epochs), t0_ms=float(src0.t0) * 1000.0,
                 k=[w.k for w in W], X=[w.ring.X.data_ptr() for w in W], y=[w.ring.y.data_ptr() for w in W],
                 window=[w.window.handle for w in W], w=srv.w.data_ptr(), lr=float(cfg.lr),
                 shi=[f.hi.data_ptr() for f in self._lane_frags], slo=[f.lo.data_ptr() for f in self._lane_frags],
                 sb=[f.b.data_ptr() for f in self._lane_frags], scoff=0, Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(),
                 T=ev.T, sink=self.log.native.handle, tracker=srv.tracker.handle, api=_native.host.capi(),
                 new_rows=int(cfg.iter_new_rows), new_frac=float(cfg.iter_new_frac), new_cap=int(cfg.iter_new_cap), new_ramp=int(cfg.iter_new_ramp),
                 # the asynchronous loop: server rows on the lowest live worker's deltas
                 # (ServerProcessor.java:154), straggler delays on the device
                 log_worker=min(w.k for w in W),
                 delay_us=[int(round(float(cfg.inject_worker_delay_ms.get(w.k, 0.0)) * 1000.0)) for w in W])
        d.update(ev.ell_args())  # (the asynchronous lanes' evaluation reads the sparse test rows)
        lp = h.LanesLoop(d, None)
        if self.tracer.enabled:  # --trace / --perf_log: phase times recorded by the kernels
            lp.set_trace(self._trace_cap)
        elif os.environ.get("PSX_LANES_TRACE_OUT"):  # (tools: the device phase stamps of every round)
            lp.set_trace(8192)
        lp.set_idle_wait(float(cfg.idle_wait_s))
        if os.environ.get("PSX_INJECT_SPIN_TIMEOUT"):  # tests: "round:polls"
            rr, sp_ = os.environ["PSX_INJECT_SPIN_TIMEOUT"].split(":")
            lp.inject_spin_timeout(int(rr), int(sp_))
        self._lanes, self._lanes_key = lp, key
        self._lanes_bound = (self.log.native.handle, float(cfg.lr))
        return lp

    def _lane_trace(self, lp, stream, ups: float):
        """--trace / --perf_log of a lanes loop: the phase times its kernels recorded on the
        device since the last call, placed on the host timeline by one clock probe."""
        rows = lp.trace_take(stream)
        if rows:
            self.tracer.lane_rows(rows, lp.clock_ref(stream), ups)

    def _run_bsp_lanes(self, max_rounds: int | None = None, t_start: float | None = None) -> dict:
        """BSP rounds of every live worker in the native multi-lane loop: one launch
        per round, no Python per round.  An unbounded run (max_iters 0: until the
        data or the wall clock says stop) and checkpoints run in chunks of rounds.
        An injected crash (--inject_worker_crash K:ITER) ends a chunk at round ITER of
        worker K: the failure policy then aborts the run or retires K, and the run
        goes on with the other workers in a loop of their own (max_rounds: the rest
        of max_iters; roles.py WorkerRole.compute fails at the same iteration)."""
        cfg, srv = self.cfg, self.server
        W = [w for w in self.workers if w.k not in self.failed]
        for w in W:
            w.w = srv.w
            w.ring.flush()
        if srv.pair is not None:
            srv.pair.flush(self.log)  # nothing may be pending from an earlier run
        lp = self._lanes_loop(W)
        # (the loop's own counters are current unless something moved the roles' since
        # its last run -- a resume or a test: a pybind call per worker saved per run)
        synced = getattr(self, "_lanes_synced", None)
        now = [(int(w.source.next_local), int(w._seen_at_solve)) for w in W]
        if synced is None or synced[0] is not lp or synced[1] != now:
            for i, (nl, ss) in enumerate(now):
                lp.set_next_local(i, nl)
                lp.set_seen_at_solve(i, ss)
        stream = stream_handle(self.device)
        t_start = time.time() if t_start is None else t_start
        deadline_ms = (t_start + cfg.max_wallclock_s) * 1000.0 if cfg.max_wallclock_s else 0.0
        r0 = r = self.rounds
        u0 = srv.updates
        limit = cfg.max_iters if max_rounds is None else max_rounds
        crashing = [w for w in W if w.crash_at is not None]
        crashed = []
        chunk = 256
        ck = bool(cfg.checkpoint_dir and cfg.checkpoint_every)
        if ck:
            chunk = max(1, int(cfg.checkpoint_every))
        exhausted_since = None
        try:
            while True:
                # checkpoints fire at multiples of checkpoint_every: a run that starts
                # between two of them first runs up to the next one
                todo = chunk - (r % chunk) if ck else chunk
                if limit:
                    todo = min(todo, limit - (r - r0))
                    if todo <= 0:
                        break
                if lp.all_exhausted:  # the streams ended: stale windows for idle_exit_s more
                    exhausted_since = exhausted_since or time.time()
                if self._stop(r - r0, t_start, exhausted_since):
                    break
                if crashing:  # the next injected crash ends this chunk
                    crashed = [w for w in crashing if w.iters >= w.crash_at]
                    if crashed:
                        break
                    todo = min(todo, min(w.crash_at - w.iters for w in crashing))
                self._t_lp_run_ns = time.perf_counter_ns()  # (tools/round_timeline.py)
                n = int(lp.run(int(todo), int(r), stream, float(cfg.idle_wait_s), deadline_ms))
                r += n
                if self.tracer.enabled:  # (a synchronisation per chunk of rounds: tracing only)
                    self._lane_trace(lp, stream, (srv.updates + n * len(W) - u0) / max(1e-9, time.time() - t_start))
                # the roles' counters advance with every chunk, so a checkpoint taken
                # here carries the updates / clocks of the rounds it covers
                srv.updates += n * len(W)
                for i, w in enumerate(W):
                    w.source.next_local = int(lp.next_local(i))
                    w._seen_at_solve = int(lp.seen_at_solve(i))
                    w.vc = r
                    w.iters += n
                if n:
                    maybe_checkpoint(cfg, srv, r, W)
                if n < todo:  # a worker's stream is exhausted and its window empty, or the deadline
                    break
            t_loop = time.time()
            self._t_lp_done_ns = time.perf_counter_ns()
            lp.flush(stream)
            # stream-ordered behind the rounds: the last local solve's loss / delta for code
            # that reads the roles, and the Python-side evaluation fragments of the global
            # model (the native update rewrote w); ONE synchronisation covers them all
            ca = getattr(self, "_lanes_copy_args", None)  # (the roles' tensors outlive the loop)
            if ca is None or ca[0] is not lp:
                ca = (lp, [w.solver.loss.data_ptr() for w in W], [w.solver.delta.data_ptr() for w in W])
                self._lanes_copy_args = ca
            lp.copy_out_all(ca[1], ca[2], stream)
            if srv.frag is not None:
                srv.frag.refresh(srv.w)
            if os.environ.get("PSX_LANES_TRACE_OUT") and not self.tracer.enabled:  # one JSON line per call
                with open(os.environ["PSX_LANES_TRACE_OUT"], "a") as fh:
                    fh.write(json.dumps({"rank": 0, "rows": [list(r) for r in lp.trace_take(stream)]}) + "\n")
            t_enq = time.time()
            torch.cuda.synchronize(self.device)
            t_sync = time.time()
            lp.poll_errors()  # a device error of the last rounds (the loop polls without syncs)
        except RuntimeError as e:
            if "cross-workgroup wait timed out" in str(e):
                raise WorkerFailure(W[0].k, str(e)) from e
            raise
        for i, w in enumerate(W):
            w._seen_at_solve = int(lp.seen_at_solve(i))
            if w.ring.XT is not None:
                w.ring.xt_stale = True  # the round kernel writes the row-major ring only
        self._lanes_synced = (lp, [(int(w.source.next_local), int(w._seen_at_solve)) for w in W])
        self.native_host_us_per_round = float(lp.host_us_per_round)
        self.native_host_phases_us = [round(float(x), 2) for x in lp.host_phases_us()]
        self.rounds = r
        if crashed:
            for w in crashed:  # fail: raises; drop: retired, the others go on without it
                self._worker_failed(WorkerFailure(w.k, f"injected crash at iteration {w.iters}"), w.k)
            rest = (limit - (r - r0)) if limit else None
            if (rest is None or rest > 0) and any(w.k not in self.failed for w in self.workers):
                out = self._run_bsp_lanes(rest if limit else None, t_start)
                out["updates_per_s"] = (srv.updates - u0) / max(1e-9, time.time() - t_start)
                return out
        elapsed = time.time() - t_start
        return {"rounds": r, "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": (srv.updates - u0) / elapsed if elapsed > 0 else 0.0, "native_loop": True,
                "lanes": len(W), "hand_off_scope": int(lp.hand_off_scope),
                # host wall clock of the run's parts (ms): rounds enqueued, tail enqueued, device done
                "phases_ms": {"rounds": round((t_loop - t_start) * 1e3, 3), "tail": round((t_enq - t_loop) * 1e3, 3),
                              "sync": round((t_sync - t_enq) * 1e3, 3)}}

    def _run_async_lanes(self) -> dict:
        """SSP / ASP of every live worker in ONE persistent launch
        (LanesLoop.run_async, csrc/kernels/lanes_async.hip): each worker solves on its
        own XCD as soon as the tracker releases it, pushes with a device ticket
        (updates serial in arrival order, ServerProcessor.java:143-183), and evaluates
        its local model (plus the global model on the logging worker, :154-165); the
        C++ tracker answers every delta from the host loop (MessageTracker.java:
        69-87).  max_iters: iterations per worker (max_iters x workers updates);
        unbounded runs and checkpoints run in chunks."""
        cfg, srv = self.cfg, self.server
        W = [w for w in self.workers if w.k not in self.failed]
        for w in W:
            w.ring.flush()
        if srv.pair is not None:
            srv.pair.flush(self.log)
        lp = self._lanes_loop(W)
        # (the loop's own counters are current unless something moved the roles' since
        # its last run -- a resume or a test: a pybind call per worker saved per run)
        synced = getattr(self, "_lanes_synced", None)
        now = [(int(w.source.next_local), int(w._seen_at_solve)) for w in W]
        if synced is None or synced[0] is not lp or synced[1] != now:
            for i, (nl, ss) in enumerate(now):
                lp.set_next_local(i, nl)
                lp.set_seen_at_solve(i, ss)
        stream = stream_handle(self.device)
        t_start = time.time()
        deadline_ms = (t_start + cfg.max_wallclock_s) * 1000.0 if cfg.max_wallclock_s else 0.0
        u0 = srv.updates
        clock0 = {w.k: int(srv.tracker.clock(w.k)) for w in W}
        clock_start = dict(clock0)
        total = int(cfg.max_iters) * len(W) if cfg.max_iters else 0
        inject = any(w.crash_at is not None for w in W) or bool(cfg.inject_worker_stop)
        crashed: list[WorkerFailure] = []
        ck = bool(cfg.checkpoint_dir and cfg.checkpoint_every)
        chunk = max(1, int(cfg.checkpoint_every)) if ck else 1 << 16
        if self.tracer.enabled:  # one device trace row per update: a chunk never outruns the trace ring
            chunk = min(chunk, self._trace_cap)
        done = 0
        gone: set[int] = set(self.left)  # workers that left (earlier runs) or crashed / left in an earlier chunk
        exhausted_since = None
        try:
            while True:
                todo = chunk - (srv.updates % chunk) if ck else chunk
                if total:
                    todo = min(todo, total - done)
                    if todo <= 0:
                        break
                if lp.all_exhausted:
                    exhausted_since = exhausted_since or time.time()
                if self._stop(done // max(1, len(W)), t_start, exhausted_since):
                    break
                # max_iters iterations per worker exactly (under ASP the fast workers would
                # otherwise take the slow ones' share): each lane's remaining share, also
                # across the chunks of a checkpointed run
                budget = ([0 if w.k in gone else
                           max(0, int(cfg.max_iters) - (int(srv.tracker.clock(w.k)) - clock_start[w.k])) for w in W]
                          if cfg.max_iters else 0)
                if inject:  # crashes / clean leaves: solves left before each (roles.py WorkerRole.compute)
                    crash = [max(0, w.crash_at - w.iters) if (w.crash_at is not None and w.k not in self.failed
                                                              and w.k not in gone) else -1 for w in W]
                    stop = [max(0, int(cfg.inject_worker_stop[w.k]) - w.iters)
                            if (w.k in cfg.inject_worker_stop and w.k not in gone) else -1 for w in W]
                    lp.set_injection(crash, stop, drop_on_failure(cfg))
                n = int(lp.run_async(int(todo), stream, float(cfg.worker_timeout_s), deadline_ms, budget))
                done += n
                srv.updates += n
                if self.tracer.enabled:
                    self._lane_trace(lp, stream, done / max(1e-9, time.time() - t_start))
                for i, w in enumerate(W):
                    w.source.next_local = int(lp.next_local(i))
                    w._seen_at_solve = int(lp.seen_at_solve(i))
                    w.vc = int(srv.tracker.clock(w.k))
                    w.iters += w.vc - clock0[w.k]
                    clock0[w.k] = w.vc
                if inject:
                    for k in lp.crashed:  # (the loop retired it already under drop, or stopped the run)
                        crashed.append(WorkerFailure(k, f"injected crash at iteration {self.workers[k].iters}"))
                    self.left.update(int(k) for k in lp.left)
                    gone.update(int(k) for k in lp.crashed)
                    gone.update(int(k) for k in lp.left)
                if n and ck:
                    maybe_checkpoint(cfg, srv, srv.updates, W)
                if crashed and not drop_on_failure(cfg):
                    break
                if n < todo:  # the streams ended, the deadline passed
                    break
            ca = getattr(self, "_lanes_copy_args", None)  # (the roles' tensors outlive the loop)
            if ca is None or ca[0] is not lp:
                ca = (lp, [w.solver.loss.data_ptr() for w in W], [w.solver.delta.data_ptr() for w in W])
                self._lanes_copy_args = ca
            lp.copy_out_all(ca[1], ca[2], stream)
            if srv.frag is not None:
                srv.frag.refresh(srv.w)
            torch.cuda.synchronize(self.device)
            lp.poll_errors()
        except RuntimeError as e:
            if "cross-workgroup wait timed out" in str(e):
                raise WorkerFailure(W[0].k, str(e)) from e
            raise
        for w in W:
            if w.ring.XT is not None:
                w.ring.xt_stale = True
        for e in crashed:
            if not drop_on_failure(cfg):
                raise e
            self.failed.add(e.worker)
            print(f"psx: worker {e.worker} failed ({e}); continuing with {srv.tracker.num_live} workers", flush=True)
        self.native_host_us_per_round = float(lp.host_us_per_update)
        self.native_host_busy_us_per_token = float(lp.host_busy_us_per_token)
        elapsed = time.time() - t_start
        self.rounds = int(srv.tracker.min_clock())
        return {"rounds": self.rounds, "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": (srv.updates - u0) / elapsed if elapsed > 0 else 0.0, "native_loop": True,
                "lanes": len(W), "async_lanes": True, "hand_off_scope": int(lp.hand_off_scope)}

    def _run_bsp_native(self) -> dict:
        """BSP rounds in the native loop: every round enqueued from C++ (producer,
        window, fused ingest, solve with the previous rows riding in it, the
        update fused into the solve, log records, tracker) -- no Python per round."""
        cfg, srv = self.cfg, self.server
        wk = self.workers[0]
        wk.w = srv.w
        wk.vc = self.rounds
        wk.ring.flush()
        srv.pair.flush(self.log)  # nothing may be pending from an earlier run
        src, ring, sp = wk.source, wk.ring, self.spec
        ev = wk.evalset
        d = dict(dsX=src.ds.X.data_ptr(), dsy=src.ds.y.data_ptr(), ds_rows=int(src.ds.rows), k=wk.k, N=src.N,
                 per_iter_rows=src.rows_per_iter if src.mode == "per_iter" else 0, p_ms=float(src.p_ms),
                 epochs=int(src.epochs), t0_ms=float(src.t0) * 1000.0, X=ring.X.data_ptr(), XT=ring.XT.data_ptr(),
                 y=ring.y.data_ptr(), cap=ring.cap, Fp=sp.Fp, K=sp.K, F=sp.F, window=wk.window.handle,
                 whi=wk.solver.frag.hi.data_ptr(), wlo=wk.solver.frag.lo.data_ptr(), wb=wk.solver.frag.b.data_ptr(),
                 loss=wk.solver.loss.data_ptr(), delta=wk.solver.delta.data_ptr(), w=srv.w.data_ptr(),
                 shi=srv.frag.hi.data_ptr(), slo=srv.frag.lo.data_ptr(), sb=srv.frag.b.data_ptr(),
                 scoff=srv.frag.coff, lr=float(cfg.lr), tracker=srv.tracker.handle, Xt=ev.X.data_ptr(),
                 yt=ev.y.data_ptr(), T=ev.T, acc=wk.scratch.acc.data_ptr(), ticket=wk.scratch.ticket.data_ptr(),
                 sink=self.log.native.handle, log_server=1, api=_native.host.capi())
        h = _native.hip()
        loop = h.BspLoop(wk.solver._native, None, d)
        loop.next_local = int(src.next_local)
        stream = stream_handle(self.device)
        t_start = time.time()
        r0 = self.rounds
        u0 = srv.updates
        n = int(loop.run(int(cfg.max_iters), int(r0), stream))
        loop.flush(stream)
        src.next_local = int(loop.next_local)
        r = r0 + n
        srv.updates += n
        wk.vc = r
        wk.iters += n
        wk._seen_at_solve = wk.tuples_seen
        self.native_host_us_per_round = float(loop.host_us_per_round)
        self.log.drain()
        torch.cuda.synchronize(self.device)
        elapsed = time.time() - t_start
        self.rounds = r
        return {"rounds": r, "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": (srv.updates - u0) / elapsed if elapsed > 0 else 0.0, "native_loop": True}

    def _run_bsp(self) -> dict:
        # one worker: the native loop around the one-XCD persistent solve beats the lanes
        # loop's one-lane launch (14.4-14.5k against 12.4-12.6k updates/s, profiles/r06/s37);
        # runs it cannot take (tracing, checkpoints, wall clock, cadence) stay on the lanes
        if len(self.workers) == 1 and self._native_bsp_ok():
            return self._run_bsp_native()
        if self._lanes_ok():
            return self._run_bsp_lanes()
        if self._native_bsp_ok():
            return self._run_bsp_native()
        if self._wide_lanes_ok():
            return self._run_wide_lanes()
        cfg, srv = self.cfg, self.server
        # bootstrap broadcast, vc 0 (ServerProcessor.java:75-87).  Under BSP every
        # worker pulls the same version right after the server update, and all
        # solves of a round finish (stream order) before the update, so the
        # workers' pulled copy IS the server tensor: no per-round copies.
        for w in self.workers:
            w.w = srv.w
            w.vc = self.rounds
        t_start = time.time()
        exhausted_since = None
        r = self.rounds
        u_start = srv.updates
        lanes = (_WorkerLanes(self.device, self.workers)
                 if is_gpu(self.device) and len(self.workers) > 1 and cfg.concurrent_workers else None)
        if srv.pair is not None and lanes is None:
            # the deferred evaluation rows ride in the next solve; one worker: the
            # server update is fused into that worker's solve as well
            srv.pair.set_ride(True, fuse_update=len(self.workers) == 1)
        while not self._stop(r - self.rounds, t_start, exhausted_since):
            W = [w for w in self.workers if w.k not in self.failed]
            if not W:
                break
            self.tracer.round_begin()
            if lanes is not None:  # workers run concurrently, one HIP stream each
                lanes.begin()
            with self.tracer.span("ingest"):
                for w in W:
                    with lanes.on(w) if lanes is not None else _Null():
                        w.ingest()
            if all(w.source.exhausted for w in W):
                exhausted_since = exhausted_since or time.time()
            if not all(w.ready() for w in W):
                time.sleep(0.001)
                continue
            deltas, done = [], []
            with self.tracer.span("solve"):
                for w in W:
                    try:
                        with lanes.on(w) if lanes is not None else _Null():
                            deltas.append(w.compute(self.log))
                        done.append(w)
                    except WorkerFailure as e:
                        self._worker_failed(e, w.k)
            if lanes is not None:
                lanes.join(done)
            if not deltas:
                break
            with self.tracer.span("server"):
                srv.apply_round(deltas, r, self.log)  # w += lr*sum(deltas), then the server eval row
                for w in done:
                    srv.tracker.received(w.k, r)
                srv.updates += len(done)
                for w in done:
                    srv.tracker.sent(w.k, r + 1)
                    w.vc = r + 1
            self.tracer.round_end(r, srv.updates - u_start)
            r += 1
            maybe_checkpoint(cfg, srv, r, W)
            self.log.drain()
        srv.flush_deferred(self.log)  # the last round's server row
        if srv.pair is not None:
            srv.pair.set_ride(False)
        if is_gpu(self.device):
            torch.cuda.synchronize(self.device)
        elapsed = time.time() - t_start
        self.rounds = r
        return {"rounds": r, "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": srv.updates / elapsed if elapsed > 0 else 0.0}

    # ------------------------------------------------------------------
    def _wide_lanes_ok(self) -> bool:
        """The wide / sparse model with 2..8 in-process GPU workers runs in rounds of
        ONE launch (csrc/solver/wide_solver.h WideLanes: every worker's persistent
        solve on an XCD of its own), one evaluation pass and the ordered sparse
        applies -- instead of ~14 launches per solve on per-worker streams that HIP's
        4 hardware queues serialise (profiles/r06/README.md section 7).  Runs that
        need Python between a worker's solves (tracing, injected faults) keep the
        per-worker schedulers."""
        c = self.cfg
        mode = os.environ.get("PSX_WIDE_LANES", "auto")  # 0: never, 1: 2..8 workers, auto: 5..8
        if mode == "0" or not is_gpu(self.device) or self.evalset is None:
            return False
        W = [w for w in self.workers if w.k not in self.failed]
        # auto: from 5 workers on.  With 2-4 the per-worker graphs on their streams measured
        # faster (6.5k / 7.7k / 9.4k against 5.7k / 7.2k / 9.1k updates/s: a lane's one-XCD
        # solve is latency-bound, and 2-4 chains of full-GPU launches overlap well), with 8
        # the lanes (15.0k against 8.9k) -- profiles/r06/README.md section 9
        lo = 2 if mode == "1" else 5
        if not lo <= len(W) <= 8 or self.tracer.enabled:
            return False
        if any(not w.wide or w.solver.dense_delta for w in W):
            return False
        if any(c.inject_worker_delay_ms.values()) or c.inject_worker_crash or c.inject_worker_stop:
            return False
        return True

    def _wide_lanes_for(self, W):
        """The WideLanes object over these workers' solvers, every one bound to the
        server weights (each lane pulls them in-kernel: no per-worker copy of the
        F*KP-float vector per release)."""
        for w in W:
            w.solver._bind(w.ring, self.server.w)
        key = tuple((w.k, id(w.solver._native)) for w in W)
        lp = getattr(self, "_wlanes", None)
        if lp is None or self._wlanes_key != key:
            lp = _native.hip().WideLanes([w.solver._native for w in W], 0)
            self._wlanes, self._wlanes_key = lp, key
        return lp

    def _run_wide_lanes(self) -> dict:
        """Rounds of the wide model's workers in one process (BSP, SSP and ASP):

        1. every worker ingests its new tuples (WorkerSamplingProcessor.java:50-113);
        2. ONE launch solves every worker's window from the current server weights,
           worker l on XCD l (LogisticRegressionTaskSpark.java:142-221);
        3. ONE evaluation pass: the worker rows of these solves (local models,
           LogisticRegressionTaskSpark.java:186) and the server row of the previous
           round (the global model, unchanged until step 4);
        4. the server applies the sparse pushes one after the other, worker 0's last
           (ServerProcessor.java:143-151: each delta on arrival; the server row,
           ServerProcessor.java:154-165, follows worker 0's delta and is the model the
           next round's pass evaluates), and the tracker records the deltas.

        Under SSP / ASP every worker is released on its own delta; the round only
        fixes one interleaving of arrivals the reference could produce (deltas that
        arrive together, applied in order).  A worker re-pulls at the next launch."""
        cfg, srv = self.cfg, self.server
        W = [w for w in self.workers if w.k not in self.failed]
        L = len(W)
        lp = self._wide_lanes_for(W)
        ev = self.evalset
        ds = ev.ds
        stream = stream_handle(self.device)
        bsp = cfg.consistency_model == 0
        lr = float(cfg.lr)
        order = list(range(1, L)) + [0]  # worker 0 (the server-row worker) last
        row_w = min(range(L), key=lambda i: W[i].k)  # the lowest live worker logs the server rows
        if row_w != 0:
            order = [i for i in range(L) if i != row_w] + [row_w]
        native = self.log.native
        r0 = r = self.rounds
        if not bsp:
            for w in W:  # bootstrap: the current version to everybody (as _run_async_events)
                u = int(srv.tracker.clock(w.k))
                if u > 0:
                    srv.tracker.sent(w.k, u)
                w.vc = u
        else:
            for w in W:
                w.vc = r
        for w in W:
            w.w = srv.w
        pending_srv = None  # (vc) the server row of the last round, evaluated by the next pass
        t_start = time.time()
        exhausted_since = None
        from ..ops.sparse import IngestBatch

        batch = IngestBatch()  # every worker's deliveries of a round: one launch
        for w in W:
            w.ring.batch = batch
        try:
            while not self._stop(r - r0, t_start, exhausted_since):
                for w in W:
                    w.ingest()
                batch.flush(self.device)
                if all(w.source.exhausted for w in W):
                    exhausted_since = exhausted_since or time.time()
                if not all(w.ready() for w in W):
                    if all(w.window.size <= 0 and w.source.exhausted for w in W):
                        break
                    time.sleep(0.0005)
                    continue
                Bs, starts, seen = [], [], []
                for w in W:
                    Bs.append(int(w.window.size))
                    starts.append(int(w.window.start))
                    w._seen_at_solve = w.tuples_seen
                    seen.append(w._seen_at_solve)
                lp.run(Bs, starts, stream)
                # worker rows of this round + the server row of the previous one, one pass
                slots, seqs, subs = [], [], []
                for i, w in enumerate(W):
                    s_, q_, a_ = native.acquire()
                    slots.append(a_)
                    seqs.append(q_)
                    subs.append((s_, q_, 0, w.k, w.vc, seen[i]))
                ss = sq = 0
                if pending_srv is not None:
                    s_, sq, ss = native.acquire()
                    subs.insert(0, (s_, sq, 1, -1, pending_srv, 0))
                lp.eval(ds.indptr.data_ptr(), ds.idx.data_ptr(), ds.val.data_ptr(), ds.y.data_ptr(), ev.T,
                        srv.w.data_ptr(), L, slots, seqs, ss, sq, stream)
                for s_, q_, kind, part, vc, ns in subs:
                    native.submit(s_, q_, kind, -1, part, int(vc), int(ns))
                lp.apply(srv.w.data_ptr(), lr, order, stream)
                srv.updates += L
                if bsp:
                    for w in W:
                        srv.tracker.received(w.k, r)
                    for w in W:
                        srv.tracker.sent(w.k, r + 1)
                        w.vc = r + 1
                    pending_srv = r
                else:
                    rel = {}
                    for i in order:
                        v = W[i].vc
                        for j, u in srv.tracker.on_delta(W[i].k, v):
                            rel[j] = u
                        if i == row_w:
                            pending_srv = v
                    if len(rel) != L:
                        raise RuntimeError(f"wide lanes: the tracker released {sorted(rel)} of {L} workers after a round")
                    for w in W:
                        w.vc = rel[w.k]
                for w in W:
                    w.iters += 1
                r += 1
                maybe_checkpoint(cfg, srv, srv.updates if not bsp else r, W)
            if pending_srv is not None:  # the last round's server row
                s_, sq, ss = native.acquire()
                lp.eval(ds.indptr.data_ptr(), ds.idx.data_ptr(), ds.val.data_ptr(), ds.y.data_ptr(), ev.T,
                        srv.w.data_ptr(), 0, [], [], ss, sq, stream)
                native.submit(s_, sq, 1, -1, -1, int(pending_srv), 0)
        finally:
            batch.flush(self.device)
            for w in W:
                w.ring.batch = None
            torch.cuda.synchronize(self.device)
        self.rounds = r if bsp else int(srv.tracker.min_clock())
        elapsed = time.time() - t_start
        return {"rounds": self.rounds, "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": (r - r0) * L / elapsed if elapsed > 0 else 0.0, "wide_lanes": L}

    def _event_scheduler(self) -> bool:
        """SSP/ASP in one process: event polling (True) or a thread per worker."""
        mode = self.cfg.async_scheduler
        if mode not in ("auto", "events", "threads"):
            raise ValueError(f"async_scheduler must be auto, events or threads, not {mode!r}")
        if mode == "auto":
            # a straggler sleeps inside its solve, which must not stall the others
            return is_gpu(self.device) and not any(self.cfg.inject_worker_delay_ms.values())
        return mode == "events"

    def _run_async_events(self) -> dict:
        """SSP/ASP with every worker driven from this one host thread.

        The server side is the same as the threaded loop (ServerProcessor.java:143-183:
        apply on arrival, eval row on worker-0 deltas, reply to whom the tracker
        releases).  A released worker gets the server weights copied on the main
        stream, then its ingest + solve + eval row are launched on its own HIP stream
        and an event is recorded behind them; the loop polls the in-flight events
        oldest first and applies each finished delta in completion order.  A hand-off
        is one hipEventQuery, not a queue.Queue round trip through the GIL (4 workers
        ASP: 3.6k -> 13.4k updates/s, profiles/r01_v7).  On the CPU the launch is
        synchronous and completion is FIFO.
        """
        cfg, srv, W = self.cfg, self.server, self.workers
        gpu = is_gpu(self.device)
        main = torch.cuda.current_stream(self.device) if gpu else None
        streams = {w.k: torch.cuda.Stream(self.device) for w in W} if gpu else {}
        alive = {w.k for w in W if w.k not in self.failed}
        pending: dict[int, tuple[int, object]] = {}  # released, not yet launched: k -> (vc, ev)
        inflight: list[tuple[int, int, torch.Tensor, object]] = []  # (k, vc, delta, ev), launch order

        # a worker has at most one release pending and one solve in flight, so one
        # event of each kind per worker is reused (no event creation per update)
        rel_ev = {w.k: torch.cuda.Event() for w in W} if gpu else {}
        done_ev = {w.k: torch.cuda.Event() for w in W} if gpu else {}

        def release(j: int, u: int):
            W[j].w.copy_(srv.w)
            ev = None
            if gpu:
                ev = rel_ev[j]
                ev.record(main)
            pending[j] = (u, ev)

        def launch(k: int) -> bool:
            w = W[k]
            u, ev = pending[k]
            w.vc = u
            failure = None
            if gpu:  # (set_stream: the stream context manager costs ~10 us of host time)
                torch.cuda.set_stream(streams[k])
            try:
                w.ingest()
                if not w.ready():
                    return False
                del pending[k]
                if ev is not None:  # the pulled weights (copied on the main stream)
                    streams[k].wait_event(ev)
                try:
                    delta = w.compute(self.log)
                except WorkerFailure as e:
                    failure = e
                else:
                    if gpu:
                        done_ev[k].record(streams[k])
            finally:
                if gpu:
                    torch.cuda.set_stream(main)
            if failure is not None:  # releases copy on the main stream, like every pull
                for j, v in self._worker_failed(failure, k):
                    release(j, v)
                alive.discard(k)
                return True
            inflight.append((k, u, delta, done_ev[k] if gpu else None))
            return True

        for j in sorted(alive):  # bootstrap: the current version to everybody
            u = int(srv.tracker.clock(j))
            if u > 0:  # a later run of this engine resumes at the tracked clocks
                srv.tracker.sent(j, u)
            release(j, u)
        t_start = time.time()
        exhausted: set[int] = set()
        exhausted_since = None
        per_worker = {k: 0 for k in alive}
        while alive:
            if self._stop(min(per_worker[k] for k in alive), t_start, exhausted_since):
                break
            progressed = False
            for k in sorted(pending):
                if k in alive:
                    progressed |= launch(k)
                else:
                    del pending[k]
            hit = next((i for i, t in enumerate(inflight) if t[3] is None or t[3].query()), None)
            if hit is None:
                # a solve is ~70 us: spin on the events (a sleep would cost more than
                # the solve); sleep only while every released worker waits for data
                if not progressed and not inflight:
                    time.sleep(0.001)
                continue
            k, v, delta, ev = inflight.pop(hit)
            if k not in alive:
                continue
            if W[k].source.exhausted:
                exhausted.add(k)
                if alive <= exhausted:
                    exhausted_since = exhausted_since or time.time()
            if ev is not None:
                main.wait_event(ev)
            # server eval rows follow the deltas of worker 0 (ServerProcessor.java:154-165),
            # or of the lowest surviving worker once 0 has failed
            if k == min(alive):
                srv.apply_and_log(delta, v, self.log)
            else:
                srv.apply(delta)
            srv.updates += 1
            per_worker[k] += 1
            for j, u in srv.tracker.on_delta(k, v):
                release(j, u)
            maybe_checkpoint(cfg, srv, srv.updates)
            self.log.drain()
        if gpu:
            torch.cuda.synchronize(self.device)
        elapsed = time.time() - t_start
        return {"rounds": int(srv.tracker.min_clock()), "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": srv.updates / elapsed if elapsed > 0 else 0.0}

    def _run_async(self) -> dict:
        cfg, srv, W = self.cfg, self.server, self.workers
        gpu = is_gpu(self.device)
        to_server: queue.Queue = queue.Queue()
        inbox = [queue.Queue() for _ in W]
        stop = threading.Event()
        log_lock = threading.Lock()
        errors = []

        class _LockedLog:
            def __init__(s, inner):
                s.inner = inner

            def worker_eval(s, *a, **k):
                with log_lock:
                    s.inner.worker_eval(*a, **k)

        locked = _LockedLog(self.log)

        def worker_loop(w: WorkerRole):
            try:
                stream = torch.cuda.Stream(self.device) if gpu else None
                ctx = torch.cuda.stream(stream) if gpu else _Null()
                with ctx:
                    while True:
                        msg = inbox[w.k].get()
                        if msg is None:
                            return
                        vc, ev = msg
                        if ev is not None:
                            torch.cuda.current_stream(self.device).wait_event(ev)
                        w.vc = vc
                        w.ingest()
                        while not w.ready():
                            if stop.is_set():
                                return
                            time.sleep(0.001)
                            w.ingest()
                        try:
                            delta = w.compute(locked)
                        except WorkerFailure as e:
                            to_server.put(("fail", w.k, e))
                            return
                        ev2 = None
                        if gpu:
                            ev2 = torch.cuda.Event()
                            ev2.record(torch.cuda.current_stream(self.device))
                        to_server.put((w.k, vc, delta, ev2, w.source.exhausted))
            except Exception as e:  # surfaced by the server loop
                errors.append(e)
                to_server.put(None)

        threads = [threading.Thread(target=worker_loop, args=(w,), daemon=True) for w in W]
        for t in threads:
            t.start()

        def send(j: int, u: int):
            W[j].w.copy_(srv.w)
            ev = None
            if gpu:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
            inbox[j].put((u, ev))

        alive = {w.k for w in W if w.k not in self.failed}
        for j in sorted(alive):  # bootstrap: vc 0 to everybody, tracker untouched
            u = int(srv.tracker.clock(j))
            if u > 0:  # a later run of this engine resumes at the tracked clocks
                srv.tracker.sent(j, u)
            send(j, u)
        t_start = time.time()
        exhausted = set()
        exhausted_since = None
        per_worker = {k: 0 for k in alive}
        while alive:
            if errors:
                break
            done_iters = min(per_worker[k] for k in alive)
            if self._stop(done_iters, t_start, exhausted_since):
                break
            try:
                tok = to_server.get(timeout=0.05)
            except queue.Empty:
                continue
            if tok is None:
                break
            if tok[0] == "fail":
                _, k, e = tok
                with log_lock:
                    for j, u in self._worker_failed(e, k):
                        send(j, u)
                alive.discard(k)
                continue
            k, v, delta, ev, ex = tok
            if ex:
                exhausted.add(k)
                if alive <= exhausted:
                    exhausted_since = exhausted_since or time.time()
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
            with log_lock:
                # server eval rows follow the deltas of worker 0 (ServerProcessor.java:154-165),
                # or of the lowest surviving worker once 0 has failed
                if k == min(alive):
                    srv.apply_and_log(delta, v, self.log)
                else:
                    srv.apply(delta)
                srv.updates += 1
                per_worker[k] += 1
                for j, u in srv.tracker.on_delta(k, v):
                    send(j, u)
                maybe_checkpoint(cfg, srv, srv.updates)
                self.log.drain()
        stop.set()
        for q in inbox:
            q.put(None)
        for t in threads:
            t.join(timeout=30)
        if gpu:
            torch.cuda.synchronize(self.device)
        if errors:
            raise errors[0]
        elapsed = time.time() - t_start
        return {"rounds": int(srv.tracker.min_clock()), "updates": srv.updates, "elapsed_s": elapsed,
                "updates_per_s": srv.updates / elapsed if elapsed > 0 else 0.0}


class _WorkerLanes:
    """One HIP stream per in-process worker (BSP).  A local solve is a chain of
    latency-bound kernels that occupies a few dozen of the 256 CUs, so the N
    workers' solves of a round run side by side instead of back to back.
    Round start: every lane waits for the previous server update (main
    stream); round end: the server update waits for every lane."""

    def __init__(self, device, workers):
        self.device = torch.device(device)
        self.streams = {w.k: torch.cuda.Stream(self.device) for w in workers}
        self.done = {w.k: torch.cuda.Event() for w in workers}
        self.start = torch.cuda.Event()
        self.main = torch.cuda.current_stream(self.device)  # the engine loop's stream
        self._on = {k: _OnStream(st, self.main) for k, st in self.streams.items()}

    def begin(self):
        self.start.record(self.main)
        for st in self.streams.values():
            st.wait_event(self.start)

    def on(self, w):
        return self._on[w.k]

    def join(self, workers):
        main = self.main
        for w in workers:
            ev = self.done[w.k]
            ev.record(self.streams[w.k])
            main.wait_event(ev)


class _OnStream:
    """Make `stream` current for a block, then restore `prev` (a fixed stream).
    torch.cuda.stream() looks the device and the current stream up on every
    entry, ~10 us of host time per block -- per solve, for in-process workers."""

    __slots__ = ("stream", "prev")

    def __init__(self, stream, prev):
        self.stream, self.prev = stream, prev

    def __enter__(self):
        torch.cuda.set_stream(self.stream)
        return self

    def __exit__(self, *a):
        torch.cuda.set_stream(self.prev)
        return False


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
