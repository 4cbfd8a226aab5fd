"""Worker and server roles (device state + one iteration each).

WorkerRole  <- WorkerTrainingProcessor + WorkerSamplingProcessor + the
               per-key LogisticRegressionTaskSpark (reference:
               WorkerTrainingProcessor.java:63-98, WorkerSamplingProcessor.java:50-113)
ServerRole  <- ServerProcessor + MessageTracker (ServerProcessor.java:143-228,
               MessageTracker.java:42-88)

Transport-agnostic: the engines (in-process or RCCL multi-process) move the
delta / weight tensors; roles only enqueue device work on the current stream.
"""
from __future__ import annotations

import dataclasses

import math
import os
import time
from contextlib import contextmanager

import torch

from .. import _native
from ..models.logreg import ModelSpec
from ..models.wide import WideSpec
from ..ops.lr import EvalScratch, EvalSet, Fragments, LocalSolveOp, is_gpu, server_apply, stream_handle
from ..ops.sparse import SparseRing, WideEvalSet, WideSolveOp, nz_capacity, wide_server_apply
from .buffer import DeviceRing, StreamSource
from .config import PSConfig, new_tuples_needed
from .faults import WorkerFailure


class SideStream:
    """Evaluation work off the critical path (GPU): it runs on its own stream
    after the work that produced its inputs, and the next writer of those
    inputs waits for it (:meth:`fence`).  On one MI355X the latency-bound
    solver kernels leave most CUs idle, so a test-set evaluation on the side
    stream overlaps the next solve instead of adding to the round time."""

    def __init__(self, device, force: bool = False):
        self.device = torch.device(device)
        self.gpu = is_gpu(self.device) and (force or os.environ.get("PSX_SIDE_EVAL", "0") == "1")
        self.stream = torch.cuda.Stream(self.device) if self.gpu else None
        self._ready = torch.cuda.Event() if self.gpu else None
        self._done = torch.cuda.Event() if self.gpu else None
        self._pending = False

    @contextmanager
    def run(self):
        if not self.gpu:
            yield
            return
        self._ready.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(self._ready)
        with torch.cuda.stream(self.stream):
            yield
        self._done.record(self.stream)
        self._pending = True

    def fence(self):
        if self._pending:
            torch.cuda.current_stream(self.device).wait_event(self._done)
            self._pending = False


def is_wide(spec) -> bool:
    return isinstance(spec, WideSpec)


def make_evalset(spec, test, device):
    """Device-resident test set of either model (dense MFMA tiles / sparse CSR)."""
    if test is None:
        return None
    if is_wide(spec):
        return WideEvalSet(spec, test, device)
    return EvalSet(spec, test.X, test.y, device)


class WorkerRole:
    def __init__(self, k: int, spec, cfg: PSConfig, device, train, evalset, t0: float | None = None,
                 xcd: int = 0):
        self.k, self.spec, self.cfg, self.device = k, spec, cfg, torch.device(device)
        self.wide = is_wide(spec)
        if self.wide:
            nz = cfg.ring_nz or nz_capacity(train.max_nnz)
            self.ring = SparseRing(cfg.max_buffer_size, nz, self.device)
        else:
            self.ring = DeviceRing(cfg.max_buffer_size, spec.Fp, self.device, defer=cfg.solver.fused_ingest,
                                   dtype=cfg.dtype)
        self.window = _native.host.SlidingWindow(cfg.min_buffer_size, cfg.max_buffer_size,
                                                 cfg.buffer_size_coefficient, 500, self.ring.cap)
        self.source = StreamSource(train, k, cfg.num_workers, self.ring, self.window,
                                   p_ms=cfg.producer_time_per_event, mode=cfg.stream_mode,
                                   rows_per_iter=cfg.rows_per_iter, epochs=cfg.epochs, t0=t0)
        if self.wide:
            self.solver = WideSolveOp(spec, self.ring.cap, self.ring.NZ, self.device, cfg.solver,
                                      dense_delta=cfg.wide_dense_delta)
        else:
            # xcd: the XCD of the solve's cooperating workgroups (-1: spread over the XCDs,
            # for workers that share the GPU with other workers' concurrent solves)
            self.solver = LocalSolveOp(spec, self.ring.cap, self.device, dataclasses.replace(cfg.solver, xcd=xcd))
        self.evalset = evalset
        self.w = torch.zeros(spec.P, dtype=torch.float32, device=self.device)  # pulled weights
        self.scratch = EvalScratch(self.device)
        self.side = SideStream(self.device)
        self.pair = None  # EvalPair with the colocated server (BSP)
        self.vc = 0  # version of the weights currently held
        self.iters = 0
        self._seen_at_solve = 0  # tuples seen when the last solve started (--iter_new_rows)
        self.delay_s = float(cfg.inject_worker_delay_ms.get(k, 0.0)) / 1000.0
        crash = cfg.inject_worker_crash.get(k)
        self.crash_at = int(crash) if crash is not None else None

    @property
    def tuples_seen(self) -> int:
        return int(self.window.tuples_seen)

    def ingest(self) -> int:
        return self.source.poll()

    def ready(self) -> bool:
        """Data to train on; with --iter_new_rows K, only once K new tuples arrived
        since the last solve (a stream-driven cadence: re-solving an unchanged
        window only re-fits the same rows)."""
        if self.window.size <= 0:
            return False
        K = new_tuples_needed(self.cfg, int(self.window.size), self.iters)
        return K <= 0 or self.tuples_seen - self._seen_at_solve >= K or self.source.exhausted

    def compute(self, log=None) -> torch.Tensor:
        """One local solve on the current window; returns the delta tensor.

        The worker's metrics are those of the LOCALLY trained model
        (LogisticRegressionTaskSpark.java:186), logged with the weights version
        it trained from and numTuplesSeen = the newest insertion id.
        """
        delta = self.solve()
        self.log_eval(log)
        return delta

    def solve(self):
        """The local solve alone (the evaluation row is :meth:`log_eval`): lets a
        multi-rank schedule put its collective between the two so that the
        evaluation overlaps the communication."""
        if self.crash_at is not None and self.iters >= self.crash_at:
            raise WorkerFailure(self.k, f"injected crash at iteration {self.iters}")
        if self.delay_s > 0:
            time.sleep(self.delay_s)
        B, start = int(self.window.size), int(self.window.start)
        self._seen_at_solve = self.tuples_seen
        ride = ap = None
        if self.pair is not None:
            # the deferred rows ride in this solve's launches, or (no ride) a deferred
            # row reads the model this solve overwrites: evaluated first
            ride, ap = self.pair.before_solve()
        self.side.fence()  # the last evaluation read the solver outputs this solve overwrites
        if ride is None and ap is None:
            self.solver.run(self.ring, B, start, self.w)
        else:
            self.solver.run(self.ring, B, start, self.w, ride=ride[0] if ride else None, apply=ap)
        if self.pair is not None:
            self.pair.after_solve(ride, ap)
        self.iters += 1
        if self.wide and not self.solver.dense_delta:
            return self.solver.sparse_delta()
        return self.solver.delta

    def check_device_health(self):
        """Raise if any device solve of this worker hit a timed-out cross-workgroup
        wait (its delta was garbage; the logged loss of that row is NaN)."""
        if self.solver.barrier_errors():
            raise WorkerFailure(self.k, "device solver: a cross-workgroup wait timed out (non-resident workgroup)")

    def log_eval(self, log):
        """Worker row of the last solve: metrics of the LOCALLY trained model
        (LogisticRegressionTaskSpark.java:186)."""
        if self.pair is not None:
            self.pair.worker_row(log)
            return
        if log is not None and self.evalset is not None:
            if self.wide:  # local model = pulled weights overlaid with the subspace solution
                # (in line: the overlay reads the pulled weights, which the server update rewrites)
                log.worker_eval(self.evalset, self.solver, self.w, self.scratch, self.solver.loss, self.k, self.vc,
                                self.tuples_seen)
            else:
                with self.side.run():
                    log.worker_eval(self.evalset, self.solver.frag, self.solver.w_new, self.scratch,
                                    self.solver.loss, self.k, self.vc, self.tuples_seen)


class ServerRole:
    def __init__(self, spec, cfg: PSConfig, device, evalset, w0: torch.Tensor):
        self.spec, self.cfg, self.device = spec, cfg, torch.device(device)
        self.wide = is_wide(spec)
        self.w = w0.to(self.device, torch.float32).clone()
        self.frag = Fragments(spec, self.device) if is_gpu(self.device) and not self.wide else None
        self.frag_next = None  # EvalPair: the second fragment buffer of the fused update
        if self.frag is not None:
            self.frag.refresh(self.w)
        self.tracker = _native.host.VectorClockTracker(cfg.num_workers, cfg.consistency_model)
        self.evalset = evalset
        self.scratch = EvalScratch(self.device)
        self.side = SideStream(self.device)
        self.pair = None  # EvalPair with the colocated worker (BSP)
        self.updates = 0
        self.acc = torch.zeros(spec.P, dtype=torch.float32, device=self.device)

    def apply(self, delta: torch.Tensor, lr: float | None = None):
        """w += lr * delta   (ServerProcessor.java:148-151 with lr = 1/N)."""
        lr = self.cfg.lr if lr is None else lr
        if self.pair is not None and self.pair.fused_apply([delta], lr):
            return
        self.before_update()  # the last server evaluation reads w / the fragments rewritten here
        if self.wide:
            wide_server_apply(self.spec, self.w, delta, lr)
        else:
            server_apply(self.spec, self.w, delta, lr, self.frag)

    def before_update(self):
        """Every reader of the current global model is enqueued before w / the
        fragments are rewritten (a deferred paired row, a side-stream evaluation)."""
        if self.pair is not None:
            self.pair.before_server_update()
        self.side.fence()

    def apply_round(self, deltas, vc: int, log, lr: float | None = None):
        """BSP round: w += lr * sum(deltas), then the server eval row."""
        if len(deltas) == 1:
            self.apply_and_log(deltas[0], vc, log, lr)
            return
        if all(isinstance(d, torch.Tensor) for d in deltas):
            if self.pair is not None and self.pair.fused_apply(deltas, self.cfg.lr if lr is None else lr):
                self.log_eval(vc, log)
                return
            if self.frag is not None and not self.wide and len(deltas) <= 16:  # one fused kernel
                self.before_update()
                sp = self.spec
                _native.hip().server_apply_n(sp.K, sp.F, sp.Fp, self.w.data_ptr(), [d.data_ptr() for d in deltas],
                                             float(self.cfg.lr if lr is None else lr), self.frag.hi.data_ptr(),
                                             self.frag.lo.data_ptr(), self.frag.b.data_ptr(),
                                             stream_handle(self.device), self.frag.coff)
                self.log_eval(vc, log)
                return
            self.acc.copy_(deltas[0])
            for d in deltas[1:]:
                self.acc.add_(d)
            self.apply_and_log(self.acc, vc, log, lr)
            return
        for d in deltas:  # sparse pushes: sequential applies == one applied sum
            self.apply(d, lr)
        self.log_eval(vc, log)

    def apply_and_log(self, delta: torch.Tensor, vc: int, log, lr: float | None = None):
        """apply() then the global-model evaluation row.  (A single fused
        update+eval kernel was measured slower: every workgroup rebuilt the
        weight fragments from fp32 -- profiles/r01_v2.)"""
        self.apply(delta, lr)
        self.log_eval(vc, log)

    def log_eval(self, vc: int, log, ts: int | None = None):
        """Global-model test metrics, logged on worker-0 deltas (ServerProcessor.java:154-165)."""
        if log is None or self.evalset is None:
            return
        if self.pair is not None:  # evaluated together with the worker's next row
            self.pair.defer_server_row(log, vc, ts)
            return
        with self.side.run():
            log.server_eval(self.evalset, self.frag, self.w, self.scratch, vc, ts=ts)

    def flush_deferred(self, log):
        if self.pair is not None:
            self.pair.flush(log)


class EvalPair:
    """Sequential consistency with a colocated server: the worker's row of
    round r (its locally trained model) and the server's row of round r-1 (the
    global model, unchanged until the update of round r) are evaluated in ONE
    pass over the device-resident test set, and on the GPU that same launch also
    performs the server update of round r:

    * the worker's solver writes its model's MFMA fragments at columns [0, KP)
      of its own buffer; the server keeps TWO fragment buffers (columns
      [16 - K, 16)) -- ``server.frag`` holds the current global model, the update
      writes the other one, then they swap -- so nothing a launch reads is
      written by it;
    * the worker row is deferred from ``worker_row`` to the server update that
      follows it (``fused_apply``); if no update comes before the worker's next
      solve, it is evaluated on its own first.

    Server rows keep the timestamp of the update that produced them."""

    def __init__(self, server: "ServerRole", worker: WorkerRole):
        self.server, self.worker = server, worker
        self.pending = None  # (log, vc, ts) of a deferred server row
        self.pending_worker = None  # (log, vc, nseen, ts) of a deferred worker row
        self.fuse = os.environ.get("PSX_FUSED_APPLY", "1") != "0"
        # Ride mode (GPU, dense, eager small-window solver): the deferred rows are
        # evaluated by spare workgroups of the worker's NEXT solve (EvalRide,
        # csrc/kernels/lr_kernels.h) instead of by a launch of their own; the
        # server update is then a plain update launch, or -- when the engine sets
        # ``fuse_update`` (the server's update of a round is exactly this worker's
        # delta: one in-process BSP worker) -- part of the solve's finalisation.
        self.ride_ok = os.environ.get("PSX_EVAL_RIDE", "1") != "0"
        self.ride = False  # enabled by an engine loop whose solves and updates share one stream
        self.fuse_update = False
        self._applied = False  # this round's update already ran inside the solve
        spec = server.spec
        self.shared = (is_gpu(server.device) and not server.wide and server.evalset is worker.evalset
                       and server.evalset is not None and _solver_padded_classes(spec.K) + spec.K <= 16)
        self.wide_pair = (is_gpu(server.device) and server.wide and server.evalset is worker.evalset
                          and server.evalset is not None)
        if self.shared:
            server.frag = Fragments(spec, server.device, coff=16 - spec.K)
            server.frag.refresh(server.w)
            server.frag_next = Fragments(spec, server.device, coff=16 - spec.K)
        server.pair = self
        worker.pair = self

    # ---- ride mode ------------------------------------------------------
    def set_ride(self, on: bool, fuse_update: bool = False):
        """Engine hook: ride mode for the loop that follows (its worker solves and
        server updates are enqueued in order on one stream); ``fuse_update``: the
        server's update of every round is exactly this worker's delta."""
        self.ride = bool(on) and self.ride_ok
        self.fuse_update = self.ride and bool(fuse_update)
        self._applied = False

    def _riding(self) -> bool:
        wk = self.worker
        return self.ride and self.shared and not wk.wide and wk.solver.can_ride(wk.ring, wk.w)

    def before_solve(self):
        """(ride, apply) for the worker's next solve: the deferred rows to evaluate
        inside it ((kwargs, submit) or None) and the fused server update (or None).
        Without ride mode: the deferred worker row is evaluated now (the solve
        overwrites its model) and both are None."""
        if not self._riding():
            self.flush_worker()
            return None, None
        ride = self._take_ride()
        ap = None
        if self.fuse_update and self.fuse:
            srv = self.server
            srv.side.fence()
            ap = (srv.w, float(srv.cfg.lr), srv.frag_next)
        return ride, ap

    def after_solve(self, ride, ap):
        if ride is not None:
            ride[1]()  # the rows' records: submitted once their pass is enqueued
        if ap is not None:
            srv = self.server
            srv.frag, srv.frag_next = srv.frag_next, srv.frag
            self._applied = True

    def _take_ride(self):
        pw, pend = self.pending_worker, self.pending
        if pw is None and pend is None:
            return None
        log = pw[0] if pw is not None else pend[0]
        if pend is not None and pend[0] is not log:  # a different sink: evaluated on its own
            self.pending = None
            self._server_only(pend)
            pend = None
        self.pending_worker = self.pending = None
        wk, srv = self.worker, self.server
        nat = log.native
        if pw is not None:
            _, vc_w, nseen, ts_w = pw
            slot_w, seq_w, addr_w = nat.acquire()
            slot_s = seq_s = addr_s = 0
            if pend is not None:
                slot_s, seq_s, addr_s = nat.acquire()
            kw = wk.evalset.ride_args(wk.solver.frag, srv.frag, wk.scratch, addr_w, seq_w, wk.solver.loss, addr_s,
                                      seq_s)
        else:  # a server row alone: the global model as the pass's only model
            slot_s, seq_s, addr_s = nat.acquire()
            kw = wk.evalset.ride_args(srv.frag, None, wk.scratch, addr_s, seq_s, None, 0, 0)

        def submit():
            if pend is not None:
                nat.submit(slot_s, seq_s, 1, int(pend[2]), -1, int(pend[1]), 0)
            if pw is not None:
                nat.submit(slot_w, seq_w, 0, int(ts_w), int(wk.k), int(vc_w), int(nseen))

        return kw, submit

    def before_server_update(self):
        """The server's w / fragments are about to be rewritten: a deferred row that
        reads them is evaluated first."""
        if self.ride and self.shared:
            if self.pending is not None:  # a deferred server row reads the current global model
                self.flush(self.pending[0])
            return
        self.flush_worker()

    def defer_server_row(self, log, vc: int, ts: int | None):
        if self.pending is not None:
            self.flush(self.pending[0])
        self.pending = (log, int(vc), int(ts) if ts is not None else -1)  # -1: stamped when evaluated

    def worker_row(self, log):
        wk = self.worker
        if log is None or wk.evalset is None:
            return
        self.flush_worker()
        if self.shared:  # evaluated together with the server update that follows
            self.pending_worker = (log, int(wk.vc), int(wk.tuples_seen), -1)
            return
        pend, srv = self.pending, self.server
        if (pend is not None and pend[0] is log and self.wide_pair and wk.w.data_ptr() == srv.w.data_ptr()):
            # wide model: the worker's local model (overlay) and the global model it
            # was trained from (= the previous server row's model) in one pass
            self.pending = None
            log.pair_eval(wk.evalset, wk.solver, wk.w, wk.solver.loss, wk.k, int(wk.vc), int(wk.tuples_seen), None,
                          srv.w, pend[1], pend[2], wk.scratch)
            return
        self.flush(self.pending[0] if self.pending is not None else None)
        self._worker_only(log, int(wk.vc), int(wk.tuples_seen))

    def fused_apply(self, deltas, lr: float) -> bool:
        """The server update of this round in the launch that evaluates the
        deferred worker row (and the pending server row).  False: nothing to fuse
        with (the caller applies on its own)."""
        if self.ride and self.shared and self._riding():
            # ride mode: the rows wait for the next solve; the update ran inside the
            # solve (fuse_update) or is a plain update launch (False)
            applied, self._applied = self._applied, False
            return applied
        pw = self.pending_worker
        if pw is None or not self.shared or not self.fuse or not (1 <= len(deltas) <= 16):
            return False
        if not all(isinstance(d, torch.Tensor) for d in deltas):
            return False
        self.pending_worker = None
        srv = self.server
        srv.side.fence()
        self._pair(pw, apply=(srv.w, list(deltas), float(lr), srv.frag_next))
        srv.frag, srv.frag_next = srv.frag_next, srv.frag
        return True

    def flush_worker(self):
        """Evaluate a deferred worker row now (before the solver overwrites its model)."""
        pw = self.pending_worker
        if pw is None:
            return
        self.pending_worker = None
        self._pair(pw)

    def _pair(self, pw, apply=None):
        log, vc, nseen, ts = pw
        wk, srv = self.worker, self.server
        pend = self.pending
        if pend is not None and pend[0] is not log:  # a different sink (bench swapped logs): flush separately
            self._server_only(pend)
            pend = None
        self.pending = None
        log.pair_eval(wk.evalset, wk.solver.frag, wk.solver.w_new, wk.solver.loss, wk.k, vc, nseen, srv.frag, srv.w,
                      pend[1] if pend is not None else None, pend[2] if pend is not None else 0, wk.scratch, ts_w=ts,
                      apply=apply)

    def _worker_only(self, log, vc: int, nseen: int):
        wk = self.worker
        if wk.wide:
            log.worker_eval(wk.evalset, wk.solver, wk.w, wk.scratch, wk.solver.loss, wk.k, vc, nseen)
        else:
            log.worker_eval(wk.evalset, wk.solver.frag, wk.solver.w_new, wk.scratch, wk.solver.loss, wk.k, vc, nseen)

    def _server_only(self, pend):
        log, vc, ts = pend
        srv = self.server
        log.server_eval(srv.evalset, srv.frag, srv.w, srv.scratch, vc, ts=ts)

    def flush(self, log=None):
        self.flush_worker()
        if self.pending is not None:
            pend = self.pending
            self.pending = None
            self._server_only(pend)


def _solver_padded_classes(K: int) -> int:
    return 2 if K <= 2 else 4 if K <= 4 else 8 if K <= 8 else 16
