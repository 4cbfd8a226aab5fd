"""The native asynchronous server loop (csrc/runtime/async_server.h) on ONE GPU.

RCCL refuses two ranks on one device, so on a one-GPU box the production
server loop runs over :class:`LocalP2P` (stream-ordered device copies in
place of ncclSend / ncclRecv) with in-process stand-in workers
(:class:`LocalFeeder`: threads that push the token of a prepared delta as soon
as the server has released them).  Everything else -- the token queue, the
vector-clock tracker, the update / evaluation kernels, the metrics sink, the
no-host-sync schedule -- is the code path of the multi-GPU run; this harness is
what the GPU tests and ``tools/async_server_bench.py`` measure.
Reference semantics: ServerProcessor.java:143-183, MessageTracker.java:69-87.
"""
from __future__ import annotations

import os
import time

import torch

from .. import _native
from ..models.logreg import ModelSpec
from ..ops.lr import EvalScratch, EvalSet, Fragments
from ..utils.logsink import LogSink


class LocalAsyncHarness:
    def __init__(self, num_workers: int, consistency: int, features: int = 1024, classes: int = 6,
                 test=None, lr: float | None = None, seed: int = 0, device="cuda:0", log: bool = True):
        h, host = _native.hip(), _native.host
        self.N, self.c = int(num_workers), int(consistency)
        self.device = torch.device(device)
        self.spec = spec = ModelSpec(features, classes)
        P = spec.P
        self.lr = 1.0 / self.N if lr is None else float(lr)
        g = torch.Generator().manual_seed(seed)
        # worker k's delta (its outbox) and its pulled weights (its inbox)
        self.deltas = [(torch.randn(P, generator=g) * 1e-3).to(self.device) for _ in range(self.N)]
        self.inbox = [torch.zeros(P, device=self.device) for _ in range(self.N)]
        self.w = torch.zeros(P, device=self.device)
        self.buf = torch.zeros(P, device=self.device)
        self.frag = Fragments(spec, self.device)
        self.frag.refresh(self.w)
        self.scratch = EvalScratch(self.device)
        self.tracker = host.VectorClockTracker(self.N, self.c)
        self.queue = host.CtrlQueue(f"/psx_local_async_{os.getpid()}_{id(self)}"[:250], 4096, True)
        self.log = LogSink(spec.eval_classes, self.device) if log else None
        self.evalset = None
        if test is not None:
            self.evalset = EvalSet(spec, test.X, test.y, self.device)
        self.p2p = h.LocalP2P(self.N, [d.data_ptr() for d in self.deltas], [], [b.data_ptr() for b in self.inbox])
        d = dict(nworkers=self.N, model=0, lr=self.lr, P=P, w=self.w.data_ptr(), buf=self.buf.data_ptr(), K=spec.K,
                 F=spec.F, FP=spec.Fp, coff=self.frag.coff, fhi=self.frag.hi.data_ptr(), flo=self.frag.lo.data_ptr(),
                 fb=self.frag.b.data_ptr(), api=host.capi(), tracker=self.tracker.handle, ctrl=self.queue.handle)
        if self.log is not None and self.evalset is not None:
            ev = self.evalset
            d.update(sink=self.log.native.handle, acc=self.scratch.acc.data_ptr(),
                     ticket=self.scratch.ticket.data_ptr(), Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=ev.T)
        self.server = h.AsyncServer(self.p2p, d, torch.cuda.current_stream(self.device).cuda_stream)

    def run(self, iters: int, timeout_s: float = 120.0) -> dict:
        """Every stand-in worker pushes ``iters`` deltas (the last one final)."""
        h = _native.hip()
        vc0 = [int(self.tracker.clock(k)) for k in range(self.N)]  # a later run continues at the tracked clocks
        feeder = h.LocalFeeder(_native.host.capi(), self.queue.handle, self.p2p, self.N, int(iters), 0,
                               float(timeout_s), vc0)
        torch.cuda.synchronize(self.device)
        u0 = self.server.updates
        t0 = time.perf_counter()
        self.server.begin()
        feeder.start()
        code, k, upd = self.server.run(0)
        ok = feeder.join()
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - t0
        if code != h.ASYNC_DONE or not ok:
            raise RuntimeError(f"native async server: code {code} worker {k}, feeder ok={ok}")
        n = int(upd) - int(u0)
        return {"updates": n, "seconds": dt, "updates_per_s": n / dt, "host_seconds": t_host,
                "host_us_per_update": float(self.server.host_us_per_update), "max_vc_gap": int(self.tracker.max_gap)}

    def close(self):
        if self.log is not None:
            self.log.close()
        self.queue.unlink()
