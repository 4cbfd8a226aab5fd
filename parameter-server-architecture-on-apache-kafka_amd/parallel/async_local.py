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


class LocalAsyncWideHarness:
    """The native loop's sparse model on one GPU: stand-in workers push fixed
    sparse deltas (feature ids + values, the wide model's push) and receive
    sparse pulls (the logged deltas since their previous pull) or dense ones."""

    def __init__(self, num_workers: int, consistency: int, features: int = 1 << 20, kp: int = 8, nnz: int = 2000,
                 lr: float | None = None, seed: int = 0, device="cuda:0", sparse_pull: bool = True):
        h, host = _native.hip(), _native.host
        self.N, self.F, self.KP = int(num_workers), int(features), int(kp)
        self.device = torch.device(device)
        self.P = self.F * self.KP + self.KP
        self.lr = 1.0 / self.N if lr is None else float(lr)
        g = torch.Generator().manual_seed(seed)
        self.uniq = [torch.randperm(self.F, generator=g)[:nnz].sort().values.to(torch.int32).to(self.device)
                     for _ in range(self.N)]
        self.dloc = [(torch.randn((nnz + 1) * self.KP, generator=g) * 1e-3).to(self.device) for _ in range(self.N)]
        self.inbox = [torch.zeros(self.P, device=self.device) for _ in range(self.N)]
        self.w = torch.zeros(self.P, device=self.device)
        self.ubuf = torch.zeros(nnz, dtype=torch.int32, device=self.device)
        self.dbuf = torch.zeros((nnz + 1) * self.KP, device=self.device)
        self.U = int(nnz)
        self.tracker = host.VectorClockTracker(self.N, int(consistency))
        base = f"/psx_local_wide_{os.getpid()}_{id(self)}"[:200]
        self.queue = host.CtrlQueue(base, 4096, True)
        self.replies = [host.CtrlQueue(f"{base}_r{j}", 64, True) for j in range(self.N)] if sparse_pull else []
        cap = 16 * (self.U + 1)
        self.lids = torch.zeros(cap, dtype=torch.int32, device=self.device)
        self.lvals = torch.zeros(cap * self.KP, device=self.device)
        self.p2p = h.LocalP2P(self.N, [d.data_ptr() for d in self.dloc], [u.data_ptr() for u in self.uniq],
                              [b.data_ptr() for b in self.inbox])
        d = dict(nworkers=self.N, model=1, lr=self.lr, P=self.P, w=self.w.data_ptr(), KP=self.KP, K=self.KP,
                 Fw=self.F, umax=self.U, ubuf=self.ubuf.data_ptr(), dbuf=self.dbuf.data_ptr(), api=host.capi(),
                 tracker=self.tracker.handle, ctrl=self.queue.handle)
        if sparse_pull:
            d.update(sparse_pull=1, lids=self.lids.data_ptr(), lvals=self.lvals.data_ptr(), logcap=cap,
                     replies=[q.handle for q in self.replies])
        self.server = h.AsyncServer(self.p2p, d, torch.cuda.current_stream(self.device).cuda_stream)

    def expected(self, iters: int) -> torch.Tensor:
        """w after every worker's delta was applied `iters` times."""
        w = torch.zeros(self.P, device=self.device)
        for u, dl in zip(self.uniq, self.dloc):
            w[self.F * self.KP: self.F * self.KP + self.KP] += dl[: self.KP] * self.lr * iters
            idx = (u.long() * self.KP).unsqueeze(1) + torch.arange(self.KP, device=self.device).unsqueeze(0)
            w.index_add_(0, idx.reshape(-1), dl[self.KP:] * (self.lr * iters))
        return w

    def run(self, iters: int, timeout_s: float = 120.0) -> dict:
        h = _native.hip()
        vc0 = [int(self.tracker.clock(k)) for k in range(self.N)]
        feeder = h.LocalFeeder(_native.host.capi(), self.queue.handle, self.p2p, self.N, int(iters), self.U,
                               float(timeout_s), vc0, [q.handle for q in self.replies])
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        self.server.begin()
        feeder.start()
        code, k, upd = self.server.run(0)
        ok = feeder.join()
        torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - t0
        if code != h.ASYNC_DONE or not ok:
            raise RuntimeError(f"native async server (wide): code {code} worker {k}, feeder ok={ok}")
        return {"updates": int(upd), "seconds": dt, "sparse_pulls": int(self.server.sparse_pulls),
                "dense_pulls": int(self.server.dense_pulls), "pull_floats": int(self.server.pull_floats),
                "feeder_sparse": int(feeder.sparse_pulls), "host_us_per_update": float(self.server.host_us_per_update)}

    def close(self):
        self.queue.unlink()
        for q in self.replies:
            q.unlink()
