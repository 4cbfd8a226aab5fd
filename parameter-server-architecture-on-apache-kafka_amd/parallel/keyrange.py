"""Key-range sharded parameter server (BASELINE.json config 5).

The reference tags every message with the ``KeyRange`` of the weights it carries
(BaseMessage.java:24-27, KeyRange.java:11-49) so that a server can own a range
of the key space (README.md:117-119, 333); its one server holds them all.  Here
every rank hosts one worker AND the server shard of its key range

    [lo, hi) = [rank * S, min(F, (rank + 1) * S)),   S = ceil(F / world)

and stores nothing else of the model: the coefficients ``shard [(hi-lo)*KP]``
(+ KP trailing zeros, so the shard is itself a wide-model vector of hi-lo
features) and the KP intercepts (replicated, all-reduced).  A round (BSP):

  plan   the window's distinct features (the wide solver's first phase),
         grouped by owner;
  pull   counts all-to-all, the ids to their owners, the owners' coefficients
         back -- only the ids the window touches;
  solve  the local solve in that subspace (second phase);
  push   the deltas of the same ids to their owners (who already hold the ids),
         applied sender by sender in rank order; intercept deltas all-reduced;
  rows   partial test margins of every shard, all-reduced: rank 0's server row
         is margins + intercepts, each worker row the previous round's margins
         + its window delta (the locally trained model).

Traffic per round is ``4 W + 8 U + 8 U KP`` bytes of model data per rank (U = the
window's distinct features) -- proportional to the window, independent of F --
plus ``4 T KP`` for the evaluation margins.  On GPUs the round is the native
:class:`KeyRangeLoop` (csrc/runtime/keyrange_loop.h, RCCL grouped send/recv);
on CPU ranks (gloo) the same protocol runs here with ``all_to_all_single`` and
the float64 reference solve.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from .. import _native
from ..ops.lr import _write_slot_cpu, is_gpu, stream_handle
from ..ops.sparse import SparseDataset, SparseRing, WideSolveOp, nz_capacity
from ..runtime.buffer import StreamSource
from ..runtime.config import PSConfig
from ..runtime.engine import load_datasets
from ..utils.logsink import LogSink, summarize


def key_range(F: int, world: int, rank: int) -> tuple[int, int, int]:
    """(lo, hi, S) of ``rank``'s features (KeyRange.java:11-49: [start, end))."""
    S = -(-int(F) // int(world))
    lo = int(rank) * S
    return lo, min(int(F), lo + S), S


def shard_csr(ds: SparseDataset, lo: int, hi: int) -> SparseDataset:
    """The entries of ``ds`` whose feature lies in [lo, hi), with local ids f - lo
    (every row kept, possibly empty): the test rows a shard evaluates."""
    lens = ds.indptr[1:] - ds.indptr[:-1]
    row = torch.repeat_interleave(torch.arange(ds.rows, device=ds.idx.device), lens)
    keep = (ds.idx >= lo) & (ds.idx < hi)
    cnt = torch.bincount(row[keep], minlength=ds.rows)
    indptr = torch.zeros(ds.rows + 1, dtype=torch.int64, device=ds.idx.device)
    indptr[1:] = torch.cumsum(cnt, 0)
    return SparseDataset(indptr, (ds.idx[keep] - lo).to(torch.int32), ds.val[keep], ds.y, hi - lo)


def _confusion(z: torch.Tensor, y: torch.Tensor, K: int) -> torch.Tensor:
    """16x16 confusion counts (row = label, column = prediction) of margins z [T, KP]."""
    pred = (z[:, 0] > 0).long() if K == 1 else z[:, :K].argmax(1)
    yl = (y > 0).long() if K == 1 else y.long()
    yl = yl.clamp(0, 15)
    c = torch.zeros(256, dtype=torch.int64)
    c.index_add_(0, (yl * 16 + pred).cpu(), torch.ones(yl.numel(), dtype=torch.int64))
    return c.to(torch.int32)


def _csr_mm(ds: SparseDataset, W: torch.Tensor) -> torch.Tensor:
    """[rows, KP] = ds @ W for W [F, KP] (CPU)."""
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)  # sparse CSR support is in beta
        m = torch.sparse_csr_tensor(ds.indptr, ds.idx.long(), ds.val.float(), size=(ds.rows, W.shape[0]))
    return m @ W


class KeyRangeEngine:
    """One rank of the key-range sharded BSP parameter server (every rank: one
    worker + one server shard).  Same surface as :class:`DistEngine` (run, log,
    close, train_start_ms)."""

    def __init__(self, cfg: PSConfig, rank: int, world: int, device, train=None, test=None):
        if cfg.consistency_model != 0:
            raise ValueError("the key-range sharded server runs sequential consistency (BSP) rounds")
        self.cfg, self.rank, self.world, self.device = cfg, int(rank), int(world), torch.device(device)
        if self.world > 1 and not dist.is_initialized():
            raise RuntimeError("key-range sharding over several ranks needs torch.distributed")
        cfg.num_workers = self.world
        self.spec, train, test = load_datasets(cfg, train, test)
        sp = self.spec
        if not hasattr(sp, "KP"):
            raise ValueError("the key-range sharded server holds the wide (sparse-input) model")
        self.lo, self.hi, self.S = key_range(sp.F, self.world, self.rank)
        if self.lo >= self.hi:
            raise ValueError(f"{self.world} ranks for {sp.F} features: rank {self.rank} owns no key")
        dev = self.device
        # this rank's server shard, and the replicated intercepts
        self.shard = sp.init_range(cfg.init, cfg.seed, self.lo, self.hi, device=dev)
        self.b = torch.zeros(sp.KP, dtype=torch.float32, device=dev)
        self.lr = cfg.lr
        # the worker: ring, window, producer, solver buffers (window-sized only)
        nz = cfg.ring_nz or nz_capacity(train.max_nnz)
        self.train = train.to(dev)
        self.ring = SparseRing(cfg.max_buffer_size, nz, dev)
        self.window = _native.host.SlidingWindow(cfg.min_buffer_size, cfg.max_buffer_size,
                                                 cfg.buffer_size_coefficient, 500, self.ring.cap)
        self.t0 = time.time()
        self.source = StreamSource(self.train, self.rank, self.world, self.ring, self.window,
                                   p_ms=cfg.producer_time_per_event, mode=cfg.stream_mode,
                                   rows_per_iter=cfg.rows_per_iter, epochs=cfg.epochs, t0=self.t0)
        self.solver = WideSolveOp(sp, self.ring.cap, self.ring.NZ, dev, cfg.solver)
        # evaluation: the whole test set (worker rows) and this shard's entries of it
        self.test = test.to(dev) if test is not None else None
        self.test_shard = shard_csr(self.test, self.lo, self.hi) if self.test is not None else None
        self.log = self._open_log()
        self.tracker = _native.host.VectorClockTracker(self.world, 0) if self.rank == 0 else None
        self.rounds = 0
        self.model_bytes = 0
        self.eval_bytes = 0
        self.last_round_bytes = 0
        self.last_u = 0
        self.comm = None
        self._loop = None
        self._z = None  # CPU: reduced margins of the current global model
        self.train_start_ms = None

    # ------------------------------------------------------------------
    def _open_log(self) -> LogSink:
        """Rank 0 creates both logs (reference headers); the other ranks then append
        whole worker lines to the shared logs-worker.csv."""
        cfg = self.cfg
        wp = sp = None
        if cfg.logging:
            wp = f"{cfg.log_dir}/logs-worker.csv"
            sp = f"{cfg.log_dir}/logs-server.csv" if self.rank == 0 else None
        mk = lambda: LogSink(self.spec.eval_classes, self.device, wp, sp, keep_records=(self.rank == 0),
                             worker_append=self.rank != 0)
        log = mk() if self.rank == 0 else None
        if cfg.logging and self.world > 1:
            dist.barrier()  # the files exist, headers written
        return log if log is not None else mk()

    def weight_bytes(self) -> int:
        """Model bytes this rank stores: its shard + the replicated intercepts."""
        return (self.shard.numel() + self.b.numel()) * 4

    def mark_start(self):
        if self.train_start_ms is None:
            self.train_start_ms = time.time() * 1000.0

    def run(self) -> dict:
        """Run cfg.max_iters rounds, then close the communicator and the logs
        (``_run_bsp``: the rounds alone, for callers that continue the run)."""
        try:
            out = self._run_bsp()
        except BaseException:
            comm, self.comm = self.comm, None
            if comm is not None:
                comm.c.abort()  # peers may be gone: no collective teardown
            raise
        self.close()
        if self.log is not None:
            self.log.close()
        return out

    def _run_bsp(self) -> dict:
        self.mark_start()
        t_start = time.time()
        r0 = self.rounds
        n = self._run_native() if is_gpu(self.device) else self._run_cpu()
        if is_gpu(self.device):
            torch.cuda.synchronize(self.device)
        self.rounds += n
        elapsed = time.time() - t_start
        out = {"rounds": self.rounds, "updates": self.rounds * self.world, "elapsed_s": elapsed,
               "updates_per_s": (self.rounds - r0) * self.world / elapsed if elapsed > 0 else 0.0,
               "max_vc_gap": int(self.tracker.max_gap) if self.tracker is not None else 0,
               "keyrange": {"lo": self.lo, "hi": self.hi, "weight_bytes": self.weight_bytes(),
                            "model_bytes": self.model_bytes, "eval_bytes": self.eval_bytes,
                            "last_round_bytes": self.last_round_bytes, "last_u": self.last_u}}
        if self.log is not None and self.log.book is not None:
            out.update(summarize(self.log.book))
        return out

    def close(self):
        self._loop = None
        comm, self.comm = self.comm, None
        if comm is not None:
            comm.close()

    # ------------------------------------------------------------------ GPU
    def _run_native(self) -> int:
        cfg = self.cfg
        if self._loop is None:
            if self.world > 1:
                from .comm import make_comm

                self.comm = make_comm(self.rank, self.world, self.device)
                if self.comm is None:
                    raise RuntimeError("key-range sharding on GPUs needs the native RCCL communicator")
            h = _native.hip()
            sp, o, so = self.spec, cfg.solver, self.solver
            c = h.WideCfg()
            c.K, c.KP, c.F, c.cap, c.NZ = sp.K, sp.KP, sp.F, self.ring.cap, self.ring.NZ
            c.iters, c.hist, c.ls_max, c.nslots = o.iters, o.hist, o.ls_max, o.nslots
            c.mode = 1 if o.mode == "gd" else 0
            c.gd_lr, c.tol = o.gd_lr, o.tol
            c.standardize, c.center, c.zero_const = int(o.standardize), int(o.center), int(o.zero_const)
            tr, te, ts, rg = self.train, self.test, self.test_shard, self.ring
            d = dict(wcfg=c, use_graph=int(o.use_graph is not False), indptr=tr.indptr.data_ptr(),
                     idx=tr.idx.data_ptr(), val=tr.val.data_ptr(), y=tr.y.data_ptr(), ds_rows=tr.rows, k=self.rank,
                     N=self.world, per_iter_rows=cfg.rows_per_iter if cfg.stream_mode == "per_iter" else 0,
                     p_ms=float(cfg.producer_time_per_event), epochs=cfg.epochs, t0_ms=self.t0 * 1000.0,
                     ridx=rg.idx.data_ptr(), rval=rg.val.data_ptr(), rnnz=rg.nnz.data_ptr(), ry=rg.y.data_ptr(),
                     trunc=rg.trunc.data_ptr(), window=self.window.handle, shard=self.shard.data_ptr(),
                     b=self.b.data_ptr(), lr=float(self.lr), dloc=so.dloc.data_ptr(), wloc=so.wloc.data_ptr(),
                     loss=so.loss.data_ptr(), stats=so.stats.data_ptr(), uniq=so.uniq.data_ptr(),
                     sink=self.log.native.handle if self.log is not None else 0, log_server=1,
                     log_workers=int(cfg.log_workers), tracker=self.tracker.handle if self.tracker else 0,
                     api=_native.host.capi())
            if te is not None:
                d.update(t_indptr=te.indptr.data_ptr(), t_idx=te.idx.data_ptr(), t_val=te.val.data_ptr(),
                         t_y=te.y.data_ptr(), T=te.rows, s_indptr=ts.indptr.data_ptr(), s_idx=ts.idx.data_ptr(),
                         s_val=ts.val.data_ptr())
            self._loop = h.KeyRangeLoop(d, self.comm.c if self.comm is not None else None)
        lp = self._loop
        n = lp.run(int(cfg.max_iters), int(self.rounds), stream_handle(self.device))
        self.model_bytes, self.eval_bytes = lp.model_bytes, lp.eval_bytes
        self.last_round_bytes = lp.last_round_bytes
        torch.cuda.synchronize(self.device)
        self.last_u = lp.last_u
        if int(self.solver.stats[4].item()):
            from ..runtime.faults import WorkerFailure

            raise WorkerFailure(self.rank, "device solver: a cross-workgroup wait timed out")
        return n

    # ------------------------------------------------------------------ CPU
    def _a2a(self, x: torch.Tensor, out_rows: int, in_splits, out_splits) -> torch.Tensor:
        out = torch.empty((out_rows,) + tuple(x.shape[1:]), dtype=x.dtype)
        if self.world == 1:
            out.copy_(x)
        else:
            dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits)
        return out

    def _margins_cpu(self) -> torch.Tensor:
        sp = self.spec
        n = self.hi - self.lo
        z = _csr_mm(self.test_shard, self.shard[: n * sp.KP].view(n, sp.KP))
        if self.world > 1:
            dist.all_reduce(z)
            self.eval_bytes += z.numel() * 4
        return z

    def _run_cpu(self) -> int:
        cfg, sp, so = self.cfg, self.spec, self.solver
        W, KP = self.world, sp.KP
        ev = self.test is not None and self.log is not None
        if ev and self._z is None:
            self._z = self._margins_cpu()
        done = 0
        while done < cfg.max_iters:
            r = self.rounds + done
            rb = 0
            while True:  # BSP: every worker has rows (a worker out of data ends the run everywhere)
                self.source.poll()
                ok = torch.tensor([1 if int(self.window.size) > 0 else 0])
                if W > 1:
                    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if int(ok) == 1:
                    break
                stop = torch.tensor([1 if self.source.exhausted else 0])
                if W > 1:
                    dist.all_reduce(stop, op=dist.ReduceOp.MAX)
                if int(stop):
                    return done
                time.sleep(0.001)
            B, start, seen = int(self.window.size), int(self.window.start), int(self.window.tuples_seen)
            # plan + pull
            ids = so.plan_cpu(self.ring, B, start)
            owner = torch.clamp(ids.long() // self.S, max=W - 1)
            scnt = torch.bincount(owner, minlength=W)
            rcnt = self._a2a(scnt, W, [1] * W, [1] * W)
            sl, rl = scnt.tolist(), rcnt.tolist()
            req = self._a2a(ids, sum(rl), sl, rl)
            n = self.hi - self.lo
            shard2 = self.shard[: n * KP].view(n, KP)
            ans = shard2[req.long() - self.lo]
            w_pull = self._a2a(ans, len(ids), rl, sl)
            rb += 4 * (W - 1) + 4 * (sum(sl) - sl[self.rank]) + 4 * KP * (sum(rl) - rl[self.rank])
            # the local solve in the window subspace
            so.finish_cpu(w_pull, self.b)
            U = int(ids.numel())
            dl = so.dloc[KP: KP + U * KP].view(U, KP)
            # push: deltas of the pulled ids to their owners, applied in sender order
            got = self._a2a(dl, sum(rl), sl, rl)
            rb += 4 * KP * (sum(sl) - sl[self.rank])
            off = 0
            for j in range(W):
                rows = req[off: off + rl[j]].long() - self.lo
                shard2.index_add_(0, rows, got[off: off + rl[j]] * self.lr)
                off += rl[j]
            db = so.dloc[:KP].clone()
            if W > 1:
                dist.all_reduce(db)
                rb += 4 * KP
            self.b += self.lr * db
            self.model_bytes += rb
            self.last_round_bytes = rb
            self.last_u = U
            # rows: the server's global model (rank 0), this worker's local model
            if ev:
                z_prev = self._z
                self._z = self._margins_cpu()
                if self.rank == 0:
                    self._row(self._z + self.b, 1, r, -1, 0, None)
                if cfg.log_workers:
                    zw = z_prev.clone()
                    te = self.test
                    if U:  # the window's features of each test row: + value * delta
                        pos = torch.searchsorted(ids, te.idx).clamp(max=U - 1)
                        hit = ids[pos] == te.idx
                        row = torch.repeat_interleave(torch.arange(te.rows), te.indptr[1:] - te.indptr[:-1])
                        zw.index_add_(0, row[hit], te.val[hit].float().unsqueeze(1) * dl[pos[hit]])
                    zw += so.wloc[:KP]
                    self._row(zw, 0, r, self.rank, seen, float(so.loss.item()))
            if self.tracker is not None:
                self.tracker.bsp_round(r)
            done += 1
        return done

    def _row(self, z: torch.Tensor, kind: int, vc: int, partition: int, nseen: int, loss):
        nat = self.log.native
        slot, seq, addr = nat.acquire()
        _write_slot_cpu(addr, _confusion(z, self.test.y, self.spec.K), loss or 0.0, seq)
        nat.submit(slot, seq, kind, -1, int(partition), int(vc), int(nseen))


__all__ = ["KeyRangeEngine", "key_range", "shard_csr"]
