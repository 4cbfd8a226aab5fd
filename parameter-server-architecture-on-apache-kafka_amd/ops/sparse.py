"""Device ops of the wide / sparse logistic-regression model.

GPU: the hand-written HIP kernels of ``csrc/kernels/wide_kernels.hip`` (the
local solve is the native :class:`WideSolver`, one hipGraph per solve).  There
is no PyTorch fallback on the device.  CPU: the same math on torch, in the
window's feature subspace, with :func:`psx.models.reference.local_solve_reference`
as the solver -- the oracle the GPU path is tested against.
"""
from __future__ import annotations

import warnings
from dataclasses import dataclass

import torch

from .. import _native
from ..models.reference import local_solve_reference
from ..models.wide import WideSpec
from .lr import SolverOptions, _write_slot_cpu, is_gpu, stream_handle


@dataclass
class SparseDataset:
    """CSR rows: ``indptr`` int64 [N+1], ``idx`` int32 [nnz], ``val`` bf16 [nnz], labels int32 [N]."""

    indptr: torch.Tensor
    idx: torch.Tensor
    val: torch.Tensor
    y: torch.Tensor
    num_features: int

    @property
    def rows(self) -> int:
        return int(self.y.shape[0])

    @property
    def nnz(self) -> int:
        return int(self.idx.shape[0])

    @property
    def max_nnz(self) -> int:
        if self.rows == 0:
            return 0
        return int((self.indptr[1:] - self.indptr[:-1]).max().item())

    @property
    def device(self):
        return self.idx.device

    def to(self, device) -> "SparseDataset":
        return SparseDataset(self.indptr.to(device), self.idx.to(device), self.val.to(device), self.y.to(device),
                             self.num_features)

    def slice(self, r0: int, r1: int) -> "SparseDataset":
        a, b = int(self.indptr[r0]), int(self.indptr[r1])
        return SparseDataset(self.indptr[r0:r1 + 1] - a, self.idx[a:b], self.val[a:b], self.y[r0:r1], self.num_features)

    def dense(self, rows=None) -> torch.Tensor:
        """float32 [n, F] of the given rows (tests; small F only)."""
        rows = torch.arange(self.rows) if rows is None else torch.as_tensor(rows)
        ip = self.indptr.cpu()
        out = torch.zeros(len(rows), self.num_features, dtype=torch.float32)
        for i, r in enumerate(rows.tolist()):
            a, b = int(ip[r]), int(ip[r + 1])
            out[i].index_add_(0, self.idx[a:b].cpu().long(), self.val[a:b].cpu().float())
        return out


class SparseRing:
    """ELL ring of one worker: ``cap`` slots of up to ``NZ`` non-zeros each."""

    def __init__(self, cap: int, NZ: int, device):
        self.cap, self.NZ, self.device = int(cap), int(NZ), torch.device(device)
        if not 1 <= self.NZ <= 512:
            raise ValueError(f"ring rows hold 1..512 non-zeros (got {NZ})")
        self.idx = torch.zeros(self.cap, self.NZ, dtype=torch.int32, device=self.device)
        self.val = torch.zeros(self.cap, self.NZ, dtype=torch.bfloat16, device=self.device)
        self.nnz = torch.zeros(self.cap, dtype=torch.int32, device=self.device)
        self.y = torch.zeros(self.cap, dtype=torch.int32, device=self.device)
        self.trunc = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.batch: IngestBatch | None = None  # set: deliveries are collected, one launch for every ring

    def ingest_from(self, ds: SparseDataset, src_first: int, src_step: int, n: int, dst_first: int):
        """Copy rows src_first + i*src_step (i < n) of ``ds`` into slots (dst_first + i) % cap."""
        if n <= 0:
            return
        if self.batch is not None and is_gpu(self.device):
            self.batch.add(self, ds, src_first, src_step, n, dst_first)
            return
        if is_gpu(self.device):
            _native.hip().sparse_ring_ingest(ds.indptr.data_ptr(), ds.idx.data_ptr(), ds.val.data_ptr(),
                                             ds.y.data_ptr(), int(src_first), int(src_step), int(n),
                                             self.idx.data_ptr(), self.val.data_ptr(), self.nnz.data_ptr(),
                                             self.y.data_ptr(), int(dst_first), self.cap, self.NZ,
                                             self.trunc.data_ptr(), stream_handle(self.device))
            return
        src = torch.arange(n) * src_step + src_first
        dst = (torch.arange(n) + dst_first) % self.cap
        ip = ds.indptr
        for s, d in zip(src.tolist(), dst.tolist()):
            a, b = int(ip[s]), int(ip[s + 1])
            k = min(b - a, self.NZ)
            if b - a > self.NZ:
                self.trunc += 1
            self.idx[d, :k] = ds.idx[a:a + k]
            self.val[d, :k] = ds.val[a:a + k]
            self.nnz[d] = k
            self.y[d] = ds.y[s]


class IngestBatch:
    """Deliveries of several :class:`SparseRing` s (one geometry, one dataset) collected
    and copied in ONE launch (the wide lanes' rounds: one ingest launch, not one per
    worker and epoch split)."""

    def __init__(self):
        self.jobs: list[list[int]] = []
        self.ds = None
        self.geom = None

    def add(self, ring: SparseRing, ds: SparseDataset, src_first: int, src_step: int, n: int, dst_first: int):
        if (self.ds is not None and ds is not self.ds) or (self.geom is not None and self.geom != (ring.cap, ring.NZ)) \
                or len(self.jobs) >= 16:
            self.flush(ring.device)
        self.ds, self.geom = ds, (ring.cap, ring.NZ)
        self.jobs.append([int(src_first), int(src_step), int(n), int(dst_first), ring.idx.data_ptr(),
                          ring.val.data_ptr(), ring.nnz.data_ptr(), ring.y.data_ptr(), ring.trunc.data_ptr()])

    def flush(self, device):
        if self.jobs:
            ds = self.ds
            _native.hip().sparse_ring_ingest_many(ds.indptr.data_ptr(), ds.idx.data_ptr(), ds.val.data_ptr(),
                                                  ds.y.data_ptr(), self.jobs, self.geom[0], self.geom[1],
                                                  stream_handle(device))
        self.jobs, self.ds, self.geom = [], None, None


class SparseDelta:
    """A worker's push in the window subspace: ``dloc`` = KP intercepts then U*KP coefficients of features ``uniq``."""

    def __init__(self, spec: WideSpec, uniq: torch.Tensor, dloc: torch.Tensor, count: int | None, count_ptr: int = 0):
        self.spec, self.uniq, self.dloc = spec, uniq, dloc
        self.count = count  # host-known U (None: only on device, count_ptr)
        self.count_ptr = count_ptr

    def to_dense(self) -> torch.Tensor:
        s = self.spec
        U = self.host_count()
        out = torch.zeros(s.P, dtype=torch.float32, device=self.dloc.device)
        out[s.F * s.KP:] = self.dloc[: s.KP]
        if U:
            rows = self.uniq[:U].long()
            out[: s.F * s.KP].view(s.F, s.KP)[rows] = self.dloc[s.KP: s.KP + U * s.KP].view(U, s.KP)
        return out

    def host_count(self) -> int:
        if self.count is None:
            raise RuntimeError("delta size is only known on the device")
        return int(self.count)


class WideSolveOp:
    """One worker's local solve on a :class:`SparseRing` window -> delta (sparse, and dense if asked)."""

    def __init__(self, spec: WideSpec, cap: int, NZ: int, device, opts: SolverOptions, dense_delta: bool = False):
        self.spec, self.cap, self.NZ, self.device, self.opts = spec, int(cap), int(NZ), torch.device(device), opts
        self.umax = min(spec.F, self.cap * self.NZ)
        self.plmax = spec.KP + self.umax * spec.KP
        dev = self.device
        self.dloc = torch.zeros(self.plmax, dtype=torch.float32, device=dev)
        self.wloc = torch.zeros(self.plmax, dtype=torch.float32, device=dev)
        self.uniq = torch.zeros(self.umax, dtype=torch.int32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.stats = torch.zeros(8, dtype=torch.int32, device=dev)
        self.dense_delta = bool(dense_delta)
        self.delta = torch.zeros(spec.P, dtype=torch.float32, device=dev) if dense_delta else None
        self._native = None
        self._bound = None
        self._count_cpu = 0
        self._map_cpu = None  # CPU: feature -> local id of the last solve

    # -- native binding ------------------------------------------------------
    def _bind(self, ring: SparseRing, w_old: torch.Tensor):
        key = (ring.idx.data_ptr(), w_old.data_ptr())
        if self._bound == key:
            return
        h = _native.hip()
        s, o = self.spec, self.opts
        c = h.WideCfg()
        c.K, c.KP, c.F, c.cap, c.NZ = s.K, s.KP, s.F, self.cap, self.NZ
        c.iters, c.hist, c.ls_max, c.nslots = o.iters, o.hist, o.ls_max, o.nslots
        c.mode = 1 if o.mode == "gd" else 0
        c.gd_lr, c.tol = o.gd_lr, o.tol
        c.standardize, c.center, c.zero_const = int(o.standardize), int(o.center), int(o.zero_const)
        c.dense_delta = int(self.dense_delta)
        self._native = h.WideSolver(c, ring.idx.data_ptr(), ring.val.data_ptr(), ring.nnz.data_ptr(),
                                    ring.y.data_ptr(), w_old.data_ptr(), self.dloc.data_ptr(), self.wloc.data_ptr(),
                                    self.loss.data_ptr(), self.stats.data_ptr(), self.uniq.data_ptr(),
                                    self.delta.data_ptr() if self.delta is not None else 0,
                                    o.use_graph is not False)
        self._bound = key

    @property
    def table(self) -> tuple[int, int]:
        """(device pointer, mask) of the feature -> local id table of the last solve."""
        if self._native is None:
            return 0, 0
        return self._native.table_ptr, self._native.table_mask

    def run(self, ring: SparseRing, B: int, start: int, w_old: torch.Tensor):
        if B <= 0:
            raise ValueError("local solve on an empty buffer")
        if ring.cap != self.cap or ring.NZ != self.NZ:
            raise ValueError("ring geometry differs from the solver's")
        if w_old.numel() != self.spec.P or w_old.dtype != torch.float32:
            raise ValueError("w_old must be fp32 [F*KP + KP]")
        if is_gpu(self.device):
            self._bind(ring, w_old)
            self._native.run(int(B), int(start), stream_handle(self.device))
            return
        self._run_cpu(ring, B, start, w_old)

    def barrier_errors(self) -> int:
        """Sticky flag: a grid barrier of the device solver timed out (see LocalSolveOp)."""
        return int(self.stats[4].item()) if is_gpu(self.device) else 0

    def sparse_delta(self) -> SparseDelta:
        if is_gpu(self.device):
            return SparseDelta(self.spec, self.uniq, self.dloc, None, self._native.ucount_ptr)
        return SparseDelta(self.spec, self.uniq, self.dloc, self._count_cpu)

    def host_count(self) -> int:
        """U of the last solve (GPU: valid once the stream has synchronised)."""
        return int(self._native.ucount_host) if is_gpu(self.device) else self._count_cpu

    # -- CPU oracle path ---------------------------------------------------------
    def _run_cpu(self, ring: SparseRing, B: int, start: int, w_old: torch.Tensor):
        s = self.spec
        uniq = self.plan_cpu(ring, B, start)
        W = w_old[: s.F * s.KP].view(s.F, s.KP)
        self.finish_cpu(W[uniq.long()], w_old[s.F * s.KP:])

    def plan_cpu(self, ring: SparseRing, B: int, start: int) -> torch.Tensor:
        """Phase 1 of a pulled solve (CPU): the window's distinct features, sorted
        (= grouped by key-range owner).  The caller pulls their coefficients and
        calls :meth:`finish_cpu`."""
        slots = ((torch.arange(B) + start) % self.cap).tolist()
        feats = [ring.idx[sl, : int(ring.nnz[sl])] for sl in slots]
        uniq = torch.unique(torch.cat(feats)) if feats else torch.zeros(0, dtype=torch.int32)
        self._plan = (slots, uniq.to(torch.int32), ring)
        return self._plan[1]

    def finish_cpu(self, w_pull: torch.Tensor, b_old: torch.Tensor):
        """Phase 2 (CPU): the local solve from the pulled coefficients ``w_pull``
        [U, KP] of the planned features and the intercepts ``b_old`` [KP]."""
        s, o = self.spec, self.opts
        slots, uniq, ring = self._plan
        B = len(slots)
        U = int(uniq.numel())
        pos = {int(f): i for i, f in enumerate(uniq.tolist())}
        X = torch.zeros(B, U, dtype=torch.float64)
        for r, sl in enumerate(slots):
            k = int(ring.nnz[sl])
            for f, v in zip(ring.idx[sl, :k].tolist(), ring.val[sl, :k].float().tolist()):
                X[r, pos[f]] += v
        y = ring.y[slots].long()
        coef_old = w_pull[:, : s.K].t().double() if U else torch.zeros(s.K, 0, dtype=torch.float64)
        b_old = b_old[: s.K].double()
        res = local_solve_reference(X, y, coef_old, b_old, iters=o.iters, hist=o.hist, ls_max=o.ls_max,
                                    nslots=o.nslots, mode=o.mode, gd_lr=o.gd_lr, center=o.center,
                                    zero_const=o.zero_const, tol=o.tol, standardize=o.standardize)
        self.dloc.zero_()
        self.wloc.zero_()
        self.dloc[: s.K] = res.delta_intercept
        self.wloc[: s.K] = res.intercept
        if U:
            self.dloc[s.KP: s.KP + U * s.KP].view(U, s.KP)[:, : s.K] = res.delta_coef.t()
            self.wloc[s.KP: s.KP + U * s.KP].view(U, s.KP)[:, : s.K] = res.coef.t()
            self.uniq[:U] = uniq
        self._count_cpu = U
        self._map_cpu = pos
        self.loss.fill_(res.loss)
        self.stats.copy_(torch.tensor([res.evals, res.accepted, res.ls_fail, 0, 0, 0, 0, 0], dtype=torch.int32))
        if self.delta is not None:
            self.delta.copy_(self.sparse_delta().to_dense())

    def local_model(self, w_old: torch.Tensor) -> torch.Tensor:
        """Dense locally trained model (CPU evaluation / tests)."""
        return w_old + self.sparse_delta().to_dense().to(w_old.device)


class WideEvalSet:
    """Test rows (CSR) resident on the device + argmax / confusion evaluation."""

    def __init__(self, spec: WideSpec, test: SparseDataset, device):
        self.spec = spec
        self.device = torch.device(device)
        if test.num_features > spec.F:
            raise ValueError(f"test set has {test.num_features} features, model {spec.F}")
        self.ds = test.to(self.device)
        self.T = test.rows
        self._csr = None

    def _margins_cpu(self, w: torch.Tensor) -> torch.Tensor:
        s = self.spec
        if self._csr is None:
            ds = self.ds
            with warnings.catch_warnings():  # "sparse CSR support is in beta"
                warnings.simplefilter("ignore", UserWarning)
                self._csr = torch.sparse_csr_tensor(ds.indptr, ds.idx.long(), ds.val.float(), size=(ds.rows, s.F))
        W = w[: s.F * s.KP].view(s.F, s.KP).float()
        return (self._csr @ W) + w[s.F * s.KP:].float()

    def predict_cpu(self, w: torch.Tensor) -> torch.Tensor:
        z = self._margins_cpu(w)
        if self.spec.K == 1:
            return (z[:, 0] > 0).long()
        return z[:, : self.spec.K].argmax(1)

    def confusion_cpu(self, w: torch.Tensor) -> torch.Tensor:
        pred = self.predict_cpu(w)
        y = self.ds.y.long()
        if self.spec.K == 1:
            y = (y > 0).long()
        y = y.clamp(0, 15)
        c = torch.zeros(256, dtype=torch.int64)
        c.index_add_(0, y * 16 + pred, torch.ones_like(y))
        return c.to(torch.int32)

    def eval_to_slot(self, overlay, w: torch.Tensor, scratch, slot_addr: int, seq: int, loss: torch.Tensor | None = None):
        """Confusion counts of ``w`` (overlaid with a worker's local solution when
        ``overlay`` is a :class:`WideSolveOp`) into the host EvalSlot at ``slot_addr``."""
        s = self.spec
        if is_gpu(self.device):
            tab, mask = overlay.table if overlay is not None else (0, 0)
            wloc_ptr = overlay.wloc.data_ptr() if overlay is not None else 0
            _native.hip().wide_eval(s.K, s.KP, s.F, self.ds.indptr.data_ptr(), self.ds.idx.data_ptr(),
                                    self.ds.val.data_ptr(), self.ds.y.data_ptr(), self.T, w.data_ptr(), tab, mask,
                                    wloc_ptr, scratch.acc.data_ptr(), scratch.ticket.data_ptr(), int(slot_addr),
                                    loss.data_ptr() if loss is not None else 0, int(seq), stream_handle(self.device))
            return
        weff = overlay.local_model(w) if overlay is not None else w
        _write_slot_cpu(slot_addr, self.confusion_cpu(weff), float(loss.item()) if loss is not None else 0.0, seq)

    def eval_pair_to_slots(self, overlay, w_a: torch.Tensor, _frag_b, w_b: torch.Tensor, scratch, slot_a: int,
                           seq_a: int, loss_a, slot_b: int, seq_b: int, apply=None):
        """Row a: ``w_a`` overlaid with the worker's local solution; row b: the plain
        global model ``w_b``.  On the GPU, when ``w_b`` IS ``w_a`` (the worker
        trained from the current global model), both come from ONE pass: the two
        models differ only on the window's features."""
        if apply is not None:
            raise ValueError("the wide evaluation does not fuse the server update")
        if (is_gpu(self.device) and slot_b and overlay is not None and w_a.data_ptr() == w_b.data_ptr()):
            s = self.spec
            _native.hip().wide_eval(s.K, s.KP, s.F, self.ds.indptr.data_ptr(), self.ds.idx.data_ptr(),
                                    self.ds.val.data_ptr(), self.ds.y.data_ptr(), self.T, w_a.data_ptr(),
                                    *overlay.table, overlay.wloc.data_ptr(), scratch.acc.data_ptr(),
                                    scratch.ticket.data_ptr(), int(slot_a),
                                    loss_a.data_ptr() if loss_a is not None else 0, int(seq_a),
                                    stream_handle(self.device), int(slot_b), int(seq_b))
            return
        self.eval_to_slot(overlay, w_a, scratch, slot_a, seq_a, loss_a)
        if slot_b:
            self.eval_to_slot(None, w_b, scratch, slot_b, seq_b, None)


def wide_server_apply(spec: WideSpec, w: torch.Tensor, delta, lr: float):
    """w += lr * delta; ``delta`` dense [P] or a :class:`SparseDelta`."""
    gpu = is_gpu(w.device)
    if isinstance(delta, SparseDelta):
        if gpu:
            umax = int(delta.uniq.numel())
            _native.hip().wide_apply_sparse(w.data_ptr(), spec.F, spec.KP, delta.count_ptr if delta.count is None else 0,
                                            int(delta.count or 0), delta.uniq.data_ptr(), delta.dloc.data_ptr(),
                                            float(lr), umax, stream_handle(w.device))
        else:
            U = delta.host_count()
            w[spec.F * spec.KP:] += lr * delta.dloc[: spec.KP]
            if U:
                rows = delta.uniq[:U].long()
                w[: spec.F * spec.KP].view(spec.F, spec.KP)[rows] += lr * delta.dloc[spec.KP: spec.KP + U * spec.KP].view(U, spec.KP)
        return
    if gpu:
        _native.hip().axpy(w.data_ptr(), delta.data_ptr(), float(lr), int(w.numel()), stream_handle(w.device))
    else:
        w.add_(delta, alpha=lr)


def wide_logits(spec: WideSpec, ds: SparseDataset, w: torch.Tensor) -> torch.Tensor:
    """[T, KP] margins of a CSR set (tests)."""
    out = torch.zeros(ds.rows, spec.KP, dtype=torch.float32, device=w.device)
    if is_gpu(w.device):
        _native.hip().wide_logits(spec.K, spec.KP, spec.F, ds.indptr.data_ptr(), ds.idx.data_ptr(), ds.val.data_ptr(),
                                  ds.rows, w.data_ptr(), out.data_ptr(), stream_handle(w.device))
        return out
    ev = WideEvalSet(spec, ds, w.device)
    return ev._margins_cpu(w)[:, : spec.KP]


def nz_capacity(max_nnz: int) -> int:
    """Ring row width for rows of up to ``max_nnz`` non-zeros (multiple of 8, <= 512)."""
    n = max(8, -(-int(max_nnz) // 8) * 8)
    if n > 512:
        raise ValueError(f"rows with {max_nnz} non-zeros exceed the 512-entry ring rows")
    return n


__all__ = ["SparseDataset", "SparseRing", "IngestBatch", "SparseDelta", "WideSolveOp", "WideEvalSet", "wide_server_apply",
           "wide_logits", "nz_capacity"]
