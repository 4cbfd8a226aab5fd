"""Device ops for the logistic-regression parameter server.

On a GPU every op goes through the hand-written HIP kernels in ``_psx_hip``
(gfx950); there is no PyTorch fallback on the device -- a missing extension is
a hard error.  On the CPU (tests, the plumbing config of BASELINE.json #1) the
same ops run the PyTorch reference in :mod:`psx.models.reference`.
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import numpy as np
import torch

from .. import _native
from ..models.logreg import ModelSpec
from ..models.reference import local_solve_reference


def is_gpu(device) -> bool:
    return torch.device(device).type == "cuda"


_DEV_INDEX: dict = {}


def stream_handle(device) -> int:
    """hipStream_t of the current stream of `device` (every native launch asks).
    torch.cuda.current_stream() builds a Stream object and re-resolves the device
    on each call; the raw accessor with a cached index is a single C call."""
    idx = _DEV_INDEX.get(device)
    if idx is None:
        d = torch.device(device)
        idx = d.index if d.index is not None else torch.cuda.current_device()
        _DEV_INDEX[device] = idx
    return torch._C._cuda_getCurrentRawStream(idx)


@dataclass
class SolverOptions:
    iters: int = 2  # reference numMaxIter (LogisticRegressionTaskSpark.java:35)
    hist: int = 10  # Spark/breeze L-BFGS history
    ls_max: int = 4  # line-search evaluations per iteration (device slot budget)
    mode: str = "lbfgs"  # or "gd"
    gd_lr: float = 1.0
    center: bool = True  # Spark centring when regParam == 0
    zero_const: bool = True  # Spark: zero-std features get coefficient 0
    tol: float = 1e-6
    standardize: bool = True  # Spark default; the dense MFMA solver always standardises
    # None = per-solver default: the dense solve launches eagerly (measured faster on
    # MI355X: a graph's completion barrier costs ~8 us before the next launch, more
    # than the 8 eager launches' host time, which the GPU-bound loop hides), the
    # wide solve replays one hipGraph
    use_graph: bool | None = None
    max_eval_wg: int = 512
    fused_ingest: bool = True  # GPU: new stream rows are copied into the ring by the solve's first kernel
    # the small-window solve as stats_prep + ONE persistent launch (its workgroups must
    # be co-resident: only for a solver that has the GPU to itself).  With <= 32 solve
    # workgroups they all run on one XCD and hand off through its L2: 57.6 us per
    # solve against 62.5 us for the 8-launch chain (profiles/r02_v5).  None = the
    # engine decides: LocalEngine turns it on for a lone GPU worker; DistEngine and
    # several in-process workers keep the chain (kernels of other streams -- RCCL,
    # other workers -- could hold the XCD's CUs the persistent workgroups wait for).
    persist: bool | None = None
    # XCD (0..7) of the persistent solve's workgroups / the chain's backward slices
    # (in-L2 hand-offs); -1: spread over the XCDs (sc1 hand-offs) -- for a solver
    # whose GPU runs other solvers' launches concurrently
    xcd: int = 0
    # False: no tail launch (its grid barriers need co-resident workgroups); every
    # budgeted line-search slot is its own launch pair -- for concurrent in-process workers
    tail: bool = True

    @property
    def nslots(self) -> int:
        return 1 + self.iters * (1 if self.mode == "gd" else self.ls_max)


class Fragments:
    """bf16 hi/lo MFMA-fragment copy of a weight vector + fp32 intercepts.

    The 16 fragment columns can carry two models: ``coff`` is the first class
    column of the model written through THIS handle (a worker's solver writes
    columns [0, KP), the colocated server [16 - K, 16); see EvalPair)."""

    def __init__(self, spec: ModelSpec, device, coff: int = 0, share: "Fragments | None" = None):
        self.spec = spec
        self.coff = int(coff)
        if share is not None:
            self.hi, self.lo, self.b = share.hi, share.lo, share.b
        else:
            self.hi = torch.zeros(16 * spec.Fp, dtype=torch.int16, device=device)
            self.lo = torch.zeros(16 * spec.Fp, dtype=torch.int16, device=device)
            self.b = torch.zeros(16, dtype=torch.float32, device=device)

    def refresh(self, w: torch.Tensor):
        s = self.spec
        _native.hip().make_fragments(s.K, s.F, s.Fp, w.data_ptr(), self.hi.data_ptr(), self.lo.data_ptr(),
                                     self.b.data_ptr(), stream_handle(w.device), self.coff)


class LocalSolveOp:
    """One worker's local solve: window of the device ring -> delta (+ new weights).

    GPU: a native LocalSolver whose whole kernel chain is one hipGraph replay.
    CPU: :func:`local_solve_reference`.
    """

    def __init__(self, spec: ModelSpec, cap: int, device, opts: SolverOptions):
        self.spec, self.cap, self.device, self.opts = spec, cap, torch.device(device), opts
        P = spec.P
        self.delta = torch.zeros(P, dtype=torch.float32, device=self.device)
        self.w_new = torch.zeros(P, dtype=torch.float32, device=self.device)
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.stats = torch.zeros(8, dtype=torch.int32, device=self.device)
        self.frag = Fragments(spec, self.device) if is_gpu(self.device) else None
        self._native = None
        self._bound = None

    def _bind(self, ring, w_old: torch.Tensor):
        xt = ring.XT.data_ptr() if ring.XT is not None else 0  # None: large-window (rows) solver
        key = (ring.X.data_ptr(), xt, ring.y.data_ptr(), w_old.data_ptr())
        if self._bound == key:
            return
        if (ring.X.dtype not in (torch.bfloat16, torch.float32) or ring.X.shape != (self.cap, self.spec.Fp)
                or ring.y.dtype != torch.int32):
            raise ValueError("ring must be bf16 / fp32 [cap, Fp] with int32 labels")
        h = _native.hip()
        s, o = self.spec, self.opts
        cfg = h.SolverCfg()
        cfg.K, cfg.F, cfg.Fp, cfg.P, cfg.cap = s.K, s.F, s.Fp, s.P, self.cap
        cfg.iters, cfg.hist, cfg.ls_max = o.iters, o.hist, o.ls_max
        cfg.mode = 1 if o.mode == "gd" else 0
        cfg.center, cfg.zero_const = int(o.center), int(o.zero_const)
        cfg.nslots, cfg.gd_lr, cfg.tol = o.nslots, o.gd_lr, o.tol
        cfg.xf32 = int(ring.X.dtype == torch.float32)
        cfg.persist = int(bool(o.persist))
        cfg.xcd = int(o.xcd) if o.xcd < 0 else int(o.xcd) % 8
        cfg.tail = int(bool(o.tail))
        self._native = h.LocalSolver(
            cfg, ring.X.data_ptr(), xt, ring.y.data_ptr(), w_old.data_ptr(), self.delta.data_ptr(),
            self.w_new.data_ptr(), self.frag.hi.data_ptr(), self.frag.lo.data_ptr(), self.frag.b.data_ptr(),
            self.loss.data_ptr(), self.stats.data_ptr(), o.max_eval_wg, bool(o.use_graph))
        self._bound = key

    def barrier_errors(self) -> int:
        """Sticky flag of the device solver: a cross-workgroup wait timed out (a
        workgroup was not co-resident) and a solve's result was garbage.  Reads
        the device (a stream sync): the engines check it at the end of a run."""
        return int(self.stats[4].item()) if self.frag is not None else 0

    def can_ride(self, ring, w_old: torch.Tensor) -> bool:
        """True when this solver can carry a riding evaluation pass (GPU, eager
        launches, small-window kernels): see :meth:`run`."""
        if self.frag is None:
            return False
        self._bind(ring, w_old)
        return bool(self._native.eager) and not bool(self._native.rows_mode)

    def run(self, ring, B: int, start: int, w_old: torch.Tensor, ride: dict | None = None,
            apply: tuple | None = None):
        """Enqueue a solve over the window [start, start+B) (mod cap) of ``ring`` (a DeviceRing).

        GPU extras (eager solver): ``ride`` = keyword arguments of an evaluation
        pass executed by spare workgroups of the solve's bwd_update launches
        (:class:`EvalRide`, csrc/kernels/lr_kernels.h); ``apply`` = (w, lr,
        Fragments): the colocated server's update ``w = w_old + lr * delta`` fused
        into the solve's finalisation, with that model's fragments written to the
        given buffer."""
        if B <= 0:
            raise ValueError("local solve on an empty buffer")
        if ring.cap != self.cap:
            raise ValueError(f"ring capacity {ring.cap} != solver capacity {self.cap}")
        X, y = ring.X, ring.y
        if self.frag is not None:  # GPU
            if getattr(ring, "xt_stale", False):  # rows written by the multi-lane round kernel
                ring.sync_transposed()
                ring.xt_stale = False
            self._bind(ring, w_old)
            pend = ring.take_pending(B, start) if hasattr(ring, "take_pending") else None
            if ride is None and apply is None:
                if pend is None:
                    self._native.run(int(B), int(start), stream_handle(self.device))
                else:
                    sX, sy, first, step, n, dst = pend
                    self._native.run_ingest(int(B), int(start), stream_handle(self.device), sX.data_ptr(),
                                            sy.data_ptr(), first, step, n, dst)
                return
            kw = dict(ride or {})
            if pend is not None:
                sX, sy, first, step, n, dst = pend
                kw.update(src=sX.data_ptr(), ysrc=sy.data_ptr(), first=int(first), step=int(step), n=int(n),
                          dst=int(dst))
            if apply is not None:
                w, lr, fo = apply
                kw.update(ap_w=w.data_ptr(), ap_lr=float(lr), ap_hi=fo.hi.data_ptr(), ap_lo=fo.lo.data_ptr(),
                          ap_b=fo.b.data_ptr(), ap_coff=fo.coff)
            self._native.run_full(int(B), int(start), stream_handle(self.device), **kw)
            return
        if ride is not None:
            raise ValueError("riding evaluation: GPU solver only")
        s, o = self.spec, self.opts
        idx = (torch.arange(B) + start) % self.cap
        Xw = X[idx, : s.F].float()
        yw = y[idx].long()
        res = local_solve_reference(
            Xw, yw, s.coef(w_old), s.intercept(w_old), iters=o.iters, hist=o.hist, ls_max=o.ls_max,
            nslots=o.nslots, mode=o.mode, gd_lr=o.gd_lr, center=o.center, zero_const=o.zero_const, tol=o.tol)
        self.w_new.copy_(s.pack(res.coef, res.intercept))
        self.delta.copy_(self.w_new - w_old)
        if apply is not None:  # the fused server update, same arithmetic as the kernel
            w, lr, _ = apply
            w.copy_(w_old + lr * self.delta)
        self.loss.fill_(res.loss)
        self.stats.copy_(torch.tensor([res.evals, res.accepted, res.ls_fail, 0, 0, 0, 0, 0], dtype=torch.int32))


class EvalSet:
    """Test data resident on the device + argmax/confusion evaluation."""

    def __init__(self, spec: ModelSpec, X: torch.Tensor, y: torch.Tensor, device):
        self.spec = spec
        self.device = torch.device(device)
        if X.shape[1] != spec.Fp:
            raise ValueError(f"test set width {X.shape[1]} != model Fp {spec.Fp}")
        self.X = X.to(self.device, torch.bfloat16).contiguous()
        self.y = y.to(self.device, torch.int32).contiguous()
        self.T = int(self.X.shape[0])
        self._Xf = None
        self.ell_idx = self.ell_val = None
        self.ell_nz = 0
        self._build_ell()

    def _build_ell(self, max_nz: int = 128):
        """The test rows in ELL form for the evaluation passes that read the whole set per
        update (the asynchronous lanes): [T][nz] feature ids (int16) + bf16 values, nonzeros
        first in feature order, nz = the longest row rounded up to 8.  The hashed
        bag-of-words rows of the reference's data are sparse (the reference itself builds
        Vectors.sparse rows, LogisticRegressionTaskSpark.java:146-162): ~34 of 1,024 in the
        synthetic set, 1.3 MB instead of 10 MB per pass.  Only when nz <= max_nz and the
        rows are at most 1/4 dense (PSX_SPARSE_EVAL=0: never)."""
        if not is_gpu(self.device) or self.T == 0 or os.environ.get("PSX_SPARSE_EVAL", "1") == "0":
            return
        mask = self.X != 0
        mx = int(mask.sum(1).max().item())
        nz = max(8, (mx + 7) // 8 * 8)
        if nz > max_nz or 4 * nz > self.spec.Fp:
            return
        order = torch.argsort((~mask).to(torch.int8), dim=1, stable=True)[:, :nz]
        keep = torch.gather(mask, 1, order)
        self.ell_idx = torch.where(keep, order, torch.zeros_like(order)).to(torch.int16).contiguous()
        self.ell_val = torch.where(keep, torch.gather(self.X, 1, order), torch.zeros((), dtype=self.X.dtype,
                                                                                   device=self.device)).contiguous()
        self.ell_nz = nz

    def ell_args(self) -> dict:
        """The native loops' ELL arguments (tnz 0: the dense pass)."""
        if self.ell_idx is None:
            return {}
        return {"Ti": self.ell_idx.data_ptr(), "Tv": self.ell_val.data_ptr(), "tnz": int(self.ell_nz)}

    def confusion_async(self, frag: Fragments | None, w: torch.Tensor, out: torch.Tensor):
        """Write the [16,16] confusion counts of model ``w`` into ``out`` (int32)."""
        s = self.spec
        if is_gpu(self.device):
            out.zero_()
            _native.hip().test_eval(s.Fp, s.K, self.X.data_ptr(), self.y.data_ptr(), self.T, frag.hi.data_ptr(),
                                    frag.lo.data_ptr(), frag.b.data_ptr(), out.data_ptr(), stream_handle(self.device))
            return
        if self._Xf is None:
            self._Xf = self.X[:, : s.F].float()
        pred = (self._Xf @ s.coef(w).t() + s.intercept(w)).argmax(1)
        yy = self.y.long().clamp(0, 15)
        c = torch.zeros(16 * 16, dtype=torch.int64)
        c.index_add_(0, yy * 16 + pred, torch.ones_like(yy))
        out.view(-1).copy_(c.to(torch.int32))


    def eval_to_slot(self, frag: Fragments | None, w: torch.Tensor, scratch: "EvalScratch", slot_addr: int, seq: int,
                     loss: torch.Tensor | None = None):
        """Confusion counts of ``w`` (+ ``loss``) into the host EvalSlot at ``slot_addr``, published with ``seq``.

        GPU: one kernel; its last workgroup writes the pinned slot directly and
        releases ``seq`` (no fill / copy / event).  CPU: computed here.
        """
        s = self.spec
        if is_gpu(self.device):
            _native.hip().test_eval(s.Fp, s.K, self.X.data_ptr(), self.y.data_ptr(), self.T, frag.hi.data_ptr(),
                                    frag.lo.data_ptr(), frag.b.data_ptr(), scratch.acc.data_ptr(),
                                    stream_handle(self.device), scratch.ticket.data_ptr(), int(slot_addr),
                                    loss.data_ptr() if loss is not None else 0, int(seq), frag.coff)
            return
        conf = torch.zeros(256, dtype=torch.int32)
        self.confusion_async(None, w, conf)
        _write_slot_cpu(slot_addr, conf, float(loss.item()) if loss is not None else 0.0, seq)

    def ride_args(self, frag_a: "Fragments", frag_b: "Fragments | None", scratch: "EvalScratch", slot_a: int,
                  seq_a: int, loss_a, slot_b: int, seq_b: int) -> dict:
        """Keyword arguments of a riding evaluation pass (LocalSolveOp.run): model a
        (columns frag_a.coff..) -> slot_a with ``loss_a``; model b (its own buffer,
        columns frag_b.coff..; slot_b = 0: none) -> slot_b."""
        kw = dict(ride_Xt=self.X.data_ptr(), ride_yt=self.y.data_ptr(), ride_T=self.T, whi=frag_a.hi.data_ptr(),
                  wlo=frag_a.lo.data_ptr(), wb=frag_a.b.data_ptr(), coff1=frag_a.coff, acc=scratch.acc.data_ptr(),
                  ticket=scratch.ticket.data_ptr(), slot=int(slot_a), seq=int(seq_a),
                  loss=loss_a.data_ptr() if loss_a is not None else 0)
        if slot_b:
            if frag_b.coff < frag_a.coff + self.spec.K:
                raise ValueError("riding evaluation: model a's columns must precede model b's")
            kw.update(shi=frag_b.hi.data_ptr(), slo=frag_b.lo.data_ptr(), sb=frag_b.b.data_ptr(), coff2=frag_b.coff,
                      slot2=int(slot_b), seq2=int(seq_b))
        return kw

    def eval_pair_to_slots(self, frag_a: Fragments | None, w_a: torch.Tensor, frag_b: Fragments | None,
                           w_b: torch.Tensor, scratch: "EvalScratch", slot_a: int, seq_a: int, loss_a, slot_b: int,
                           seq_b: int, apply=None):
        """Model a (fragment columns frag_a.coff..) and model b (columns frag_b.coff..,
        its own buffer; slot_b = 0: no row for b) evaluated in ONE pass over the
        test set.  ``apply`` = (w, deltas, lr, frag_out): the same launch also does
        the server update w += lr * sum(deltas) with the new fragments written to
        ``frag_out`` (a buffer this launch does not read)."""
        s = self.spec
        if is_gpu(self.device):
            if frag_a.coff + s.K > frag_b.coff:
                raise ValueError("paired evaluation: model a's columns must precede model b's")
            w = ds = None
            lr, fo = 0.0, None
            if apply is not None:
                w, ds, lr, fo = apply
            _native.hip().eval_apply(
                s.Fp, s.K, s.F, self.X.data_ptr(), self.y.data_ptr(), self.T, frag_a.hi.data_ptr(),
                frag_a.lo.data_ptr(), frag_a.b.data_ptr(), frag_b.hi.data_ptr(), frag_b.lo.data_ptr(),
                frag_b.b.data_ptr(), scratch.acc.data_ptr(), stream_handle(self.device), scratch.ticket.data_ptr(),
                int(slot_a), loss_a.data_ptr() if loss_a is not None else 0, int(seq_a), frag_a.coff, frag_b.coff,
                int(slot_b), int(seq_b), w.data_ptr() if w is not None else 0,
                [d.data_ptr() for d in ds] if ds else [], float(lr), fo.hi.data_ptr() if fo else 0,
                fo.lo.data_ptr() if fo else 0, fo.b.data_ptr() if fo else 0)
            return
        self.eval_to_slot(frag_a, w_a, scratch, slot_a, seq_a, loss_a)
        if slot_b:
            self.eval_to_slot(frag_b, w_b, scratch, slot_b, seq_b, None)
        if apply is not None:
            w, ds, lr, _ = apply
            for d in ds:
                w.add_(d, alpha=lr)



ACC_STRIDE = 32


class EvalScratch:
    """Private accumulator + ticket of one evaluation caller (stays zero between calls)."""

    def __init__(self, device):
        # [2 models][16][16] cells, one per 128-B line (kAccStride in csrc/kernels/lr_kernels.h);
        # x kWideEvalCopies (8): the wide evaluation spreads its workgroups' atomics over copies
        self.acc = torch.zeros(8 * 2 * 256 * ACC_STRIDE, dtype=torch.int32, device=device)
        self.ticket = torch.zeros(8, dtype=torch.int32, device=device)


def _write_slot_cpu(addr: int, conf: torch.Tensor, loss: float, seq: int):
    import ctypes

    ctypes.memmove(addr, conf.contiguous().numpy().ctypes.data, 1024)
    ctypes.c_float.from_address(addr + 1024).value = loss
    # the native reader acquires seq; the GIL-held stores above are already visible
    ctypes.c_uint64.from_address(addr + 1032).value = int(seq)


def server_apply(spec: ModelSpec, w: torch.Tensor, delta: torch.Tensor, lr: float, frag: Fragments | None):
    """w += lr * delta over all P entries (quirk Q1 fixed) + refresh eval fragments."""
    if is_gpu(w.device):
        _native.hip().server_apply(spec.K, spec.F, spec.Fp, w.data_ptr(), delta.data_ptr(), float(lr),
                                   frag.hi.data_ptr(), frag.lo.data_ptr(), frag.b.data_ptr(), stream_handle(w.device),
                                   frag.coff)
    else:
        w.add_(delta, alpha=lr)


def confusion_to_numpy(conf: torch.Tensor, K: int) -> np.ndarray:
    return conf.view(16, 16)[:K, :K].cpu().numpy()
