"""Per-worker stream source + adaptive sliding-window buffer in device memory.

Reference: the INPUT_DATA_BUFFER key-value store + WorkerSamplingProcessor
(WorkerSamplingProcessor.java:50-135, WorkerApp.java:40-42) and the producer's
round-robin / rate-limited delivery (CsvProducer.java:36-87).

MI355X design:
* the whole training set is resident in HBM (bf16 rows; 90k x 1024 is 184 MB
  of 288 GB), so "delivering" a tuple is a device-side row copy into the
  worker's ring -- no host staging, no serialisation;
* worker k owns rows k, k+N, k+2N, ... (reference round-robin, ``row % N``);
* arrival times follow the reference producer schedule (burst of N*128 rows,
  then floor(1000/p) rows per second; native ``due_rows``), or, for
  throughput runs, a fixed number of rows per iteration;
* window bookkeeping (rate estimate, target size, O(1) slot choice) is the
  native :class:`SlidingWindow`; the device ring has capacity ``max`` rows
  rounded up to whole 32-row tiles.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .. import _native
from ..ops.lr import is_gpu, stream_handle


class DeviceRing:  # dense rows; the sparse (ELL) ring is psx.ops.sparse.SparseRing
    """Row ring of one worker.  ``cap`` is rounded up to whole 32-row tiles (the
    solver walks windows as ring-aligned tiles); on the GPU a feature-major copy
    ``XT`` [Fp][cap] is kept in step so the backward / statistics kernels read
    every 32-feature slice of a window contiguously."""

    TILE = 32
    MAX_DEFERRED = 1024  # kMaxFusedIngest (csrc/kernels/solver_ctrl.h)

    def __init__(self, cap: int, Fp: int, device, defer: bool = False, dtype: str = "bf16"):
        self.requested = int(cap)
        self.cap = -(-int(cap) // self.TILE) * self.TILE
        self.Fp, self.device = int(Fp), torch.device(device)
        if dtype not in ("bf16", "fp32"):
            raise ValueError(f"ring dtype must be bf16 or fp32, not {dtype!r}")
        self.f32 = dtype == "fp32"
        self.X = torch.zeros(self.cap, self.Fp, dtype=torch.float32 if self.f32 else torch.bfloat16,
                             device=self.device)
        self.y = torch.zeros(self.cap, dtype=torch.int32, device=self.device)
        # large windows (and fp32 rows): the solver streams row-parallel fused passes
        # and needs no feature-major copy (csrc/kernels/solve_kernels.h, "rows" mode)
        self.rows_mode = is_gpu(self.device) and (self.f32 or bool(_native.hip().solver_rows_mode(self.cap)))
        self.XT = (torch.zeros(self.Fp, self.cap, dtype=torch.bfloat16, device=self.device)
                   if is_gpu(self.device) and not self.rows_mode else None)
        # defer: the last ingest is not launched on its own but handed to the next
        # local solve, whose first kernel copies it (LocalSolveOp.run); any other
        # reader of the ring must call flush() first
        self.defer = bool(defer) and is_gpu(self.device) and not self.rows_mode
        self.pending = None

    def ingest(self, src_X: torch.Tensor, src_y: torch.Tensor, src_first: int, src_step: int, n: int, dst_first: int):
        """Copy rows src_first + i*src_step (i < n) into slots (dst_first + i) % cap."""
        if n <= 0:
            return
        self.flush()
        if self.defer and n <= self.MAX_DEFERRED and src_X.dtype == torch.bfloat16 and src_X.shape[1] == self.Fp:
            self.pending = (src_X, src_y, int(src_first), int(src_step), int(n), int(dst_first) % self.cap)
            return
        self._launch(src_X, src_y, src_first, src_step, n, dst_first)

    def flush(self):
        """Launch a deferred ingest now (stream order keeps it ahead of later readers)."""
        if self.pending is not None:
            p, self.pending = self.pending, None
            self._launch(*p)

    def take_pending(self, B: int, start: int):
        """The deferred ingest for a solve over [start, start+B), if its rows end that
        window (else it is launched on its own and None is returned)."""
        p = self.pending
        if p is None:
            return None
        n, dst = p[4], p[5]
        if (dst + n - 1) % self.cap != (start + B - 1) % self.cap:
            self.flush()
            return None
        self.pending = None
        return p

    def _launch(self, src_X, src_y, src_first, src_step, n, dst_first):
        if src_X.dtype != self.X.dtype:
            raise ValueError(f"ring holds {self.X.dtype} rows, the source has {src_X.dtype}")
        if is_gpu(self.device) and self.f32:
            _native.hip().ring_ingest_f32(src_X.data_ptr(), src_y.data_ptr(), int(src_first), int(src_step), int(n),
                                          self.X.data_ptr(), self.y.data_ptr(), int(dst_first), self.cap, self.Fp,
                                          stream_handle(self.device))
        elif is_gpu(self.device):
            _native.hip().ring_ingest(src_X.data_ptr(), src_y.data_ptr(), int(src_first), int(src_step), int(n),
                                      self.X.data_ptr(), self.XT.data_ptr() if self.XT is not None else 0,
                                      self.y.data_ptr(), int(dst_first),
                                      self.cap, self.Fp, stream_handle(self.device))
        else:
            src = torch.arange(n) * src_step + src_first
            dst = (torch.arange(n) + dst_first) % self.cap
            self.X[dst] = src_X[src]
            self.y[dst] = src_y[src]

    def ingest_from(self, ds, src_first: int, src_step: int, n: int, dst_first: int):
        self.ingest(ds.X, ds.y, src_first, src_step, n, dst_first)

    def place(self, X: torch.Tensor, y: torch.Tensor, first: int = 0):
        """Write rows X[i], y[i] into slots (first + i) % cap (tests, tools)."""
        self.flush()
        idx = (torch.arange(X.shape[0]) + int(first)) % self.cap
        idx = idx.to(self.device)
        self.X[idx] = X.to(self.device, self.X.dtype)
        self.y[idx] = y.to(self.device, torch.int32)
        self.sync_transposed()

    def sync_transposed(self):
        """Rebuild XT after direct writes to X."""
        self.flush()
        if self.XT is not None:
            self.XT.copy_(self.X.t())


class StreamSource:
    """Delivers worker ``k``'s shard of a dataset into its ring per the arrival schedule.

    mode "schedule": reference producer clock (``-p`` ms per event).
    mode "per_iter": ``rows_per_iter`` new rows at every poll (throughput runs).
    ``epochs``: how many passes over the shard (the reference stops after one).
    """

    def __init__(self, dataset, k: int, num_workers: int, ring: DeviceRing, window, *, p_ms: float = 200.0,
                 mode: str = "schedule", rows_per_iter: int = 0, epochs: int = 1, t0: float | None = None):
        self.ds, self.k, self.N, self.ring, self.win = dataset, int(k), int(num_workers), ring, window
        self.p_ms, self.mode, self.rows_per_iter, self.epochs = float(p_ms), mode, int(rows_per_iter), int(epochs)
        self.t0 = time.time() if t0 is None else t0
        total = dataset.rows
        self.local_total = max(0, (total - self.k + self.N - 1) // self.N) if total > self.k else 0
        self.next_local = 0  # cursor into this worker's row list (may span epochs)
        if self.local_total == 0:
            raise ValueError(f"worker {k} has no rows (dataset has {total} rows for {num_workers} workers)")

    @property
    def exhausted(self) -> bool:
        return self.next_local >= self.local_total * self.epochs

    def poll(self, now: float | None = None) -> int:
        """Ingest every due row; returns how many rows arrived."""
        if self.exhausted:
            return 0
        now = time.time() if now is None else now
        now_ms = (now - self.t0) * 1000.0
        limit = self.local_total * self.epochs - self.next_local
        if self.mode == "per_iter":
            n = min(self.rows_per_iter, limit)
            times = np.full(n, now_ms, dtype=np.float64)
        else:
            epoch = self.next_local // self.local_total
            cur = self.next_local - epoch * self.local_total
            n, times = _native.host.due_rows(self.k, self.N, self.p_ms, self.ds.rows, cur, now_ms,
                                             min(limit, self.local_total - cur, 1 << 22))
            times = times[:n] + epoch * 0.0
        if n <= 0:
            return 0
        self._deliver(n, times)
        return int(n)

    def _deliver(self, n: int, times):
        slots = self.win.insert_many(np.asarray(times, dtype=np.float64))
        # only the last `cap` rows can survive in the window; copy those
        keep = min(n, self.ring.cap)
        skip = n - keep
        first_slot = int(slots[skip])
        pos = self.next_local + skip
        remaining = keep
        while remaining > 0:  # split at epoch boundaries of the shard
            cur = pos % self.local_total
            run = min(remaining, self.local_total - cur)
            self.ring.ingest_from(self.ds, self.k + cur * self.N, self.N, run, first_slot)
            first_slot = (first_slot + run) % self.ring.cap
            pos += run
            remaining -= run
        self.next_local += n
