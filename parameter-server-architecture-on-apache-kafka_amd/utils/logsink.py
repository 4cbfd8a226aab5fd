"""Asynchronous evaluation-record sink.

Each record reserves a slot of a pinned (GPU) or plain (CPU) host ring; the
evaluation kernel writes the 16x16 confusion counts and the worker's loss into
that slot itself and publishes the record's sequence number (see
``test_eval_kernel``); the native :class:`MetricsSink` thread waits for the
number, computes Spark's weighted F1 / accuracy (Metrics.java:15-24) and writes
the row through the native :class:`CsvLogger` in the reference's schema
(ServerAppRunner.java:78-82, WorkerAppRunner.java:77-81).  Logging therefore
costs the training loop one slot reservation + one submit per record: no
device->host copies, events, fills or Python-side metric math.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from .. import _native


def now_ms() -> int:
    return int(time.time() * 1000)


class RecordBook:
    """In-memory copy of every logged row (tests, benchmarks, plots).  Row
    timestamps are epoch milliseconds as floats: rows submitted without one are
    stamped (us resolution) when their evaluation completed."""

    def __init__(self, worker=None, server=None):
        self.worker = worker if worker is not None else []  # (ts, partition, vc, loss, f1, acc, nseen)
        self.server = server if server is not None else []  # (ts, vc, f1, acc)


class _HostSlots:
    """nslots EvalSlot records in host memory the device can write."""

    def __init__(self, nslots: int, gpu: bool):
        self.bytes = nslots * _native.host.EVAL_SLOT_BYTES
        self.gpu = gpu
        if gpu:
            self.ptr = _native.hip().pinned_alloc(self.bytes)
            self._buf = None
        else:
            self._buf = np.zeros(self.bytes, dtype=np.uint8)
            self.ptr = self._buf.ctypes.data

    def free(self):
        if self.gpu and self.ptr:
            _native.hip().pinned_free(self.ptr)
            self.ptr = 0


class LogSink:
    def __init__(self, K: int, device, worker_path: str | None = None, server_path: str | None = None,
                 to_stdout: bool = False, pool: int = 256, keep_records: bool = True, worker_append: bool = False):
        self.K = K
        self.device = torch.device(device)
        for path in (worker_path, server_path):
            if path and os.path.dirname(path):
                os.makedirs(os.path.dirname(path), exist_ok=True)
        self.gpu = self.device.type == "cuda"
        self.wlog = _native.host.CsvLogger(worker_path, True, not worker_append, worker_append) if worker_path else (
            _native.host.CsvLogger("", True, False) if to_stdout else None)
        self.slog = _native.host.CsvLogger(server_path, False, True) if server_path else (
            _native.host.CsvLogger("", False, False) if to_stdout else None)
        self.keep = keep_records
        self.slots = _HostSlots(pool, self.gpu)
        self.native = _native.host.MetricsSink(self.slots.ptr, pool, K, self.wlog, self.slog, keep_records)
        self._closed = False

    # -- producers --------------------------------------------------------
    def worker_eval(self, evalset, frag, w, scratch, loss_dev, partition: int, vc: int, nseen: int,
                    ts: int | None = None):
        """Evaluate the worker's local model ``w`` and log a worker row."""
        slot, seq, addr = self.native.acquire()
        evalset.eval_to_slot(frag, w, scratch, addr, seq, loss_dev)
        self.native.submit(slot, seq, 0, self._ts(ts), int(partition), int(vc), int(nseen))

    def server_eval(self, evalset, frag, w, scratch, vc: int, ts: int | None = None):
        """Evaluate the global model ``w`` and log a server row."""
        slot, seq, addr = self.native.acquire()
        evalset.eval_to_slot(frag, w, scratch, addr, seq, None)
        self.native.submit(slot, seq, 1, self._ts(ts), -1, int(vc), 0)

    def pair_eval(self, evalset, frag_w, w_w, loss_dev, partition: int, vc_w: int, nseen: int, frag_s, w_s,
                  vc_s: int | None, ts_s: int, scratch, ts_w: int | None = None, apply=None):
        """Worker row (local model) + server row (global model; vc_s None: none)
        from one evaluation pass, optionally fused with the server update (``apply``)."""
        slot_w, seq_w, addr_w = self.native.acquire()
        slot_s = seq_s = addr_s = 0
        if vc_s is not None:
            slot_s, seq_s, addr_s = self.native.acquire()
        evalset.eval_pair_to_slots(frag_w, w_w, frag_s, w_s, scratch, addr_w, seq_w, loss_dev, addr_s, seq_s, apply)
        if vc_s is not None:
            self.native.submit(slot_s, seq_s, 1, self._ts(ts_s), -1, int(vc_s), 0)
        self.native.submit(slot_w, seq_w, 0, self._ts(ts_w), int(partition), int(vc_w), int(nseen))

    def _ts(self, ts) -> int:
        """Row timestamp: the given one, else -1 on a GPU (the sink stamps the row when
        the device's evaluation lands in its slot) or now on the CPU, where the
        evaluation has completed before the submit (a sink thread starved on a busy
        host would otherwise stamp it late and misorder the ranks' rows)."""
        if ts is not None and int(ts) >= 0:
            return int(ts)
        return -1 if self.gpu else int(time.time() * 1000.0)

    # -- consumers ---------------------------------------------------------
    def drain(self, block: bool = False):
        """Rows are finalised by the native thread; ``block`` waits for all of them."""
        if block:
            self.native.flush()

    @property
    def book(self) -> RecordBook | None:
        if not self.keep:
            return None
        self.native.flush()
        return RecordBook(self.native.worker_rows(), self.native.server_rows())

    def close(self):
        if self._closed:
            return
        self.native.flush()
        self.native.close()
        for lg in (self.wlog, self.slog):
            if lg is not None:
                lg.close()
        self.slots.free()
        self._closed = True


def summarize(book: RecordBook) -> dict:
    """Headline numbers from a run's records (updates/s, best/final server metrics)."""
    out = {}
    if book.worker:
        ts = np.array([r[0] for r in book.worker], dtype=np.float64)
        span = (ts.max() - ts.min()) / 1000.0
        out["worker_rows"] = len(book.worker)
        out["updates_per_s_logged"] = len(book.worker) / span if span > 0 else float("nan")
    if book.server:
        f1 = [r[2] for r in book.server]
        acc = [r[3] for r in book.server]
        out["server_rows"] = len(book.server)
        out["best_server_f1"] = max(f1)
        out["best_server_acc"] = max(acc)
        out["final_server_f1"] = f1[-1]
        out["final_server_acc"] = acc[-1]
    return out
