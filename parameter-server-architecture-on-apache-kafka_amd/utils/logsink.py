"""Asynchronous CSV log sink.

Device results (loss, 16x16 confusion counts) are copied into pinned host slots
with non-blocking copies and an event; rows are finalised (weighted F1 /
accuracy) and handed to the native :class:`CsvLogger` once their event has
completed, so logging never stalls the training stream.  Row format is the
reference's (ServerAppRunner.java:78-82, WorkerAppRunner.java:77-81).
"""
from __future__ import annotations

import collections
import time

import numpy as np
import torch

from .. import _native
from .metrics import metrics_from_confusion


def now_ms() -> int:
    return int(time.time() * 1000)


class RecordBook:
    """In-memory copy of every logged row (tests, benchmarks, plots)."""

    def __init__(self):
        self.worker = []  # (ts, partition, vc, loss, f1, acc, nseen)
        self.server = []  # (ts, vc, f1, acc)


class LogSink:
    def __init__(self, K: int, device, worker_path: str | None = None, server_path: str | None = None,
                 to_stdout: bool = False, pool: int = 64, keep_records: bool = True, worker_append: bool = False):
        self.K = K
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.wlog = _native.host.CsvLogger(worker_path, True, not worker_append, worker_append) if worker_path else (
            _native.host.CsvLogger("", True, False) if to_stdout else None)
        self.slog = _native.host.CsvLogger(server_path, False, True) if server_path else (
            _native.host.CsvLogger("", False, False) if to_stdout else None)
        self.book = RecordBook() if keep_records else None
        self.pending = collections.deque()
        self.pool = pool
        self._free = []
        for _ in range(pool):
            conf = torch.zeros(256, dtype=torch.int32, pin_memory=self.gpu)
            loss = torch.zeros(1, dtype=torch.float32, pin_memory=self.gpu)
            self._free.append((conf, loss))

    def _slot(self):
        while not self._free:
            self.drain(block_one=True)
        return self._free.pop()

    def submit_worker(self, partition: int, vc: int, nseen: int, loss_dev: torch.Tensor, conf_dev: torch.Tensor,
                      ts: int | None = None):
        conf, loss = self._slot()
        conf.copy_(conf_dev.view(-1), non_blocking=True)
        loss.copy_(loss_dev.view(-1)[:1], non_blocking=True)
        ev = self._event()
        self.pending.append(("w", ts or now_ms(), partition, vc, nseen, conf, loss, ev))

    def submit_server(self, vc: int, conf_dev: torch.Tensor, ts: int | None = None):
        conf, loss = self._slot()
        conf.copy_(conf_dev.view(-1), non_blocking=True)
        ev = self._event()
        self.pending.append(("s", ts or now_ms(), -1, vc, 0, conf, loss, ev))

    def _event(self):
        if not self.gpu:
            return None
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def drain(self, block: bool = False, block_one: bool = False):
        while self.pending:
            kind, ts, part, vc, nseen, conf, loss, ev = self.pending[0]
            if ev is not None and not ev.query():
                if block or block_one:
                    ev.synchronize()
                else:
                    return
            self.pending.popleft()
            c = conf.numpy().reshape(16, 16)[: self.K, : self.K]
            f1, acc = metrics_from_confusion(c)
            if kind == "w":
                lv = float(loss.item())
                if self.wlog is not None:
                    self.wlog.log_worker(ts, part, vc, lv, f1, acc, nseen)
                if self.book is not None:
                    self.book.worker.append((ts, part, vc, lv, f1, acc, nseen))
            else:
                if self.slog is not None:
                    self.slog.log_server(ts, vc, f1, acc)
                if self.book is not None:
                    self.book.server.append((ts, vc, f1, acc))
            self._free.append((conf, loss))
            if block_one:
                return

    def close(self):
        self.drain(block=True)
        for lg in (self.wlog, self.slog):
            if lg is not None:
                lg.close()


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
