"""Lightweight phase tracer writing Chrome trace-event JSON (``--trace``).

Replaces the reference's only telemetry, Confluent monitoring interceptors
feeding Control Center (BaseKafkaApp.java:73-78), with per-phase host spans
(ingest / solve / server / comm).  Disabled tracers cost one branch per span.
"""
from __future__ import annotations

import json
import os
import threading
import time
from contextlib import contextmanager


class Tracer:
    def __init__(self, path: str | None, pid: int = 0):
        self.path = path
        self.pid = pid
        self.events = []
        self._lock = threading.Lock()

    @property
    def enabled(self) -> bool:
        return self.path is not None

    @contextmanager
    def span(self, name: str, **args):
        if self.path is None:
            yield
            return
        t0 = time.perf_counter_ns()
        try:
            yield
        finally:
            t1 = time.perf_counter_ns()
            ev = {"name": name, "ph": "X", "ts": t0 / 1000.0, "dur": (t1 - t0) / 1000.0, "pid": self.pid,
                  "tid": threading.get_ident() % 100000}
            if args:
                ev["args"] = args
            with self._lock:
                self.events.append(ev)

    def instant(self, name: str, **args):
        if self.path is None:
            return
        with self._lock:
            self.events.append({"name": name, "ph": "i", "ts": time.perf_counter_ns() / 1000.0, "pid": self.pid,
                                "tid": threading.get_ident() % 100000, "s": "t", "args": args})

    def close(self):
        if self.path is None:
            return
        d = os.path.dirname(self.path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(self.path, "w") as f:
            json.dump({"traceEvents": self.events}, f)
