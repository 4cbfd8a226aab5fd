"""Phase tracing (``--trace``) and the per-round performance log (``--perf_log``).

Replaces the reference's only telemetry, Confluent monitoring interceptors
feeding Control Center (BaseKafkaApp.java:73-78), with:

* host spans per phase (ingest / solve / server / comm / recv) as Chrome
  trace events (load the JSON in chrome://tracing or Perfetto);
* device spans of the same phases from HIP events recorded on the stream the
  phase enqueued its work on -- the GPU time of each phase, placed on the
  host timeline through a reference event -- on a "device" track;
* ``logs-perf.csv``: one row per round with the device time of
  every phase, the host time of the round and the running updates/s.  It is a
  separate file so that logs-server.csv / logs-worker.csv keep the
  reference's exact schema.

Device events are resolved lazily (at close, or once the queue is long), so
tracing never synchronises the training loop.  Disabled tracers cost one
branch per span.
"""
from __future__ import annotations

import json
import os
import threading
import time
from contextlib import contextmanager

import torch


class Tracer:
    def __init__(self, path: str | None, pid: int = 0, device=None, perf_path: str | None = None):
        self.path = path
        self.perf_path = perf_path
        self.pid = pid
        self.events = []
        self._lock = threading.Lock()
        self.device = torch.device(device) if device is not None else None
        self._gpu = self.device is not None and self.device.type == "cuda" and (path or perf_path)
        self._dev_spans = []  # (name, start_event, end_event, round)
        self._ref = None
        self._ref_host_us = 0.0
        self._round = 0
        self._round_t0 = None
        self._rows = []  # (round, host_ts_ms, host_round_us, {phase: [events]})
        self._cur = {}
        self._updates = 0
        self._t_start = None
        self._perf_fh = None
        if self._gpu:
            self._ref = torch.cuda.Event(enable_timing=True)
            self._ref.record(torch.cuda.current_stream(self.device))
            self._ref_host_us = time.perf_counter_ns() / 1000.0

    @property
    def enabled(self) -> bool:
        return self.path is not None or self.perf_path is not None

    @contextmanager
    def span(self, name: str, **args):
        if not self.enabled:
            yield
            return
        ev0 = None
        if self._gpu:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record(torch.cuda.current_stream(self.device))
        t0 = time.perf_counter_ns()
        try:
            yield
        finally:
            t1 = time.perf_counter_ns()
            if self.path is not None:
                ev = {"name": name, "ph": "X", "ts": t0 / 1000.0, "dur": (t1 - t0) / 1000.0, "pid": self.pid,
                      "tid": threading.get_ident() % 100000}
                if args:
                    ev["args"] = args
                with self._lock:
                    self.events.append(ev)
            if ev0 is not None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record(torch.cuda.current_stream(self.device))
                with self._lock:
                    self._dev_spans.append((name, ev0, ev1))
                    self._cur.setdefault(name, []).append((ev0, ev1))

    def instant(self, name: str, **args):
        if self.path is None:
            return
        with self._lock:
            self.events.append({"name": name, "ph": "i", "ts": time.perf_counter_ns() / 1000.0, "pid": self.pid,
                                "tid": threading.get_ident() % 100000, "s": "t", "args": args})

    # ---- per-round performance log -----------------------------------------
    def round_begin(self):
        if self.perf_path is None:
            return
        now = time.perf_counter()
        if self._t_start is None:
            self._t_start = now
        self._round_t0 = now
        self._cur = {}

    def round_end(self, rnd: int, updates: int):
        """Close round ``rnd``; ``updates`` = server updates applied so far in this run."""
        if self.perf_path is None or self._round_t0 is None:
            return
        now = time.perf_counter()
        self._rows.append((int(rnd), int(time.time() * 1000), (now - self._round_t0) * 1e6, self._cur,
                           updates / max(now - self._t_start, 1e-9)))
        self._cur = {}
        if len(self._rows) >= 4096:
            self._flush_perf()

    def _flush_perf(self):
        if not self._rows:
            return
        if self._perf_fh is None:
            d = os.path.dirname(self.perf_path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._perf_fh = open(self.perf_path, "w")
            self._perf_fh.write("round;timestamp;host_round_us;ingest_us;solve_us;comm_us;server_us;updates_per_s\n")
        if self._gpu:
            torch.cuda.synchronize(self.device)
        for rnd, ts, host_us, phases, ups in self._rows:
            dev = {}
            for name, evs in phases.items():
                if isinstance(evs, float):  # (lane_rows: device time already in us)
                    dev[name] = evs
                else:
                    dev[name] = sum(a.elapsed_time(b) * 1000.0 for a, b in evs) if self._gpu else float("nan")
            cols = [dev.get(p, 0.0) for p in ("ingest", "solve", "comm", "server")]
            self._perf_fh.write(f"{rnd};{ts};{host_us:.1f};" + ";".join(f"{c:.1f}" for c in cols) + f";{ups:.2f}\n")
        self._rows.clear()

    # ---- the native lanes loops: device phase times recorded by the kernels ----------
    def lane_rows(self, rows, ref, ups: float = 0.0):
        """Phase times the lanes kernels recorded on the device (LanesLoop.trace_take,
        s_memrealtime ticks of 10 ns) -> "device" trace events and logs-perf.csv rows.
        ``ref`` = LanesLoop.clock_ref: (host CLOCK_MONOTONIC ns before, device ticks, ns
        after) -- time.perf_counter_ns's clock on Linux -- places them on the host
        timeline.  BSP rows {0, round, lane, worker, stage, solve, solved, updated}: one
        perf row per round (ingest = staging + window statistics, solve, server = the
        update, the slowest lane of each); asynchronous rows {1, ticket, lane, worker,
        released, solved, pushed}: one perf row per update."""
        if not self.enabled or not rows:
            return
        off_us = (ref[0] + ref[2]) / 2000.0 - ref[1] / 100.0

        def us(t):
            return off_us + t / 100.0

        rounds = {}
        for r in rows:
            kind, n, lane, k = int(r[0]), int(r[1]), int(r[2]), int(r[3])
            t = [int(x) for x in r[4:8]]
            if kind == 0:
                if min(t) <= 0:
                    continue
                spans = (("ingest", t[0], t[1]), ("solve", t[1], t[2]), ("server", t[2], t[3]))
            else:
                if min(t[:3]) <= 0:
                    continue
                spans = (("solve", t[0], t[1]), ("push", t[1], t[2]))
            if self.path is not None:
                with self._lock:
                    for name, a, b in spans:
                        self.events.append({"name": name, "ph": "X", "ts": us(a), "dur": (b - a) / 100.0,
                                            "pid": self.pid, "tid": "device", "cat": "gpu",
                                            "args": {"round" if kind == 0 else "ticket": n, "lane": lane,
                                                     "worker": k}})
            if self.perf_path is not None:
                ph = rounds.setdefault((kind, n), {"_t0": spans[0][1], "_t1": spans[-1][2]})
                ph["_t0"] = min(ph["_t0"], spans[0][1])
                ph["_t1"] = max(ph["_t1"], spans[-1][2])
                for name, a, b in spans:
                    key = "server" if name == "push" else name
                    ph[key] = max(ph.get(key, 0.0), (b - a) / 100.0)
        for (kind, n), ph in sorted(rounds.items()):
            span_us = (ph.pop("_t1") - ph.pop("_t0")) / 100.0
            self._rows.append((n, int(time.time() * 1000), span_us, ph, ups))
        if len(self._rows) >= 4096:
            self._flush_perf()

    # ------------------------------------------------------------------
    def close(self):
        if self.perf_path is not None:
            self._flush_perf()
            if self._perf_fh is not None:
                self._perf_fh.close()
                self._perf_fh = None
        if self.path is None:
            return
        if self._gpu and self._dev_spans:
            torch.cuda.synchronize(self.device)
            for name, a, b in self._dev_spans:
                ts = self._ref_host_us + self._ref.elapsed_time(a) * 1000.0
                self.events.append({"name": name, "ph": "X", "ts": ts, "dur": a.elapsed_time(b) * 1000.0,
                                    "pid": self.pid, "tid": "device", "cat": "gpu"})
            self._dev_spans.clear()
        d = os.path.dirname(self.path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(self.path, "w") as f:
            json.dump({"traceEvents": self.events}, f)
