"""Failure detection and fault injection.

The reference has no failure handling of its own: Kafka rebalances consumer
groups, a restarted server re-zeroes its weights, and a stale vector clock
trips MessageTracker's IllegalArgumentException (MessageTracker.java:23-32).
Here:

* ``--inject_worker_delay K:MS`` makes worker K a straggler (the README's
  motivation for bounded delay / eventual consistency, README.md:180,190);
* ``--inject_worker_crash K:ITER`` makes worker K fail at its ITER-th
  iteration (raises :class:`WorkerFailure` inside the worker);
* a watchdog on the server marks a *busy* worker (weights sent, no delta back)
  silent for ``--worker_timeout`` seconds as failed;
* policy (``--on_worker_failure``): ``drop`` retires the worker from the
  vector-clock tracker (the others are no longer held back by its clock) and
  training continues with N-1 workers; ``fail`` aborts the run loudly;
  ``auto`` = drop under eventual consistency (nobody waits for anybody), fail
  under sequential / bounded delay, where a silently shrinking N would change
  the consistency guarantee.
"""
from __future__ import annotations


class WorkerFailure(RuntimeError):
    """A worker stopped participating (injected crash, exception or watchdog timeout)."""

    def __init__(self, worker: int, reason: str):
        super().__init__(f"worker {worker} failed: {reason}")
        self.worker = int(worker)
        self.reason = reason


def parse_worker_map(items) -> dict:
    """["K:V", ...] -> {K: float(V)} (CLI flags --inject_worker_delay / --inject_worker_crash)."""
    out = {}
    for it in items or []:
        k, v = str(it).split(":")
        out[int(k)] = float(v)
    return out


def drop_on_failure(cfg) -> bool:
    pol = getattr(cfg, "on_worker_failure", "auto")
    if pol == "drop":
        return True
    if pol == "fail":
        return False
    return cfg.consistency_model == -1
