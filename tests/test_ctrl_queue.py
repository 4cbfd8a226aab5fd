"""Shared-memory MPSC control queue (the GRADIENTS_TOPIC replacement for SSP/ASP tokens)."""
import multiprocessing as mp
import os

import pytest

from psx._native import host


def _producer(name, k, n):
    from psx._native import host as h

    q = h.CtrlQueue(name, 64, False)
    t = h.CtrlToken()
    t.worker = k
    for v in range(n):
        t.vc = v
        assert q.push(t, 30.0)


def test_single_process_fifo():
    name = f"/psx_test_{os.getpid()}_a"
    q = host.CtrlQueue(name, 8, True)
    try:
        assert q.try_pop() is None
        for v in range(8):
            t = host.CtrlToken()
            t.worker, t.vc = 1, v
            assert q.try_push(t)
        full = host.CtrlToken()
        assert not q.try_push(full)  # bounded
        assert [q.try_pop().vc for _ in range(8)] == list(range(8))
        assert q.pop(0.01) is None  # timeout
    finally:
        q.unlink()


def test_multi_producer_per_worker_order():
    name = f"/psx_test_{os.getpid()}_b"
    q = host.CtrlQueue(name, 64, True)
    try:
        ctx = mp.get_context("spawn")
        ps = [ctx.Process(target=_producer, args=(name, k, 300)) for k in range(3)]
        for p in ps:
            p.start()
        seen = {0: [], 1: [], 2: []}
        for _ in range(900):
            t = q.pop(60.0)
            assert t is not None
            seen[t.worker].append(t.vc)
        for p in ps:
            p.join(30)
            assert p.exitcode == 0
        for k in seen:  # per-worker order preserved (Kafka per-partition ordering)
            assert seen[k] == list(range(300))
    finally:
        q.unlink()


def test_capacity_must_be_power_of_two():
    with pytest.raises(Exception):
        host.CtrlQueue(f"/psx_test_{os.getpid()}_c", 10, True)
