"""VectorClockTracker: Appendix-A semantics of MessageTracker/ServerProcessor.workersToRespondTo."""
import random

import pytest

from psx._native import host


def test_init_state():
    t = host.VectorClockTracker(3, 0)
    assert t.clocks() == [0, 0, 0]
    assert all(t.is_sent(k) for k in range(3))  # MessageTracker.java:51 -> (0, true)


def test_sequential_releases_whole_round_at_once():
    t = host.VectorClockTracker(4, 0)
    assert t.on_delta(2, 0) == []
    assert t.on_delta(0, 0) == []
    assert t.on_delta(3, 0) == []
    assert t.on_delta(1, 0) == [(0, 1), (1, 1), (2, 1), (3, 1)]
    assert t.on_delta(1, 1) == []


def test_eventual_answers_sender_only():
    t = host.VectorClockTracker(3, -1)
    assert t.on_delta(1, 0) == [(1, 1)]
    assert t.on_delta(1, 1) == [(1, 2)]
    assert t.on_delta(0, 0) == [(0, 1)]
    assert t.max_gap == 2


def test_bounded_delay_blocks_fast_worker():
    t = host.VectorClockTracker(2, 1)
    assert t.on_delta(0, 0) == [(0, 1)]  # min vc 0 >= 1 - 1
    assert t.on_delta(0, 1) == []  # vc0 = 2, min 0 < 2 - 1 -> wait
    assert t.on_delta(1, 0) == [(0, 2), (1, 1)]  # slow worker catches up, releases both


def test_protocol_violation_is_hard_error():
    t = host.VectorClockTracker(2, 0)
    with pytest.raises(Exception):
        t.received(0, 5)
    t.received(0, 0)
    with pytest.raises(Exception):
        t.sent(0, 7)


def test_rejects_stalling_consistency_model():
    with pytest.raises(Exception):
        host.VectorClockTracker(2, -2)  # reference quirk Q4: stalls forever


def _simulate(c, speeds, updates=400, seed=0):
    """Event simulation of workers with given speeds (Appendix A reproduction)."""
    rnd = random.Random(seed)
    n = len(speeds)
    t = host.VectorClockTracker(n, c)
    now = 0.0
    busy = {k: (speeds[k] * (1 + 0.1 * rnd.random()), 0) for k in range(n)}  # k -> (finish time, vc)
    done = 0
    while done < updates and busy:
        k = min(busy, key=lambda j: busy[j][0])
        now, v = busy.pop(k)
        rel = t.on_delta(k, v)
        done += 1
        for j, u in rel:
            busy[j] = (now + speeds[j] * (1 + 0.1 * rnd.random()), u)
    return t


@pytest.mark.parametrize("c,expect", [(0, 1), (1, 1), (3, 3), (10, 10)])
def test_staleness_bound_matches_appendix_a(c, expect):
    t = _simulate(c, [1.0, 1.0, 1.3, 3.0])
    # max(vc) - min(vc) of RECEIVED clocks: BSP shows 1 (one round in flight, as in
    # sequential_logs-worker.csv); SSP(c) releases versions at most c ahead of the
    # slowest, so received clocks differ by at most c + 1 (logs: 11 for c = 10)
    if c == 0:
        assert t.max_gap == 1
    else:
        assert expect <= t.max_gap <= expect + 1


def test_eventual_is_unbounded():
    t = _simulate(-1, [1.0, 1.0, 1.3, 3.0])
    assert t.max_gap > 50


def test_restore_roundtrip():
    t = host.VectorClockTracker(3, 2)
    t.on_delta(0, 0)
    t.on_delta(1, 0)
    t2 = host.VectorClockTracker(3, 2)
    t2.restore(t.clocks(), t.sent_flags())
    assert t2.clocks() == t.clocks() and t2.sent_flags() == t.sent_flags()
