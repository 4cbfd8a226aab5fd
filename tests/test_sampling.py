"""Sliding-window buffer semantics (WorkerSamplingProcessor.java:50-135)."""
import math

import numpy as np
import pytest

from psx._native import host


def java_target(deltas, bc, lo, hi):
    mean = sum(deltas) / len(deltas) if deltas else 1000.0
    per_min = 60000.0 / mean if mean > 0 else math.inf
    v = math.floor(bc * per_min + 0.5) if math.isfinite(per_min) else hi
    return max(lo, min(hi, v))


def test_rate_estimator_window_of_500():
    r = host.RateEstimator(500)
    assert r.mean_interarrival_ms() == 1000.0  # default with no samples
    t = 0.0
    for i in range(700):
        t += 10.0 if i < 600 else 20.0
        r.arrival(t)
    assert r.samples == 500
    assert r.mean_interarrival_ms() == pytest.approx((400 * 10 + 100 * 20 - 0) / 500, rel=1e-9)


def test_target_formula():
    w = host.SlidingWindow(128, 1024, 0.3)
    assert w.target_size() == java_target([], 0.3, 128, 1024)  # 0.3*60 = 18 -> clamp 128
    times = np.cumsum(np.full(50, 5.0))  # 5 ms apart = 12000 events/min -> 3600 -> 1024
    w.insert_many(times)
    assert w.target_size() == 1024
    w2 = host.SlidingWindow(1, 100000, 0.3)
    w2.insert_many(np.cumsum(np.full(20, 40.0)))  # 1500/min -> 450
    assert w2.target_size() == 450


def reference_buffer(events, bc, lo, hi):
    """Literal re-implementation of the reference's three cases over insertion ids."""
    store = {}  # slot -> insertion id
    deltas, last = [], None
    for t in events:
        if last is not None:
            deltas.append(t - last)
            deltas = deltas[-500:]
        last = t
        target = java_target(deltas, bc, lo, hi)
        largest = max(store.values(), default=0)
        size = len(store)
        if size < target:
            slot = min(set(range(hi)) - set(store))
        elif size == target:
            slot = min(store, key=store.get)
        else:
            order = sorted(store, key=store.get)
            for s in order[: size - target]:
                del store[s]
            slot = order[size - target]
        store[slot] = largest + 1
    return sorted(store.values())


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_window_holds_most_recent_tuples(seed):
    rng = np.random.default_rng(seed)
    lo, hi, bc = 4, 40, 0.3
    # alternate slow and fast phases so the target grows and shrinks
    gaps = np.concatenate([rng.uniform(200, 400, 60), rng.uniform(5, 20, 80), rng.uniform(300, 900, 60)])
    events = np.cumsum(gaps)
    w = host.SlidingWindow(lo, hi, bc)
    ids_ring = [None] * hi
    for i, t in enumerate(events):
        a = w.insert(float(t))
        ids_ring[a.slot] = a.insertion_id
        window_ids = sorted(ids_ring[(w.start + j) % hi] for j in range(w.size))
        assert window_ids == list(range(a.insertion_id - w.size + 1, a.insertion_id + 1))
    assert window_ids == reference_buffer(list(events), bc, lo, hi)


def test_insert_many_consecutive_slots_and_wrap():
    w = host.SlidingWindow(1, 8, 100.0)
    slots = w.insert_many(np.arange(20, dtype=np.float64))
    assert list(slots) == [i % 8 for i in range(20)]
    assert w.tuples_seen == 20
    assert w.head == 19 % 8


def test_bad_arguments():
    with pytest.raises(Exception):
        host.SlidingWindow(10, 5, 0.3)
    with pytest.raises(Exception):
        host.SlidingWindow(1, 5, 0.0)


def test_window_ring_capacity_rounding():
    # the device ring rounds `max` up to whole 32-row tiles; the window size is
    # still bounded by `max` while slots wrap at the ring capacity
    w = host.SlidingWindow(10, 100, 100.0, 500, 128)
    assert w.capacity == 128 and w.max_size == 100
    for i in range(130):
        w.insert(float(i))  # 1 ms apart: target clamps to max
    assert w.size == 100
    assert w.head == 129 % 128
    assert w.start == (w.head - w.size + 1) % 128


def test_zero_mean_interarrival_policy():
    """A burst (every arrival at the same millisecond: mean inter-arrival 0) gives
    the MAX window here.  Documented deviation: Java's (int) Math.round(Infinity)
    = (int) Long.MAX_VALUE = -1, so the reference clamps such a burst to the MIN
    window (WorkerSamplingProcessor.java:115-122); an overflow artefact, not a
    policy (csrc/host/sampling.cc)."""
    w = host.SlidingWindow(128, 1024, 0.3)
    for _ in range(10):
        w.insert(5.0)  # identical timestamps
    assert w.target_size() == 1024
    java_int_cast = ((2 ** 63 - 1) + 2 ** 31) % 2 ** 32 - 2 ** 31  # (int) Long.MAX_VALUE
    assert java_int_cast == -1 and max(128, min(1024, java_int_cast)) == 128


@pytest.mark.parametrize("rate_window", [500, 1, 3, 64, 2000])
def test_bulk_insert_equals_row_by_row(rate_window):
    """The round loops' bulk insert (equal-stamp runs at the max target in one step;
    the estimator's zero deltas in closed form) leaves the window and the rate
    estimator exactly as row-by-row inserts do -- also for estimator windows shorter
    and longer than a delivery."""
    import numpy as np

    rng = np.random.default_rng(7)
    for trial in range(20):
        a = host.SlidingWindow(128, 1024, 0.3, rate_window, 1024)
        b = host.SlidingWindow(128, 1024, 0.3, rate_window, 1024)
        now = 0.0
        for _ in range(60):
            k = int(rng.integers(1, 1500))
            mode = rng.integers(0, 3)
            if mode == 0:  # a burst (one poll of per-round deliveries)
                t = np.full(k, now)
            elif mode == 1:  # producer clock: distinct stamps
                t = now + np.cumsum(rng.exponential(rng.choice([0.01, 5.0, 400.0]), k))
            else:  # mixed: runs of equal stamps
                t = np.repeat(now + np.cumsum(rng.exponential(2.0, k // 8 + 1)), 8)[:k]
            now = float(t[-1]) + float(rng.choice([0.0, 0.5, 50.0]))
            a.insert_many(t)
            first = b.insert_bulk(t)
            assert first == (b.head - k + 1) % b.capacity or k > b.capacity
            assert (a.size, a.head, a.tuples_seen, a.start) == (b.size, b.head, b.tuples_seen, b.start), trial
            assert a.mean_interarrival_ms() == b.mean_interarrival_ms(), trial
            assert a.target_size() == b.target_size()
