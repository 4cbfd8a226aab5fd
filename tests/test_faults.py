"""Failure detection / fault injection: injected worker crashes,
tracker retirement, drop-vs-fail policy, and the multi-process error path."""
import pytest

from psx.runtime.config import PSConfig
from psx.runtime.engine import LocalEngine
from psx.runtime.faults import WorkerFailure, drop_on_failure, parse_worker_map
from psx.utils.data import synth_finefood


def _cfg(c, N=3, **kw):
    base = dict(num_workers=N, consistency_model=c, producer_time_per_event=0, stream_mode="per_iter",
                rows_per_iter=32, epochs=100, max_iters=8, min_buffer_size=32, max_buffer_size=128)
    base.update(kw)
    return PSConfig(**base)


def _data():
    return synth_finefood(1500, num_features=128, seed=0), synth_finefood(200, num_features=128, seed=1)


def test_parse_and_policy():
    assert parse_worker_map(["1:3", "2:10.5"]) == {1: 3.0, 2: 10.5}
    assert drop_on_failure(_cfg(-1)) and not drop_on_failure(_cfg(0)) and not drop_on_failure(_cfg(2))
    assert drop_on_failure(_cfg(0, on_worker_failure="drop"))
    assert not drop_on_failure(_cfg(-1, on_worker_failure="fail"))


def test_tracker_retire_releases_waiters():
    from psx import _native

    t = _native.host.VectorClockTracker(3, 0)  # BSP
    assert t.on_delta(0, 0) == [] and t.on_delta(1, 0) == []
    # worker 2 dies before pushing vc 0: the round completes without it
    assert sorted(t.retire(2)) == [(0, 1), (1, 1)]
    assert t.num_live == 2 and not t.is_live(2) and t.min_clock() == 1
    with pytest.raises(Exception):
        t.received(2, 0)
    s = _native.host.VectorClockTracker(2, 1)  # SSP(1): worker 1 is the straggler
    for v in range(2):
        s.on_delta(0, v)
    assert s.releasable(0, 1) == []  # worker 0 is 2 ahead of worker 1's clock 0
    assert s.retire(1) == [(0, 2)]


def test_asp_inprocess_crash_is_dropped():
    tr, te = _data()
    eng = LocalEngine(_cfg(-1, inject_worker_crash={1: 3}), "cpu", train=tr, test=te)
    out = eng.run()
    assert out["failed_workers"] == [1]
    assert eng.workers[1].iters == 3 and eng.workers[0].iters >= 8 and eng.workers[2].iters >= 8
    assert out["server_rows"] >= 8


def test_asp_inprocess_worker0_crash_moves_server_rows():
    tr, te = _data()
    # workers 1, 2 are slowed so that worker 0's crash lands early even on a loaded host
    eng = LocalEngine(_cfg(-1, inject_worker_crash={0: 2}, inject_worker_delay_ms={1: 20.0, 2: 20.0}), "cpu",
                      train=tr, test=te)
    out = eng.run()
    assert out["failed_workers"] == [0] and out["server_rows"] >= 5  # 2 from worker 0, then worker 1's


def test_bsp_crash_fails_loudly():
    tr, te = _data()
    eng = LocalEngine(_cfg(0, inject_worker_crash={2: 4}), "cpu", train=tr, test=te)
    with pytest.raises(WorkerFailure):
        eng.run()


@pytest.mark.parametrize("c", [0, 2])
def test_crash_with_drop_policy_continues(c):
    tr, te = _data()
    eng = LocalEngine(_cfg(c, inject_worker_crash={2: 4}, on_worker_failure="drop"), "cpu", train=tr, test=te)
    out = eng.run()
    assert out["failed_workers"] == [2] and eng.workers[2].iters == 4
    assert min(eng.workers[0].iters, eng.workers[1].iters) >= 8


def test_dist_async_worker_crash_is_dropped():
    from test_dist_cpu import BASE, _run

    out, w = _run(3, dict(BASE, consistency_model=-1, max_iters=6, inject_worker_crash={1: 2}))
    assert out["failed_workers"] == [1]
    assert out["updates"] == 6 + 2  # worker 0: all 6, worker 1: 2 before its crash
