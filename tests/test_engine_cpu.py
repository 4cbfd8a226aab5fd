"""In-process engine on CPU: BASELINE.json config #1 (sequential, 2 workers, mock data)
and the asynchronous consistency models, checked from the logs the way the
reference validated them."""
import os

import pytest
import torch

from psx.runtime.config import PSConfig
from psx.runtime.engine import LocalEngine
from psx.utils.checkpoint import load_server, save_server
from psx.utils.data import synth_binary, synth_finefood

MOCK = "/root/reference/mockData/sample_input_data.csv"


def _mock_paths():
    if os.path.exists(MOCK):
        return MOCK, MOCK
    pytest.skip("reference mock data not mounted")


def test_config1_sequential_two_workers_mock(tmp_path):
    tr, te = _mock_paths()
    cfg = PSConfig(train_path=tr, test_path=te, num_workers=2, consistency_model=0, producer_time_per_event=0,
                   max_iters=8, logging=True, log_dir=str(tmp_path))
    out = LocalEngine(cfg, "cpu").run()
    assert out["rounds"] == 8 and out["updates"] == 16
    wl = (tmp_path / "logs-worker.csv").read_text().splitlines()
    sl = (tmp_path / "logs-server.csv").read_text().splitlines()
    assert wl[0] == "timestamp;partition;vectorClock;loss;fMeasure;accuracy;numTuplesSeen"
    assert sl[0] == "timestamp;partition;vectorClock;loss;fMeasure;accuracy"
    assert len(wl) == 1 + 16 and len(sl) == 1 + 8
    rows = [r.split(";") for r in wl[1:]]
    assert {r[1] for r in rows} == {"0", "1"}
    # each worker logs vector clocks 0..7 in order; numTuplesSeen = its shard (25 rows)
    for k in ("0", "1"):
        vcs = [int(r[2]) for r in rows if r[1] == k]
        assert vcs == list(range(8))
        assert all(int(r[6]) == 25 for r in rows if r[1] == k)
    srows = [r.split(";") for r in sl[1:]]
    assert all(r[1] == "-1" and r[3] == "-1" for r in srows)
    assert float(srows[-1][5]) > 0.7  # mock data is nearly separable


@pytest.mark.parametrize("c", [-1, 1, 3])
def test_async_models_staleness(c):
    train, test = synth_finefood(3000, num_features=128, seed=0), synth_finefood(300, num_features=128, seed=1)
    cfg = PSConfig(num_workers=3, consistency_model=c, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=64, epochs=100, max_iters=12, inject_worker_delay_ms={2: 15.0})
    eng = LocalEngine(cfg, "cpu", train=train, test=test)
    out = eng.run()
    assert out["updates"] >= 36
    if c > 0:
        assert out["max_vc_gap"] <= c + 1
    else:
        assert out["max_vc_gap"] >= 2  # the straggler falls behind under eventual consistency


@pytest.mark.parametrize("c", [-1, 2])
def test_single_worker_async_equals_sequential(c):
    """One worker: every consistency model releases it right after its delta, so an
    asynchronous run gives the sequential run's model and log rows."""
    train, test = synth_finefood(2000, num_features=128, seed=0), synth_finefood(300, num_features=128, seed=1)
    ws, books = [], []
    for cm in (c, 0):
        cfg = PSConfig(num_workers=1, consistency_model=cm, producer_time_per_event=0, stream_mode="per_iter",
                       rows_per_iter=64, epochs=100, max_iters=6, min_buffer_size=128, max_buffer_size=128)
        eng = LocalEngine(cfg, "cpu", train=train, test=test)
        out = eng.run()
        assert out["rounds"] == 6 and out["updates"] == 6 and out["max_vc_gap"] <= 1
        ws.append(eng.server.w.clone())
        books.append(eng.log.book)
    assert torch.allclose(ws[0], ws[1], atol=1e-6)
    assert [r[1:] for r in books[0].server] == [r[1:] for r in books[1].server]
    assert [r[1:3] for r in books[0].worker] == [r[1:3] for r in books[1].worker]


def test_schedule_mode_arrival_burst():
    """-p 200 with N=2: burst of 256 rows, then 5 rows per second in total."""
    train, test = synth_finefood(2000, num_features=128, seed=0), synth_finefood(200, num_features=128, seed=1)
    cfg = PSConfig(num_workers=2, consistency_model=0, producer_time_per_event=200, max_iters=3)
    eng = LocalEngine(cfg, "cpu", train=train, test=test)
    eng.run()
    for w in eng.workers:
        assert 128 <= w.tuples_seen <= 140  # burst share + a few scheduled rows
        assert w.window.size == min(w.tuples_seen, w.window.target_size())


def test_checkpoint_roundtrip_and_resume(tmp_path):
    train, test = synth_binary(200, 32, seed=0), synth_binary(50, 32, seed=1)
    cfg = PSConfig(num_workers=1, consistency_model=0, producer_time_per_event=0, max_iters=4,
                   checkpoint_dir=str(tmp_path), checkpoint_every=2)
    eng = LocalEngine(cfg, "cpu", train=train, test=test)
    eng.run()
    st = load_server(str(tmp_path))
    assert st["updates"] == 4 and torch.equal(st["w"], eng.server.w)
    cfg2 = PSConfig(num_workers=1, consistency_model=0, producer_time_per_event=0, max_iters=1,
                    checkpoint_dir=str(tmp_path), resume=True)
    eng2 = LocalEngine(cfg2, "cpu", train=train, test=test)
    assert torch.equal(eng2.server.w, eng.server.w)
    assert eng2.server.tracker.clocks() == [4]
    save_server(str(tmp_path), eng2.server)


def test_fault_injection_delay_slows_only_that_worker():
    train, test = synth_finefood(2000, num_features=128, seed=0), synth_finefood(100, num_features=128, seed=1)
    cfg = PSConfig(num_workers=2, consistency_model=-1, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=32, epochs=100, max_iters=5, inject_worker_delay_ms={1: 40.0})
    eng = LocalEngine(cfg, "cpu", train=train, test=test)
    eng.run()
    assert eng.workers[0].iters > eng.workers[1].iters


def test_checkpoint_resume_is_exact(tmp_path):
    """6 BSP rounds straight == 3 rounds, checkpoint (server + worker rings/cursors), resume, 3 rounds."""
    train, test = synth_finefood(3000, num_features=128, seed=0), synth_finefood(200, num_features=128, seed=1)

    def cfg(**kw):
        return PSConfig(num_workers=2, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                        rows_per_iter=48, epochs=10, min_buffer_size=100, max_buffer_size=100, init="random",
                        **kw)

    ref = LocalEngine(cfg(max_iters=6), "cpu", train=train, test=test)
    ref.run()
    a = LocalEngine(cfg(max_iters=3, checkpoint_dir=str(tmp_path), checkpoint_every=3), "cpu", train=train,
                    test=test)
    a.run()
    assert (tmp_path / "server.ckpt").exists() and (tmp_path / "worker1.ckpt").exists()
    b = LocalEngine(cfg(max_iters=3, checkpoint_dir=str(tmp_path), resume=True), "cpu", train=train, test=test)
    assert b.rounds == 3 and b.workers[1].source.next_local == a.workers[1].source.next_local
    b.run()
    assert torch.allclose(b.server.w, ref.server.w, atol=1e-6), (b.server.w - ref.server.w).abs().max()
    st = load_server(str(tmp_path))
    assert st["model"] == "dense" and st["w_reference_layout"].numel() == 6 * 128 + 6


def test_checkpoint_wide_model(tmp_path):
    from psx.utils.data import synth_sparse

    tr = synth_sparse(800, num_features=5000, nnz_mean=20, max_nnz=48, seed=0)
    te = synth_sparse(100, num_features=5000, nnz_mean=20, max_nnz=48, seed=1)
    c = PSConfig(num_workers=1, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                 rows_per_iter=64, epochs=5, max_iters=4, min_buffer_size=64, max_buffer_size=128, init="random",
                 checkpoint_dir=str(tmp_path), checkpoint_every=2)
    eng = LocalEngine(c, "cpu", train=tr, test=te)
    eng.run()
    st = load_server(str(tmp_path))
    assert st["model"] == "wide" and torch.equal(st["w"], eng.server.w) and "w_reference_layout" not in st


@pytest.mark.parametrize("c", [-1, 2])
def test_event_scheduler_async(c):
    """The one-thread event-polling scheduler (the GPU default for SSP/ASP) on CPU:
    every worker steps, the staleness bound holds and the run matches the
    tracker's accounting."""
    train, test = synth_finefood(3000, num_features=128, seed=0), synth_finefood(300, num_features=128, seed=1)
    cfg = PSConfig(num_workers=3, consistency_model=c, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=64, epochs=100, max_iters=10, async_scheduler="events")
    eng = LocalEngine(cfg, "cpu", train=train, test=test)
    assert eng._event_scheduler()
    out = eng.run()
    assert out["updates"] >= 30 and min(w.iters for w in eng.workers) >= 10
    assert out["max_vc_gap"] <= (c + 1 if c > 0 else 1)  # completion order is FIFO on the CPU
    assert {r[1] for r in eng.log.book.worker} == {0, 1, 2}
    assert out["server_rows"] >= 10


def test_event_scheduler_crash_is_dropped():
    train, test = synth_finefood(3000, num_features=128, seed=0), synth_finefood(300, num_features=128, seed=1)
    cfg = PSConfig(num_workers=3, consistency_model=-1, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=64, epochs=100, max_iters=8, async_scheduler="events",
                   inject_worker_crash={0: 2})
    eng = LocalEngine(cfg, "cpu", train=train, test=test)
    out = eng.run()
    assert out["failed_workers"] == [0] and eng.workers[0].iters == 2
    assert min(eng.workers[1].iters, eng.workers[2].iters) >= 8
    assert out["server_rows"] >= 8  # worker 0's rows, then the lowest survivor's


def test_async_scheduler_choice():
    cfg = PSConfig(num_workers=2, consistency_model=-1, async_scheduler="bogus")
    train, test = synth_finefood(500, num_features=128, seed=0), synth_finefood(100, num_features=128, seed=1)
    with pytest.raises(ValueError):
        LocalEngine(cfg, "cpu", train=train, test=test)._event_scheduler()
    cfg.async_scheduler = "auto"
    assert not LocalEngine(cfg, "cpu", train=train, test=test)._event_scheduler()  # CPU: threads


def test_cli_async_scheduler_and_rccl_trace(tmp_path):
    from psx.apps.cli import parse_or_exit, server_config, server_parser
    from psx.parallel.dist import rccl_trace_env

    a = parse_or_exit(server_parser(), ["--inprocess", "--async_scheduler", "events", "--rccl_trace",
                                        "--log_dir", str(tmp_path), "-c", "-1"])
    assert server_config(a).async_scheduler == "events" and a.rccl_trace
    env = rccl_trace_env(str(tmp_path))
    assert env["NCCL_DEBUG"] == "INFO" and "COLL" in env["NCCL_DEBUG_SUBSYS"]
    assert env["NCCL_DEBUG_FILE"].startswith(str(tmp_path)) and "%p" in env["NCCL_DEBUG_FILE"]


def test_fresh_window_cadence(tmp_path):
    """--iter_new_frac 0.5: a worker iterates only once half of its window is new
    tuples (evaluation/README.md §3), so consecutive solves are >= 64 tuples apart
    for the 128-row minimum window."""
    train, test = synth_finefood(3000, num_features=128, seed=0), synth_finefood(200, num_features=128, seed=1)
    cfg = PSConfig(num_workers=1, consistency_model=0, producer_time_per_event=2.0, max_wallclock_s=3.5,
                   min_buffer_size=128, max_buffer_size=128, iter_new_frac=0.5, logging=True, log_dir=str(tmp_path))
    LocalEngine(cfg, "cpu", train=train, test=test).run()
    rows = [r.split(";") for r in (tmp_path / "logs-worker.csv").read_text().splitlines()[1:]]
    seen = [int(r[6]) for r in rows]
    assert len(seen) >= 3
    gaps = [b - a for a, b in zip(seen, seen[1:])]
    assert min(gaps[:-1]) >= 64, gaps  # the last solve may run on an exhausted stream


def test_synth_finefood_round1_generator():
    """class_zipf = 0, text_noise = 0 keeps the round-1 generator (uniform class words)."""
    a = synth_finefood(64, num_features=128, seed=3, class_zipf=0.0, text_noise=0.0, signal=0.074)
    b = synth_finefood(64, num_features=128, seed=3)
    assert torch.equal(a.y, b.y)  # the labels come first from the same stream
    assert not torch.equal(a.X, b.X)
    n = a.float_features().norm(dim=1)
    assert torch.allclose(n, torch.ones_like(n), atol=1e-2)


def test_cadence_ramp():
    """--iter_new_ramp R: a worker's first solves wait for at most R, 2R, 4R, ... new
    tuples; afterwards (and without a solve count) the frac / cap rule alone."""
    from psx.runtime.config import PSConfig, new_tuples_needed

    c = PSConfig(iter_new_frac=0.5, iter_new_cap=128, iter_new_ramp=8)
    assert [new_tuples_needed(c, 1024, u) for u in range(6)] == [8, 16, 32, 64, 128, 128]
    assert [new_tuples_needed(c, 128, u) for u in range(5)] == [8, 16, 32, 64, 64]
    assert new_tuples_needed(c, 1024) == 128 and new_tuples_needed(c, 1024, 40) == 128
    off = PSConfig(iter_new_frac=0.5, iter_new_cap=128)
    assert new_tuples_needed(off, 1024, 0) == 128
    rows = PSConfig(iter_new_rows=20, iter_new_frac=0.5, iter_new_cap=128, iter_new_ramp=8)
    assert new_tuples_needed(rows, 1024, 0) == 20  # iter_new_rows stays a floor
