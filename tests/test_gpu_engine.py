"""End-to-end parameter-server runs on one MI355X (in-process engine)."""
import pytest
import torch

from psx import _native
from psx.ops.lr import SolverOptions
from psx.runtime.config import PSConfig
from psx.runtime.engine import LocalEngine
from psx.utils.data import synth_finefood

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    base = dict(num_workers=1, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                rows_per_iter=128, epochs=1000, max_iters=30, init="zeros")
    base.update(kw)
    return PSConfig(**base)


def test_bsp_single_worker_learns(cuda):
    train, test = synth_finefood(20000, seed=0), synth_finefood(2000, seed=1)
    eng = LocalEngine(_cfg(max_iters=150), cuda, train=train, test=test)
    out = eng.run()
    assert out["rounds"] == 150
    accs = [r[3] for r in eng.log.book.server]
    assert accs[-1] > 0.33, accs[-10:]  # well above the 0.2 prior
    assert _native.hip_loaded_path() is not None


@pytest.mark.parametrize("c", [-1, 2])
def test_async_two_workers_threads(cuda, c):
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    cfg = _cfg(num_workers=2, consistency_model=c, max_iters=20,
               inject_worker_delay_ms={1: 5.0})
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    out = eng.run()
    assert out["updates"] >= 40
    if c > 0:
        assert out["max_vc_gap"] <= c + 1
    ws = eng.log.book.worker
    assert {r[1] for r in ws} == {0, 1}


def test_gd_solver_mode(cuda):
    train, test = synth_finefood(4000, seed=0), synth_finefood(500, seed=1)
    eng = LocalEngine(_cfg(max_iters=10, solver=SolverOptions(mode="gd", gd_lr=2.0, iters=3)), cuda,
                      train=train, test=test)
    out = eng.run()
    assert out["rounds"] == 10
    torch.cuda.synchronize()


def test_perf_log_device_phases(cuda, tmp_path):
    import json

    train, test = synth_finefood(4000, seed=0), synth_finefood(500, seed=1)
    eng = LocalEngine(_cfg(max_iters=12, log_dir=str(tmp_path), perf_log=True, trace_path=str(tmp_path / "t.json")),
                      cuda, train=train, test=test)
    eng.run()
    rows = [r.split(";") for r in (tmp_path / "logs-perf.csv").read_text().strip().split("\n")[1:]]
    assert len(rows) == 12
    solve_us = [float(r[4]) for r in rows]
    assert all(5.0 < s < 50000.0 for s in solve_us), solve_us  # device time of the local solve
    ev = json.loads((tmp_path / "t.json").read_text())["traceEvents"]
    assert any(e.get("tid") == "device" and e["name"] == "solve" for e in ev)


def test_inprocess_checkpoint_resume_gpu(cuda, tmp_path):
    train, test = synth_finefood(6000, seed=0), synth_finefood(500, seed=1)
    kw = dict(num_workers=2, min_buffer_size=256, max_buffer_size=256, init="random")
    ref = LocalEngine(_cfg(max_iters=6, **kw), cuda, train=train, test=test)
    ref.run()
    a = LocalEngine(_cfg(max_iters=3, checkpoint_dir=str(tmp_path), checkpoint_every=3, **kw), cuda, train=train,
                    test=test)
    a.run()
    b = LocalEngine(_cfg(max_iters=3, checkpoint_dir=str(tmp_path), resume=True, **kw), cuda, train=train, test=test)
    b.run()
    torch.cuda.synchronize()
    d = (b.server.w - ref.server.w).abs().max().item()
    assert d < 1e-4 * max(1.0, ref.server.w.abs().max().item()), d


def test_checkpoint_mid_run_snapshot_gpu(cuda, tmp_path):
    """A checkpoint taken mid-run holds exactly the weights of its step, although
    the run keeps updating them while the D2H copy is in flight (step 5 of 9)."""
    from psx.utils.checkpoint import load_server

    train, test = synth_finefood(6000, seed=0), synth_finefood(500, seed=1)
    kw = dict(num_workers=2, min_buffer_size=256, max_buffer_size=256, init="random")
    ref = LocalEngine(_cfg(max_iters=5, **kw), cuda, train=train, test=test)
    ref.run()
    a = LocalEngine(_cfg(max_iters=9, checkpoint_dir=str(tmp_path), checkpoint_every=5, **kw), cuda, train=train,
                    test=test)
    a.run()
    torch.cuda.synchronize()
    st = load_server(str(tmp_path))
    assert st["extra"]["step"] == 5
    w5 = st["w"].to(cuda)
    d = (w5 - ref.server.w).abs().max().item()
    assert d < 1e-5 * max(1.0, ref.server.w.abs().max().item()), d
    assert (a.server.w - ref.server.w).abs().max().item() > 0  # the run did move on after the snapshot


def test_asp_crash_dropped_gpu(cuda):
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    eng = LocalEngine(_cfg(num_workers=3, consistency_model=-1, max_iters=10, inject_worker_crash={2: 4}), cuda,
                      train=train, test=test)
    out = eng.run()
    assert out["failed_workers"] == [2] and eng.workers[0].iters >= 10


@pytest.mark.parametrize("N", [1, 2])
def test_paired_eval_rows_match_unpaired(cuda, N):
    """Worker-0 rows + deferred server rows from one paired pass == separate evaluations."""
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    books, ws = [], []
    for pair in (True, False):
        eng = LocalEngine(_cfg(num_workers=N, max_iters=12, init="random", pair_eval=pair), cuda, train=train,
                          test=test)
        if pair:
            assert eng.server.pair is not None and eng.server.pair.shared
        eng.run()
        books.append(eng.log.book)
        ws.append(eng.server.w.cpu())
    # (runs are not bitwise reproducible: the window size follows the wall-clock arrival rate)
    assert torch.allclose(ws[0], ws[1], atol=2e-2 * ws[1].abs().max().item())
    s0 = sorted((r[1], r[3]) for r in books[0].server)
    s1 = sorted((r[1], r[3]) for r in books[1].server)
    assert [v for v, _ in s0] == list(range(12)) == [v for v, _ in s1]
    assert max(abs(a[1] - b[1]) for a, b in zip(s0, s1)) < 0.05
    w0 = sorted((r[1], r[2], r[5]) for r in books[0].worker)
    w1 = sorted((r[1], r[2], r[5]) for r in books[1].worker)
    assert len(w0) == len(w1) == 12 * N
    assert max(abs(a[2] - b[2]) for a, b in zip(w0, w1)) < 0.05


@pytest.mark.parametrize("N", [1, 2])
def test_riding_eval_matches_separate_launches(cuda, monkeypatch, N):
    """Evaluation rows riding in the next solve's bwd_update launches (and, for one
    worker, the server update fused into the solve's finalisation) log exactly the
    rows of the separate evaluation / update launches, and end at the same model.  (The
    Python round loop, where riding is a choice: the native loops always ride.)"""
    monkeypatch.setenv("PSX_NATIVE_LANES", "0")
    monkeypatch.setenv("PSX_NATIVE_BSP", "0")
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    kw = dict(num_workers=N, max_iters=10, init="random", min_buffer_size=512, max_buffer_size=512)
    res = []
    for ride in ("1", "0"):
        monkeypatch.setenv("PSX_EVAL_RIDE", ride)
        eng = LocalEngine(_cfg(**kw), cuda, train=train, test=test)
        if ride == "1":
            assert eng.workers[0].solver.can_ride(eng.workers[0].ring, eng.workers[0].w)
        eng.run()
        torch.cuda.synchronize()
        book = eng.log.book
        res.append((eng.server.w.cpu(), sorted((r[1], r[2], r[3]) for r in book.server),
                    sorted((r[1], r[2], r[3], r[4], r[5], r[6]) for r in book.worker)))
    assert torch.equal(res[0][0], res[1][0])
    assert [r[0] for r in res[0][1]] == list(range(10))
    assert res[0][1] == res[1][1]
    assert len(res[0][2]) == 10 * N and res[0][2] == res[1][2]


def test_native_bsp_loop_matches_python_loop(cuda, monkeypatch):
    """The native BSP round loop (csrc/runtime/bsp_loop.h) logs exactly the rows of
    the Python loop, ends at the same model, producer cursor, window and tracker."""
    monkeypatch.setenv("PSX_NATIVE_LANES", "0")  # (the single-worker loop; the lanes loop has its own tests)
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    kw = dict(num_workers=1, max_iters=25, init="random", min_buffer_size=256, max_buffer_size=256,
              rows_per_iter=96)
    res = []
    for native in ("1", "0"):
        monkeypatch.setenv("PSX_NATIVE_BSP", native)
        eng = LocalEngine(_cfg(**kw), cuda, train=train, test=test)
        assert eng._native_bsp_ok() == (native == "1")
        out = eng.run()
        assert out.get("native_loop", False) == (native == "1")
        torch.cuda.synchronize()
        wk = eng.workers[0]
        book = eng.log.book
        res.append((eng.server.w.cpu(), sorted((r[1], r[2], r[3]) for r in book.server),
                    sorted((r[1], r[2], r[3], r[4], r[5], r[6]) for r in book.worker),
                    (wk.source.next_local, wk.window.size, wk.window.start, wk.tuples_seen, wk.vc, wk.iters,
                     eng.server.updates, eng.server.tracker.min_clock())))
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1] and [r[0] for r in res[0][1]] == list(range(25))
    assert res[0][2] == res[1][2] and len(res[0][2]) == 25
    assert res[0][3] == res[1][3]


def test_native_bsp_loop_producer_clock(cuda):
    """The native loop on the reference producer clock (-p): rows arrive by the
    schedule, every round logs a worker and a server row."""
    train, test = synth_finefood(4000, seed=0), synth_finefood(500, seed=1)
    eng = LocalEngine(_cfg(stream_mode="schedule", producer_time_per_event=2.0, max_iters=40, init="random"), cuda,
                      train=train, test=test)
    assert eng._native_bsp_ok()
    out = eng.run()
    assert out["native_loop"] and out["rounds"] == 40
    book = eng.log.book
    assert [r[1] for r in book.server] == list(range(40))
    assert len(book.worker) == 40 and eng.workers[0].tuples_seen >= 128


def test_concurrent_worker_lanes_match_sequential(cuda):
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    ws, books = [], []
    for conc in (True, False):
        eng = LocalEngine(_cfg(num_workers=4, max_iters=10, init="random", concurrent_workers=conc,
                               min_buffer_size=256, max_buffer_size=256), cuda, train=train, test=test)
        out = eng.run()
        assert out["rounds"] == 10 and out["updates"] == 40
        ws.append(eng.server.w.cpu())
        books.append(eng.log.book)
    assert torch.allclose(ws[0], ws[1], atol=1e-4 * max(1.0, ws[1].abs().max().item()))
    assert len(books[0].worker) == len(books[1].worker) == 40 and len(books[0].server) == 10


@pytest.mark.parametrize("c", [-1, 3])
def test_async_event_scheduler_four_workers(cuda, c):
    """SSP/ASP default on a GPU: one host thread polling per-worker HIP events."""
    train, test = synth_finefood(16000, seed=0), synth_finefood(1000, seed=1)
    cfg = _cfg(num_workers=4, consistency_model=c, max_iters=40)
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    assert eng._event_scheduler()
    out = eng.run()
    # solves still in flight when the run stops are not applied
    assert min(w.iters for w in eng.workers) >= 40 and 160 <= out["updates"] <= sum(w.iters for w in eng.workers)
    if c > 0:
        assert out["max_vc_gap"] <= c + 1
    assert {r[1] for r in eng.log.book.worker} == {0, 1, 2, 3}
    accs = [r[3] for r in eng.log.book.server]
    assert len(accs) >= 40 and accs[-1] > 0.25


def test_async_event_scheduler_drops_crashed_worker(cuda, monkeypatch):
    """Event scheduler on a GPU: an injected crash retires the worker (ASP) and the
    survivors keep stepping; server rows move to the lowest surviving worker.  (The
    lanes loop takes such runs by default: tests/test_gpu_async_lanes.py.)"""
    monkeypatch.setenv("PSX_ASYNC_LANES", "0")
    train, test = synth_finefood(12000, seed=0), synth_finefood(1000, seed=1)
    cfg = _cfg(num_workers=3, consistency_model=-1, max_iters=20, inject_worker_crash={0: 3})
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    assert eng._event_scheduler()
    out = eng.run()
    assert out["failed_workers"] == [0] and eng.workers[0].iters == 3
    assert min(eng.workers[1].iters, eng.workers[2].iters) >= 20
    assert len(eng.log.book.server) >= 20


def test_stream_handle_follows_current_stream(cuda):
    """Every native launch takes its stream from stream_handle: it must follow
    set_stream / stream contexts exactly like torch.cuda.current_stream."""
    from psx.ops.lr import stream_handle

    dev = torch.device(cuda)
    main = torch.cuda.current_stream(dev)
    assert stream_handle(dev) == main.cuda_stream == stream_handle(cuda)
    side = torch.cuda.Stream(dev)
    torch.cuda.set_stream(side)
    try:
        assert stream_handle(dev) == side.cuda_stream
    finally:
        torch.cuda.set_stream(main)
    with torch.cuda.stream(side):
        assert stream_handle(cuda) == side.cuda_stream
    assert stream_handle(dev) == main.cuda_stream


@pytest.mark.parametrize("rows", [96, 600, 1024])
def test_fused_ingest_matches_ring_copy(cuda, monkeypatch, rows):
    """New rows copied into the ring by the solve's first kernel (fused ingest, up to
    kMaxFusedIngest = 1024 rows per solve, a fully fresh window included) end at the
    same model and log the same rows as the separate ring-ingest launch (Python
    loop), and as the native loop (which always fuses)."""
    monkeypatch.setenv("PSX_NATIVE_LANES", "0")  # (the single-worker loops; the lanes loop has its own tests)
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    res = []
    for fused, native in ((True, "0"), (False, "0"), (True, "1")):
        monkeypatch.setenv("PSX_NATIVE_BSP", native)
        cfg = _cfg(max_iters=12, init="random", min_buffer_size=1024, max_buffer_size=1024, rows_per_iter=rows,
                   solver=SolverOptions(fused_ingest=fused))
        eng = LocalEngine(cfg, cuda, train=train, test=test)
        eng.run()
        torch.cuda.synchronize()
        book = eng.log.book
        res.append((eng.server.w.cpu(), sorted((r[1], r[2], r[3], r[4], r[5], r[6]) for r in book.worker)))
    # fused vs ring copy: the window statistics add the same values in another order
    w0, w1 = res[0][0], res[1][0]
    assert torch.allclose(w0, w1, rtol=0, atol=1e-4 * w1.abs().max().item())
    assert [r[:2] + r[5:] for r in res[0][1]] == [r[:2] + r[5:] for r in res[1][1]]
    assert max(abs(a[2] - b[2]) for a, b in zip(res[0][1], res[1][1])) < 1e-3
    # native loop vs Python loop, both fused: bit for bit
    assert torch.equal(res[0][0], res[2][0])
    assert res[0][1] == res[2][1] and len(res[0][1]) == 12
