"""Asynchronous consistency (SSP / ASP) in the native lanes loop on one MI355X
(csrc/kernels/lanes_async.hip, LanesLoop.run_async): ONE persistent launch, each
worker solving on its own XCD as soon as the C++ tracker releases it, updates
serial in arrival (ticket) order on the device, the worker / server rows
evaluated by the lanes themselves.

Reference: ServerProcessor.java:95-183 (apply on arrival, release per the
tracker, server row on worker-0 deltas), MessageTracker.java:69-87."""
import pytest
import torch

from psx import _native
from psx.runtime.config import PSConfig
from psx.runtime.engine import LocalEngine
from psx.utils.data import synth_finefood

pytestmark = pytest.mark.gpu


def _engine(dev, c, workers=8, iters=12, delays=None, train_rows=20000, **kw):
    train = synth_finefood(train_rows, seed=0)
    test = synth_finefood(4877, seed=1)
    cfg = PSConfig(num_workers=workers, consistency_model=c, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=1024, epochs=1000, max_iters=iters, min_buffer_size=128, max_buffer_size=1024,
                   init="random", seed=0, inject_worker_delay_ms=dict(delays or {}), **kw)
    return LocalEngine(cfg, dev, train=train, test=test)


def _gap_in_order(rows):
    """max over the worker rows, in ticket (submission) order, of max - min of the
    workers' latest logged clocks (tools/plot_logs.py:max_vc_gap without the
    timestamp sort: rows of one millisecond keep their order)."""
    latest, gap = {}, 0
    parts = {r[1] for r in rows}
    for r in rows:
        latest[r[1]] = r[2]
        if len(latest) == len(parts):
            gap = max(gap, max(latest.values()) - min(latest.values()))
    return gap


def _replay(rows, workers, c):
    """The rows' ticket order through a fresh C++ VectorClockTracker: every delta
    is the one the tracker expects (a protocol violation raises), and a worker's
    next clock is only ever one it was released for."""
    t = _native.host.VectorClockTracker(workers, c)
    released = {k: 0 for k in range(workers)}  # bootstrap: vc 0 to everybody
    for r in rows:
        k, v = int(r[1]), int(r[2])
        assert released.get(k) == v, (k, v, released)
        del released[k]
        for j, u in t.on_delta(k, v):
            assert j not in released
            released[j] = u
    return t


@pytest.mark.parametrize("c", [-1, 3])
def test_async_lanes_run_natively(cuda, c):
    eng = _engine(cuda, c, iters=16)
    out = eng.run()
    assert out.get("async_lanes"), out
    assert eng.server.updates == 8 * 16
    book = eng.log.book
    assert len(book.worker) == 8 * 16
    assert len(book.server) == 16  # one server row per worker-0 delta (ServerProcessor.java:154)
    assert torch.isfinite(eng.server.w).all()
    assert max(r[2] for r in book.server) > 0.35  # the global model learns
    _replay(book.worker, 8, c)
    for k in range(8):
        vcs = [r[2] for r in book.worker if r[1] == k]
        assert vcs == list(range(16)), (k, vcs)


@pytest.mark.parametrize("c,bound", [(0, 1), (2, 3), (-1, None)])
def test_async_lanes_gap_with_straggler(cuda, c, bound):
    """The reference validates its consistency models from the logs (README.md:
    299-321): with worker 2 slowed on the device, the logged vector-clock gap stays
    within the model's bound (BSP <= 1, SSP(D) <= D + 1) and ASP runs ahead."""
    eng = _engine(cuda, c, iters=24, delays={2: 3.0})  # +3 ms per iteration of worker 2
    if c == 0:  # sequential consistency through the asynchronous loop (the tracker decides)
        out = eng._run_async_lanes()
    else:
        out = eng.run()
        assert out.get("async_lanes"), out
    eng.log.drain(block=True)
    rows = eng.log.book.worker
    t = _replay(rows, 8, c)
    gap = _gap_in_order(rows)
    if bound is not None:
        assert gap <= bound, gap
        assert t.max_gap <= bound, t.max_gap
    else:
        assert gap >= 4, gap  # eventual: the fast workers are not held back by worker 2


def test_async_one_lane_equals_bsp_lanes_bitwise(cuda, monkeypatch):
    """One lane: the asynchronous update w += lr * delta is the BSP lanes loop's
    update of a one-worker round -- weights and rows bit for bit (both evaluating with
    the dense MFMA pass: PSX_SPARSE_EVAL=0)."""
    monkeypatch.setenv("PSX_SPARSE_EVAL", "0")
    outs = []
    for mode in ("bsp", "async"):
        eng = _engine(cuda, -1, workers=1, iters=6)
        if mode == "bsp":
            eng._run_bsp_lanes()
        else:
            eng._run_async_lanes()
        eng.log.drain(block=True)
        torch.cuda.synchronize()
        outs.append((eng.server.w.clone(), [(r[1], r[2], r[3], r[4], r[5]) for r in eng.log.book.worker]))
        eng.log.close()
    (wa, ra), (wb, rb) = outs
    assert torch.equal(wa, wb), (wa - wb).abs().max().item()
    assert ra == rb


def test_async_lanes_continue_across_runs(cuda):
    """Two runs of the same engine: the second continues the tickets, clocks and
    snapshot of the first (the bench's warm-up + timed region)."""
    eng = _engine(cuda, 2, iters=5)
    eng.run(close_log=False)
    eng.cfg.max_iters = 7
    eng.run(close_log=False)
    eng.log.drain(block=True)
    assert eng.server.updates == 8 * 12
    rows = eng.log.book.worker
    assert len(rows) == 8 * 12
    _replay(rows, 8, 2)
    assert eng._lanes.tickets == 8 * 12


@pytest.mark.parametrize("c", [2, -1])
def test_async_lanes_replay_float64_oracle(cuda, c):
    """8 workers, SSP(2) / ASP, worker 2 a straggler: the run replayed on the CPU
    from the loop's own record of every ticket (LanesLoop.set_async_debug) --
      (1) the server's update chain w = w0 + lr * delta_t in ticket order
          reproduces the device weights (ServerProcessor.java:148-151, one
          partition = serial updates);
      (2) every delta equals the float64 oracle of the reference solve
          (psx/models/reference.py) from the SNAPSHOT its release pulled (the
          replayed weights after ticket q.snap) on the window it logged;
      (3) the float64 chain -- oracle deltas applied to oracle snapshots -- ends
          within tolerance of the device weights;
      (4) every server row's F1 / accuracy equals the replayed global model's
          test-set metrics right after the logging worker's update (:154-165)."""
    from psx.models.reference import local_solve_reference, predict
    from psx.utils.metrics import confusion, metrics_from_confusion

    iters, N = 3, 8
    eng = _engine(cuda, c, workers=N, iters=iters, delays={2: 2.0})
    spec, lr = eng.spec, float(eng.cfg.lr)
    W = list(eng.workers)
    w0 = eng.server.w.detach().double().cpu().clone()
    lp = eng._lanes_loop(W)
    n_upd = N * iters
    dbg = torch.zeros(n_upd, spec.P, dtype=torch.float32, device=cuda)
    lp.set_async_debug(dbg.data_ptr(), n_upd)
    out = eng.run()
    assert out.get("async_lanes"), out
    eng.log.drain(block=True)
    torch.cuda.synchronize()
    log = [list(r) for r in lp.async_log]
    assert [r[0] for r in log] == list(range(1, n_upd + 1)), [r[0] for r in log]
    D = dbg.double().cpu()
    ds = W[0].source.ds
    # (1) the update chain, and the snapshots it passes through
    snaps = {0: w0.clone()}
    w = w0.clone()
    for i in range(n_upd):
        w = w + lr * D[i]
        snaps[i + 1] = w.clone()
    wdev = eng.server.w.detach().double().cpu()
    assert torch.allclose(w, wdev, atol=2e-6, rtol=0), (w - wdev).abs().max().item()
    # (2) + (3) the deltas against the oracle from their pulled snapshots
    ref_snaps = {0: w0.clone()}
    wref = w0.clone()
    worst = 0.0
    for i, (t, l, k, vc, snap, B, start, first, step, n, first2, n2) in enumerate(log):
        assert n + n2 == B, (t, B, n, n2)  # (per-iteration rows: the window IS the new rows)
        rows = [first + j * step for j in range(n)] + [first2 + j * step for j in range(n2)]
        Xw = ds.X[rows, : spec.F].double().cpu()
        yw = ds.y[rows].long().cpu()
        ws = snaps[snap]
        res = local_solve_reference(Xw, yw, spec.coef(ws), spec.intercept(ws))
        ref = spec.pack(res.coef, res.intercept).double() - ws
        err, scale = (D[i] - ref).abs().max().item(), ref.abs().max().item()
        worst = max(worst, err / max(scale, 1e-12))
        assert err <= 2e-2 * scale + 1e-4, (t, k, err, scale)
        wr = ref_snaps[snap]
        r2 = local_solve_reference(Xw, yw, spec.coef(wr), spec.intercept(wr))
        wref = wref + lr * (spec.pack(r2.coef, r2.intercept).double() - wr)
        ref_snaps[i + 1] = wref.clone()
    assert worst <= 1e-3, worst  # (measured 6e-6 .. 8e-6: profiles/r05/README.md)
    chain = (wref - wdev).abs().max().item()
    assert chain <= 2e-4, chain  # (measured 1.4e-5 .. 1.7e-5)
    # (4) the server rows: worker 0's updates in ticket order
    Xt, yt = eng.evalset.X[:, : spec.F].double().cpu(), eng.evalset.y.long().cpu()
    srows = list(eng.log.book.server)
    t_log = [r[0] for r in log if r[2] == 0]
    assert len(srows) == len(t_log) == iters
    for (ts, vc, f1, acc), t in zip(srows, t_log):
        ws = snaps[t]
        pred = predict(Xt, spec.coef(ws), spec.intercept(ws))
        f1r, accr = metrics_from_confusion(confusion(yt.numpy(), pred.numpy(), spec.K))
        assert abs(f1 - f1r) <= 2e-3 and abs(acc - accr) <= 2e-3, (t, f1, f1r, acc, accr)
    print(f"replay c={c}: worst delta rel err {worst:.2e}, float64 chain max |dw| {chain:.2e}")


def test_async_sparse_eval_rows_equal_dense(cuda, monkeypatch):
    """The asynchronous lanes' evaluation over the ELL test rows (EvalSet.ell,
    lanes_body.h lane_pair_eval_ell) against the dense MFMA pass: the same training
    (weights bit for bit: the evaluation does not feed back) and the same rows -- every
    product x * w is exact in both, only the summation order differs, so at most an
    argmax tie flips (counts within 2 of 4,877)."""
    outs = []
    for sp in ("0", "1"):
        monkeypatch.setenv("PSX_SPARSE_EVAL", sp)
        eng = _engine(cuda, -1, workers=1, iters=6)  # (one worker: a deterministic schedule)
        assert (eng.evalset.ell_nz > 0) == (sp == "1")
        eng.run(close_log=False)
        eng.log.drain(block=True)
        torch.cuda.synchronize()
        outs.append((eng.server.w.clone(), sorted((r[1], r[2], r[4], r[5]) for r in eng.log.book.worker),
                     sorted((-1, r[1], r[2], r[3]) for r in eng.log.book.server)))
        eng.log.close()
    (wa, ra, sa), (wb, rb, sb) = outs
    assert torch.equal(wa, wb)
    assert len(ra) == len(rb) == 6 and len(sa) == len(sb)
    for a, b in zip(ra + sa, rb + sb):
        assert a[:2] == b[:2] and all(abs(x - y) <= 2 / 4877 + 1e-6 for x, y in zip(a[2:], b[2:])), (a, b)


# ---- fault injection on the lanes loops (the Python schedulers' semantics:
# roles.py WorkerRole.compute fails at iteration ITER, engine.py _worker_failed) ----

def test_async_lanes_crash_dropped_rows_move(cuda):
    """ASP, worker 0 crashes at its 4th iteration: the host loop retires it (drop), the
    others run their 12 iterations, and the server rows move to worker 1's deltas."""
    eng = _engine(cuda, -1, workers=4, iters=12, inject_worker_crash={0: 3})
    assert eng._async_lanes_ok()
    out = eng.run()
    assert out["async_lanes"] and out["failed_workers"] == [0]
    assert eng.workers[0].iters == 3 and [w.iters for w in eng.workers[1:]] == [12, 12, 12]
    assert out["updates"] == 3 + 36
    srv = eng.log.book.server  # worker 0's 3, then worker 1's released after the crash
    assert 3 + 6 <= len(srv) <= 3 + 12, len(srv)
    assert [r[1] for r in srv[3:]] == sorted(r[1] for r in srv[3:])
    wrows = eng.log.book.worker
    assert sum(1 for r in wrows if r[1] == 0) == 3
    assert torch.isfinite(eng.server.w).all()


def test_async_lanes_crash_fail_policy_raises(cuda):
    """SSP(2) (auto policy = fail): the crash ends the run with WorkerFailure."""
    from psx.runtime.faults import WorkerFailure

    eng = _engine(cuda, 2, workers=3, iters=10, inject_worker_crash={1: 2})
    with pytest.raises(WorkerFailure, match="worker 1"):
        eng.run()
    assert eng.workers[1].iters == 2


def test_async_lanes_stop_leaves_cleanly(cuda):
    """SSP(1): worker 2 leaves after 3 iterations (its last delta applied, then retired):
    the others are no longer held back by its clock and finish their 10."""
    eng = _engine(cuda, 1, workers=3, iters=10, inject_worker_stop={2: 3})
    out = eng.run()
    assert out.get("left_workers") == [2] and out["failed_workers"] == []
    assert [w.iters for w in eng.workers] == [10, 10, 3]
    assert out["updates"] == 23


def test_async_lanes_leave_and_crash_across_chunks(cuda, tmp_path):
    """ASP with checkpoints every 4 updates (a chunk of the run per checkpoint): worker 1
    leaves after 3 iterations and worker 2 crashes at its 3rd (drop) in early chunks.  The
    later chunks -- and a second run of the engine -- must not start either again: a retired
    worker keeps its tracker `sent` bit, and re-starting it would push a delta the tracker
    refuses ('delta from retired worker') or report the crash twice."""
    eng = _engine(cuda, -1, workers=4, iters=10, inject_worker_stop={1: 3}, inject_worker_crash={2: 2},
                  on_worker_failure="drop", checkpoint_dir=str(tmp_path / "ck"), checkpoint_every=4)
    assert eng._async_lanes_ok()
    out = eng.run(close_log=False)
    assert out.get("left_workers") == [1] and out["failed_workers"] == [2]
    assert [w.iters for w in eng.workers] == [10, 3, 2, 10]
    assert out["updates"] == 10 + 3 + 2 + 10
    eng.cfg.max_iters = 4  # a second run: the live workers only
    out2 = eng.run()
    assert out2["failed_workers"] == [2] and [w.iters for w in eng.workers] == [14, 3, 2, 14]
    assert torch.isfinite(eng.server.w).all()


def test_bsp_lanes_crash_dropped_and_delay(cuda):
    """BSP on the lanes loop: a straggler sleeps on the device (no Python scheduler), an
    injected crash (drop) ends a chunk at its round and the rest runs without it."""
    eng = _engine(cuda, 0, workers=3, iters=8, delays={1: 2.0}, inject_worker_crash={2: 4},
                  on_worker_failure="drop")
    assert eng._lanes_ok()
    out = eng.run()
    assert out["lanes"] and out["rounds"] == 8 and out["failed_workers"] == [2]
    assert [w.iters for w in eng.workers] == [8, 8, 4]
    assert out["updates"] == 4 * 3 + 4 * 2
    assert 0.002 * 8 <= out["elapsed_s"]  # the 2 ms straggler holds every round


def test_async_lanes_trace_and_perf_log(cuda, tmp_path):
    """--trace / --perf_log on the async lanes loop: the kernels record each update's
    released / solved / pushed times on the device; one perf row per update and device
    "solve" spans on the host timeline (no Python scheduler)."""
    import json

    eng = _engine(cuda, -1, workers=3, iters=6, log_dir=str(tmp_path), perf_log=True,
                  trace_path=str(tmp_path / "t.json"))
    assert eng._async_lanes_ok()
    out = eng.run()
    assert out["async_lanes"] and out["updates"] == 18
    rows = [r.split(";") for r in (tmp_path / "logs-perf.csv").read_text().strip().split("\n")[1:]]
    assert len(rows) == 18 and [int(r[0]) for r in rows] == sorted(int(r[0]) for r in rows)
    assert all(5.0 < float(r[4]) < 50000.0 for r in rows)  # the solve's device time (us)
    ev = json.loads((tmp_path / "t.json").read_text())["traceEvents"]
    dev = [e for e in ev if e.get("tid") == "device" and e["name"] == "solve"]
    assert len(dev) == 18 and {e["args"]["worker"] for e in dev} == {0, 1, 2}
    host = [e for e in ev if e.get("tid") != "device"]
    if host:  # device spans sit inside the run's host time frame
        t0 = min(e["ts"] for e in ev if e.get("tid") != "device") - 1e6
        assert all(e["ts"] > t0 for e in dev)
