"""Multi-lane BSP round kernel (csrc/kernels/lanes_kernels.hip, csrc/runtime/lanes_loop.h)
on one MI355X: every in-process worker's solve on its own XCD, the cross-lane update
and the riding evaluation in ONE launch per round."""
import os

import pytest
import torch

from psx import _native
from psx.models.logreg import ModelSpec
from psx.models.reference import local_solve_reference
from psx.ops.lr import Fragments, SolverOptions, stream_handle
from psx.runtime.config import PSConfig
from psx.runtime.engine import LocalEngine
from psx.utils.data import synth_finefood
from psx.utils.logsink import LogSink

pytestmark = pytest.mark.gpu


def _loop(spec, ks, N, train, test, w, dev, rows=1024, cap=1024, sink=None, lr=None, frags=None, opts=None,
          **extra):
    """A LanesLoop over worker ids `ks` (of N) with fresh rings / windows."""
    h, host = _native.hip(), _native.host
    o = opts or SolverOptions()
    sc = h.SolverCfg()
    sc.K, sc.F, sc.Fp, sc.P, sc.cap = spec.K, spec.F, spec.Fp, spec.P, cap
    sc.iters, sc.hist, sc.ls_max, sc.mode = o.iters, o.hist, o.ls_max, 0
    sc.center, sc.zero_const, sc.nslots, sc.gd_lr, sc.tol = 1, 1, o.nslots, o.gd_lr, o.tol
    rings = [(torch.zeros(cap, spec.Fp, dtype=torch.bfloat16, device=dev),
              torch.zeros(cap, dtype=torch.int32, device=dev)) for _ in ks]
    wins = [host.SlidingWindow(cap, cap, 0.3, 500, cap) for _ in ks]
    frags = frags or [Fragments(spec, dev) for _ in range(3)]  # (3: overlapped launches)
    d = dict(scfg=sc, dsX=train.X.data_ptr(), dsy=train.y.data_ptr(), ds_rows=int(train.rows), N=N,
             per_iter_rows=rows, k=list(ks), X=[r[0].data_ptr() for r in rings], y=[r[1].data_ptr() for r in rings],
             window=[wn.handle for wn in wins], w=w.data_ptr(), lr=float(lr if lr is not None else 1.0 / N),
             shi=[f.hi.data_ptr() for f in frags], slo=[f.lo.data_ptr() for f in frags],
             sb=[f.b.data_ptr() for f in frags], scoff=0, Xt=test.X.data_ptr(), yt=test.y.data_ptr(), T=test.T,
             sink=sink.native.handle if sink is not None else 0, api=host.capi(), **extra)
    lp = h.LanesLoop(d, None)
    return lp, (rings, wins, frags)


def _data(dev, rows=20000):
    spec = ModelSpec(1024, 6)
    train = synth_finefood(rows, seed=0).to(dev)
    from psx.ops.lr import EvalSet

    te = synth_finefood(4877, seed=1)
    return spec, train, EvalSet(spec, te.X, te.y, dev)


def _deltas(lp, L, spec, dev):
    out = []
    for l in range(L):
        d = torch.empty(spec.P, dtype=torch.float32, device=dev)
        lp.copy_out(l, 0, d.data_ptr(), stream_handle(dev))
        out.append(d)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("L", [8, 3])
def test_lanes_equal_separate_solves_bitwise(cuda, L):
    """Lane l of an L-lane round == worker l's round run alone on the GPU (bitwise)."""
    spec, train, ev = _data(cuda)
    w0 = spec.init("random", seed=3, device=cuda)
    w = w0.clone()
    lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda)
    assert lp.run(1, 0, stream_handle(cuda)) == 1
    multi = _deltas(lp, L, spec, cuda)
    for l in range(L):
        wl = w0.clone()
        lp1, keep1 = _loop(spec, [l], L, train, ev, wl, cuda)
        lp1.run(1, 0, stream_handle(cuda))
        alone = _deltas(lp1, 1, spec, cuda)[0]
        assert torch.equal(alone, multi[l]), (l, (alone - multi[l]).abs().max().item())
        assert torch.allclose(wl, w0 + multi[l] / L, atol=1e-6)  # alone: w += (1/N) * delta


def test_lanes_solve_matches_reference_and_update(cuda):
    """One lane's delta against the float64 oracle of the reference solve; the
    update is w + lr * (sum of the lane deltas)."""
    spec, train, ev = _data(cuda)
    L = 4
    w0 = spec.init("random", seed=5, device=cuda)
    w = w0.clone()
    lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda, lr=0.25)
    lp.run(1, 0, stream_handle(cuda))
    ds = _deltas(lp, L, spec, cuda)
    ref_w = w0 + 0.25 * (((ds[0] + ds[1]) + ds[2]) + ds[3])
    assert torch.allclose(w, ref_w, atol=2e-6, rtol=1e-5)
    # worker 2's window: its first 1024 shard rows (rows 2, 6, 10, ...)
    Xw = train.X[2::L][:1024, : spec.F].float().cpu()
    yw = train.y[2::L][:1024].long().cpu()
    res = local_solve_reference(Xw, yw, spec.coef(w0.cpu()), spec.intercept(w0.cpu()))
    ref = spec.pack(res.coef, res.intercept) - w0.cpu()
    got = ds[2].cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 2e-2 * scale + 1e-4, (err, scale)


def test_lanes_engine_rows_and_learning(cuda):
    """LocalEngine with 4 workers runs the lanes loop: one worker row per worker and
    one server row per round, vector clocks in order, the model learns."""
    train, test = synth_finefood(40000, seed=0), synth_finefood(2000, seed=1)
    cfg = PSConfig(num_workers=4, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=256, epochs=100, max_iters=60, min_buffer_size=128, max_buffer_size=1024,
                   init="random")
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    out = eng.run()
    assert out.get("lanes") == 4 and out["rounds"] == 60 and out["updates"] == 240
    book = eng.log.book
    assert [r[1] for r in book.server] == list(range(60))
    assert len(book.worker) == 240 and {r[1] for r in book.worker} == {0, 1, 2, 3}
    assert all(b[0] >= a[0] for a, b in zip(book.server, book.server[1:]))  # sink-stamped, in order
    assert book.server[-1][3] > 0.33, book.server[-5:]
    assert eng.server.tracker.min_clock() == 60
    loss = eng.workers[0].solver.loss.item()
    assert loss == loss and loss > 0


def test_lanes_server_rows_match_standalone_eval(cuda):
    """The riding evaluation of the global model == a standalone evaluation of it."""
    spec, train, ev = _data(cuda)
    w = spec.init("random", seed=9, device=cuda)
    log = LogSink(spec.K, cuda)
    lp, keep = _loop(spec, [0, 1], 2, train, ev, w, cuda, sink=log)
    lp.run(3, 0, stream_handle(cuda))
    lp.flush(stream_handle(cuda))
    torch.cuda.synchronize()
    book = log.book
    assert [r[1] for r in book.server] == [0, 1, 2]
    fr = Fragments(spec, cuda)
    fr.refresh(w)
    log2 = LogSink(spec.K, cuda)
    from psx.ops.lr import EvalScratch

    log2.server_eval(ev, fr, w, EvalScratch(cuda), 2)
    b2 = log2.book
    assert abs(book.server[-1][2] - b2.server[0][2]) < 1e-12 and abs(book.server[-1][3] - b2.server[0][3]) < 1e-12
    assert len(book.worker) == 6 and all(r[3] > 0 for r in book.worker)  # worker rows carry the loss
    log.close()
    log2.close()


def test_lanes_placement_fallback_same_result(cuda, monkeypatch):
    """A failed placement check (faked) runs the sc1 hand-off form: same deltas bitwise."""
    spec, train, ev = _data(cuda)
    w0 = spec.init("random", seed=4, device=cuda)
    wa, wb = w0.clone(), w0.clone()
    lpa, ka = _loop(spec, [0, 1], 2, train, ev, wa, cuda)
    assert lpa.hand_off_scope == 2
    lpa.run(2, 0, stream_handle(cuda))
    monkeypatch.setenv("PSX_FAKE_XCD_MISMATCH", "1")
    lpb, kb = _loop(spec, [0, 1], 2, train, ev, wb, cuda)
    assert lpb.hand_off_scope == 1
    lpb.run(2, 0, stream_handle(cuda))
    da, db = _deltas(lpa, 2, spec, cuda), _deltas(lpb, 2, spec, cuda)
    assert all(torch.equal(x, y) for x, y in zip(da, db))
    assert torch.equal(wa, wb)


def test_lanes_spin_timeout_is_reported(cuda):
    """A cross-workgroup wait that times out (forced: a 1-poll budget from round 3 on)
    surfaces as an error naming that solve, without a host synchronisation."""
    import re

    spec, train, ev = _data(cuda)
    w = spec.init("random", seed=4, device=cuda)
    lp, keep = _loop(spec, [0, 1], 2, train, ev, w, cuda)
    lp.inject_spin_timeout(3, 1)
    with pytest.raises(RuntimeError, match=r"timed out \(solve \d+") as ei:
        lp.run(40, 0, stream_handle(cuda))  # (raises here if the device got there first)
        torch.cuda.synchronize()
        lp.poll_errors()
    assert int(re.search(r"solve (\d+)", str(ei.value)).group(1)) >= 3, str(ei.value)
    torch.cuda.synchronize()


def test_engine_lanes_fault_maps_to_worker_failure(cuda, monkeypatch):
    from psx.runtime.faults import WorkerFailure

    monkeypatch.setenv("PSX_INJECT_SPIN_TIMEOUT", "2:1")
    train, test = synth_finefood(8000, seed=0), synth_finefood(500, seed=1)
    cfg = PSConfig(num_workers=2, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=256, epochs=100, max_iters=30, min_buffer_size=128, max_buffer_size=512)
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    with pytest.raises(WorkerFailure):
        eng.run()
    torch.cuda.synchronize()


def test_lanes_ring_rows_across_epoch_wrap(cuda):
    """Deliveries that wrap a worker's shard (the producer's next epoch) land in the
    ring inside the round kernel: slot s after round r holds the worker's tuple
    1024 r + s, i.e. dataset row k + ((1024 r + s) mod shard) * N."""
    spec, train, ev = _data(cuda, rows=3000)  # 1500 rows per worker: round 1 wraps
    w = spec.init("random", seed=2, device=cuda)
    lp, (rings, wins, frags) = _loop(spec, [0, 1], 2, train, ev, w, cuda, epochs=10)
    for rnd in range(3):
        lp.run(1, rnd, stream_handle(cuda))
        torch.cuda.synchronize()
        for k in (0, 1):
            j = torch.arange(1024) + 1024 * rnd
            rows = k + (j % 1500) * 2
            X, y = rings[k]
            assert torch.equal(X.cpu(), train.X[rows.to(cuda)].cpu()), (rnd, k)
            assert torch.equal(y.cpu(), train.y[rows.to(cuda)].cpu()), (rnd, k)


@pytest.mark.parametrize("sync", ["event", "inline"])
@pytest.mark.parametrize("L", [2, 8])
def test_side_stream_evaluation_rows_equal_riders(cuda, monkeypatch, L, sync):
    """The co-running side-stream evaluation (PSX_LANES_SIDE_EVAL=1) logs the same
    rows as the in-launch riders: every worker's local model and the global model,
    identical confusion counts."""
    spec, train, ev = _data(cuda)
    books = []
    if sync == "inline":  # the evaluation launch right behind each round on the same stream
        monkeypatch.setenv("PSX_SIDE_SYNC", "inline")
    for side in ("0", "1"):
        monkeypatch.setenv("PSX_LANES_SIDE_EVAL", side)
        w = spec.init("random", seed=6, device=cuda)
        log = LogSink(spec.K, cuda)
        lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda, sink=log)
        assert lp.side_eval == (side == "1")
        lp.run(4, 0, stream_handle(cuda))
        lp.flush(stream_handle(cuda))
        torch.cuda.synchronize()
        books.append(log.book)
        log.close()
    a, b = books
    assert [r[1:] for r in a.server] == [r[1:] for r in b.server] and len(a.server) == 4
    assert sorted(r[1:] for r in a.worker) == sorted(r[1:] for r in b.worker) and len(a.worker) == 4 * L
    monkeypatch.delenv("PSX_LANES_SIDE_EVAL")
    w = spec.init("random", seed=6, device=cuda)
    lp8, keep8 = _loop(spec, list(range(8)), 8, train, ev, w, cuda)
    assert not lp8.side_eval  # riders by default, 8 lanes too


def test_lanes_cadence_waits_for_new_tuples(cuda):
    """--iter_new_rows in the native loop: a round starts only once every lane saw
    the required new tuples since its last solve (per-round deliveries of 16 rows:
    3 deliveries per round for 48 new tuples)."""
    spec, train, ev = _data(cuda)
    w = spec.init("random", seed=3, device=cuda)
    lp, keep = _loop(spec, [0, 1], 2, train, ev, w, cuda, rows=16, new_rows=48)
    assert lp.new_tuples_needed(1024) == 48
    assert lp.run(4, 0, stream_handle(cuda)) == 4
    for l in range(2):
        assert lp.next_local(l) == 4 * 48 and lp.seen_at_solve(l) == 4 * 48
    torch.cuda.synchronize()


def test_lanes_cadence_fraction_and_cap(cuda):
    """iter_new_frac share of the window, capped at iter_new_cap (config.new_tuples_needed)."""
    from psx.runtime.config import new_tuples_needed

    spec, train, ev = _data(cuda)
    w = spec.init("zeros", device=cuda)
    lp, keep = _loop(spec, [0], 1, train, ev, w, cuda, rows=16, new_frac=0.3, new_cap=100, new_ramp=4)
    c = PSConfig(iter_new_frac=0.3, iter_new_cap=100, iter_new_ramp=4)
    for u in range(8):  # the ramp of the first solves (C++ and Python agree)
        assert lp.new_tuples_needed(1000, u) == new_tuples_needed(c, 1000, u), u
    for size in (1, 10, 16, 300, 333, 1024):
        assert lp.new_tuples_needed(size) == new_tuples_needed(c, size), size


def test_lanes_engine_producer_clock_cadence_and_deadline(cuda):
    """The reference's producer clock (-p) with the fresh-window cadence runs on the
    lanes loop: every worker row is >= the cadence's new tuples after the previous
    one, and the wall-clock stop ends a round that waits for tuples."""
    import time

    from psx.runtime.config import new_tuples_needed

    train, test = synth_finefood(40000, seed=0), synth_finefood(2000, seed=1)
    cfg = PSConfig(num_workers=4, consistency_model=0, producer_time_per_event=0.5, max_wallclock_s=3.0,
                   iter_new_frac=0.5, iter_new_cap=128, min_buffer_size=128, max_buffer_size=1024)
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    t0 = time.time()
    out = eng.run()
    took = time.time() - t0
    assert out.get("lanes") == 4, out
    assert out["rounds"] >= 4, out
    assert took < 3.0 + 1.5, took
    book = eng.log.book
    rows = {k: [r for r in book.worker if r[1] == k] for k in range(4)}
    for k, rs in rows.items():
        assert len(rs) == out["rounds"], (k, len(rs))
        seen = [r[-1] for r in rs]
        for a, b in zip(seen, seen[1:]):
            assert b - a >= min(new_tuples_needed(cfg, 128), 64), (k, seen)


@pytest.mark.parametrize("L", [1, 3, 8])
def test_lane_evaluation_rows_equal_riders(cuda, monkeypatch, L):
    """Each lane evaluating its own local model right after its solve
    (PSX_LANES_LANE_EVAL=1, LanesArgs::lane_eval; lane 0 paired with the previous
    update's global model) logs the same rows as the rider workgroups evaluating
    the previous round (the default): identical confusion counts, losses, clocks."""
    spec, train, ev = _data(cuda)
    books = []
    for riders in ("1", "0"):
        monkeypatch.setenv("PSX_LANES_LANE_EVAL", "0" if riders == "1" else "1")
        w = spec.init("random", seed=6, device=cuda)
        log = LogSink(spec.K, cuda)
        lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda, sink=log)
        assert lp.lane_eval == (riders == "0")
        lp.run(3, 0, stream_handle(cuda))
        lp.run(2, 3, stream_handle(cuda))  # a second call continues the pending server row
        lp.flush(stream_handle(cuda))
        torch.cuda.synchronize()
        books.append(log.book)
        log.close()
    a, b = books
    assert [r[1:] for r in a.server] == [r[1:] for r in b.server] and len(a.server) == 5
    assert [r[1:] for r in a.worker] == [r[1:] for r in b.worker] and len(a.worker) == 5 * L


@pytest.mark.parametrize("L", [3, 8])
def test_xcd_local_riders_rows_equal_riders(cuda, monkeypatch, L):
    """Riders popping XCD-local slices of the test set from per-XCD chunk queues
    (PSX_RIDERS_XCD=1, EvalMulti::xq; every chunk exactly once, stealing across
    XCDs) log the same rows as the default contiguous chunks."""
    spec, train, ev = _data(cuda)
    books = []
    monkeypatch.setenv("PSX_RIDERS_TILE", "0")  # (the pair-major riders' placement option)
    for xq in ("0", "1"):
        monkeypatch.setenv("PSX_RIDERS_XCD", xq)
        w = spec.init("random", seed=6, device=cuda)
        log = LogSink(spec.K, cuda)
        lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda, sink=log)
        lp.run(4, 0, stream_handle(cuda))
        lp.flush(stream_handle(cuda))
        torch.cuda.synchronize()
        books.append(log.book)
        log.close()
    a, b = books
    assert [r[1:] for r in a.server] == [r[1:] for r in b.server] and len(a.server) == 4
    assert [r[1:] for r in a.worker] == [r[1:] for r in b.worker] and len(a.worker) == 4 * L


@pytest.mark.parametrize("L,tile,ppi,gq", [(3, "1", "0", "0"), (8, "1", "0", "0"), (3, "2", "0", "0"),
                                           (8, "2", "0", "0"), (8, "2", "1", "0"), (3, "2", "2", "0"),
                                           (8, "2", "2", "1"), (3, "2", "1", "1"), (8, "1", "2", "1")])
def test_tile_resident_riders_rows_equal_pair_major(cuda, monkeypatch, L, tile, ppi, gq):
    """Riders holding their test tile in registers and running every model pair past
    it (PSX_RIDERS_TILE=1, eval_tile_body: the test set read once per round; =2: the
    lanes' own workgroups join them once their part of the round is done) log the
    same rows, bit for bit, as the pair-major riders (eval_multi_body); gq = 1: one tile
    queue per pair group, the group's fragments held across its tiles (PSX_RIDERS_GQ)."""
    spec, train, ev = _data(cuda)
    books = []
    monkeypatch.setenv("PSX_RIDERS_PPI", ppi)  # (work items of ppi model pairs; 0: all)
    monkeypatch.setenv("PSX_RIDERS_GQ", gq)
    for form in ("0", tile):
        monkeypatch.setenv("PSX_RIDERS_TILE", form)
        w = spec.init("random", seed=6, device=cuda)
        log = LogSink(spec.K, cuda)
        lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda, sink=log)
        lp.run(4, 0, stream_handle(cuda))
        lp.flush(stream_handle(cuda))
        torch.cuda.synchronize()
        books.append(log.book)
        log.close()
    a, b = books
    assert [r[1:] for r in a.server] == [r[1:] for r in b.server] and len(a.server) == 4
    assert [r[1:] for r in a.worker] == [r[1:] for r in b.worker] and len(a.worker) == 4 * L


def test_copy_out_all_equals_per_lane_copies(cuda):
    """The end-of-run batched copy (one launch for every lane's delta and loss)
    delivers what the per-lane copies deliver."""
    spec, train, ev = _data(cuda)
    L = 5
    w = spec.init("random", seed=2, device=cuda)
    lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda)
    lp.run(2, 0, stream_handle(cuda))
    one = _deltas(lp, L, spec, cuda)
    d_all = [torch.full((spec.P,), float("nan"), device=cuda) for _ in range(L)]
    l_all = [torch.full((1,), float("nan"), device=cuda) for _ in range(L)]
    l_one = [torch.full((1,), float("nan"), device=cuda) for _ in range(L)]
    lp.copy_out_all([x.data_ptr() for x in l_all], [x.data_ptr() for x in d_all], stream_handle(cuda))
    for i in range(L):
        lp.copy_out(i, l_one[i].data_ptr(), 0, stream_handle(cuda))
    torch.cuda.synchronize()
    for i in range(L):
        assert torch.equal(d_all[i], one[i]), i
        assert torch.equal(l_all[i], l_one[i]) and torch.isfinite(l_all[i]).all(), i


@pytest.mark.parametrize("L,tile,rows", [(8, "2", True), (3, "2", True), (8, "0", True), (8, "2", False)])
def test_overlapped_launches_equal_serial(cuda, monkeypatch, L, tile, rows):
    """Overlapped round launches (PSX_LANES_OVERLAP=1, LanesArgs::ovl: round r + 1's
    launch dispatched while round r's evaluation still runs, the hand-offs through
    the applied / evdone counters, fragments over three buffers) give the serial
    launches' weights and deltas bit for bit and the same rows, across two calls."""
    spec, train, ev = _data(cuda)
    monkeypatch.setenv("PSX_RIDERS_TILE", tile)
    out = []
    for ov in ("0", "1"):
        monkeypatch.setenv("PSX_LANES_OVERLAP", ov)
        w = spec.init("random", seed=6, device=cuda)
        log = LogSink(spec.K, cuda) if rows else None
        frags = [Fragments(spec, cuda) for _ in range(3)]
        lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda, sink=log, frags=frags)
        assert lp.overlap == (ov == "1")
        assert lp.run(6, 0, stream_handle(cuda)) == 6
        assert lp.run(3, 6, stream_handle(cuda)) == 3  # (a second call continues the chain)
        lp.flush(stream_handle(cuda))
        torch.cuda.synchronize()
        lp.poll_errors()
        out.append((w.clone(), _deltas(lp, L, spec, cuda), log.book if rows else None))
        if rows:
            log.close()
    (wa, da, a), (wb, db, b) = out
    assert torch.equal(wa, wb), (wa - wb).abs().max().item()
    for l in range(L):
        assert torch.equal(da[l], db[l]), l
    if rows:
        assert [r[1:] for r in a.server] == [r[1:] for r in b.server] and len(a.server) == 9
        assert [r[1:] for r in a.worker] == [r[1:] for r in b.worker] and len(a.worker) == 9 * L


@pytest.mark.parametrize("cap", [2048, 4096])
def test_lanes_long_ring_matches_reference(cuda, cap):
    """Rings over 1,024 rows (-max 2048 / 4096) stay on the one-launch path: each row
    workgroup stages several ring tiles every slot.  One lane's delta against the
    float64 oracle of the reference solve over its full window, and the update."""
    spec, train, ev = _data(cuda, rows=4 * cap + 64)
    assert _native.hip().lanes_supported(spec.Fp, spec.K, cap)
    L = 4
    w0 = spec.init("random", seed=5, device=cuda)
    w = w0.clone()
    lp, keep = _loop(spec, list(range(L)), L, train, ev, w, cuda, rows=cap, cap=cap, lr=0.25)
    assert lp.run(1, 0, stream_handle(cuda)) == 1
    ds = _deltas(lp, L, spec, cuda)
    lp.poll_errors()
    ref_w = w0 + 0.25 * (((ds[0] + ds[1]) + ds[2]) + ds[3])
    assert torch.allclose(w, ref_w, atol=2e-6, rtol=1e-5)
    Xw = train.X[1::L][:cap, : spec.F].float().cpu()
    yw = train.y[1::L][:cap].long().cpu()
    res = local_solve_reference(Xw, yw, spec.coef(w0.cpu()), spec.intercept(w0.cpu()))
    ref = spec.pack(res.coef, res.intercept) - w0.cpu()
    got = ds[1].cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 2e-2 * scale + 1e-4, (err, scale)


def test_lanes_long_ring_wraps_and_equals_alone(cuda):
    """A 2,048-row ring filled 1,500 rows per round: the second round's window wraps
    the ring at an unaligned start (its newest rows share the first ring tile).  The
    ring holds the expected rows, and lane l of the 3-lane round equals worker l's
    round run alone, bit for bit, in both rounds."""
    cap, rows, L = 2048, 1500, 3
    spec, train, ev = _data(cuda, rows=3 * 3000 + 64)
    w0 = spec.init("random", seed=3, device=cuda)
    w = w0.clone()
    lp, (rings, wins, frags) = _loop(spec, list(range(L)), L, train, ev, w, cuda, rows=rows, cap=cap, lr=0.0)
    multi = []
    for rnd in range(2):
        lp.run(1, rnd, stream_handle(cuda))
        multi.append(_deltas(lp, L, spec, cuda))
    lp.poll_errors()
    for k in range(L):
        j = torch.arange(3000)
        X, y = rings[k]
        slots = j % cap
        keep_ = j >= 3000 - cap
        src = (k + j * L)[keep_]
        assert torch.equal(X[slots[keep_].to(cuda)].cpu(), train.X[src.to(cuda)].cpu()), k
        assert torch.equal(y[slots[keep_].to(cuda)].cpu(), train.y[src.to(cuda)].cpu()), k
    for l in range(L):  # the wrapped window against the float64 oracle
        src = (l + torch.arange(3000 - cap, 3000) * L).to(cuda)
        res = local_solve_reference(train.X[src][:, : spec.F].float().cpu(), train.y[src].long().cpu(),
                                    spec.coef(w0.cpu()), spec.intercept(w0.cpu()))
        ref = spec.pack(res.coef, res.intercept) - w0.cpu()
        err = (multi[1][l].cpu() - ref).abs().max().item()
        assert err <= 2e-2 * ref.abs().max().item() + 1e-4, (l, err, ref.abs().max().item())
    for l in range(L):
        wl = w0.clone()  # (held: the loop keeps only its address)
        lp1, keep1 = _loop(spec, [l], L, train, ev, wl, cuda, rows=rows, cap=cap, lr=0.0)
        for rnd in range(2):
            lp1.run(1, rnd, stream_handle(cuda))
            alone = _deltas(lp1, 1, spec, cuda)[0]
            assert torch.equal(alone, multi[rnd][l]), (rnd, l, (alone - multi[rnd][l]).abs().max().item())


@pytest.mark.parametrize("c", [0, 10])
def test_engine_long_window_runs_on_lanes(cuda, c):
    """-max 4096 with several workers: BSP on the one-launch lanes loop, SSP on the
    asynchronous lanes loop (no fallback to the per-worker stream schedulers)."""
    train, test = synth_finefood(40000, seed=0), synth_finefood(2000, seed=1)
    cfg = PSConfig(num_workers=4, consistency_model=c, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=1024, epochs=100, max_iters=8, min_buffer_size=128, max_buffer_size=4096,
                   init="random")
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    out = eng.run()
    if c == 0:
        assert out.get("lanes") == 4 and out["rounds"] == 8, out
    else:
        assert out.get("async_lanes"), out
    assert len(eng.log.book.server) >= 8
    loss = eng.workers[0].solver.loss.item()
    assert loss == loss and loss > 0
