"""Numerics of the HIP kernels against plain PyTorch fp32/fp64 references (MI355X)."""
import numpy as np
import pytest
import torch

from psx import _native
from psx.models.logreg import ModelSpec
from psx.models.reference import local_solve_reference
from psx.ops.lr import EvalSet, Fragments, LocalSolveOp, SolverOptions, server_apply, stream_handle
from psx.runtime.buffer import DeviceRing
from psx.utils.data import synth_binary, synth_finefood

pytestmark = pytest.mark.gpu


def _rand_w(spec, seed, scale=0.1):
    g = torch.Generator().manual_seed(seed)
    return spec.pack(torch.randn(spec.K, spec.F, generator=g) * scale, torch.randn(spec.K, generator=g) * scale)


def test_native_hip_loaded(cuda):
    h = _native.hip()
    info = h.device_arch(0)
    assert "gfx950" in info["gcnArchName"], info
    assert _native.hip_loaded_path().endswith(".so")


@pytest.mark.parametrize("F,K,T", [(1024, 6, 4877), (99, 2, 50), (300, 6, 97), (2000, 11, 130)])
def test_logits_match_fp32(cuda, F, K, T):
    spec = ModelSpec(F, K)
    g = torch.Generator().manual_seed(F + K)
    X = torch.zeros(T, spec.Fp)
    X[:, :F] = torch.randn(T, F, generator=g) * 0.05
    Xb = X.to(torch.bfloat16)
    w = _rand_w(spec, 1)
    frag = Fragments(spec, cuda)
    wd = w.to(cuda)
    frag.refresh(wd)
    out = torch.zeros(T, K, device=cuda)
    Xd = Xb.to(cuda)
    _native.hip().logits(spec.Fp, K, Xd.data_ptr(), T, frag.hi.data_ptr(), frag.lo.data_ptr(), frag.b.data_ptr(),
                         out.data_ptr(), stream_handle(cuda))
    ref = Xb[:, :F].double() @ spec.coef(w).double().t() + spec.intercept(w).double()
    err = (out.cpu().double() - ref).abs().max().item()
    assert err < 2e-5 * max(1.0, ref.abs().max().item()), err


def _ring_with(ds, cap, start, B, device):
    ring = DeviceRing(cap, ds.Fp, device)
    ring.place(ds.X[:B], ds.y[:B], start)
    return ring


@pytest.mark.parametrize(
    "mode,iters,B,start,F",
    [("lbfgs", 2, 700, 900, 1024), ("lbfgs", 6, 1024, 0, 1024), ("gd", 3, 333, 10, 1024), ("lbfgs", 2, 50, 0, 99),
     ("lbfgs", 2, 1024, 1000, 1024)],  # full wrapped window: its first ring tile is visited twice
)
@pytest.mark.parametrize("persist", [False, True])  # launch chain / one persistent launch
def test_local_solve_matches_reference(cuda, mode, iters, B, start, F, persist):
    cap = 1024
    if F == 99:
        ds = synth_binary(B, F, seed=3)
        spec = ModelSpec(F, 2)
    else:
        ds = synth_finefood(B, F, seed=4)
        spec = ModelSpec(F, 6)
    ring = _ring_with(ds, cap, start, B, cuda)
    w_old = _rand_w(spec, 7, scale=0.05)
    opts = SolverOptions(iters=iters, mode=mode, gd_lr=0.5, ls_max=6, persist=persist)
    op = LocalSolveOp(spec, cap, cuda, opts)
    wd = w_old.to(cuda)
    op.run(ring, B, start, wd)
    torch.cuda.synchronize()
    assert bool(op._native.persistent) == persist
    ref = local_solve_reference(ds.float_features(), ds.y.long(), spec.coef(w_old), spec.intercept(w_old),
                                iters=iters, hist=opts.hist, ls_max=opts.ls_max, nslots=opts.nslots, mode=mode,
                                gd_lr=opts.gd_lr)
    delta = op.delta.cpu()
    dc, db = spec.coef(delta), spec.intercept(delta)
    scale = max(ref.delta_coef.abs().max().item(), 1e-6)
    err = (dc - ref.delta_coef).abs().max().item() / scale
    errb = (db - ref.delta_intercept).abs().max().item() / max(ref.delta_intercept.abs().max().item(), 1e-6)
    stats = op.stats.cpu().tolist()
    assert abs(op.loss.item() - ref.loss) < 1e-3 * max(1.0, abs(ref.loss)), (op.loss.item(), ref.loss, stats)
    assert err < 2e-2 and errb < 2e-2, (err, errb, stats, ref.evals, ref.accepted)
    assert stats[1] == ref.accepted, (stats, ref.accepted)


@pytest.mark.parametrize("seed,iters", [(4, 2), (5, 6)])
@pytest.mark.parametrize("persist", [False, True])
def test_line_search_retries_run_in_tail(cuda, seed, iters, persist):
    """Large initial weights make some line searches need several evaluations:
    those run in the persistent tail launch and must match the reference."""
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(512, 1024, seed=seed)
    g = torch.Generator().manual_seed(seed + 100)
    w_old = torch.randn(spec.P, generator=g) * 8.0
    opts = SolverOptions(iters=iters, ls_max=6, persist=persist)
    ring = _ring_with(ds, 1024, 37, 512, cuda)
    op = LocalSolveOp(spec, 1024, cuda, opts)
    op.run(ring, 512, 37, w_old.to(cuda))
    torch.cuda.synchronize()
    ref = local_solve_reference(ds.float_features(), ds.y.long(), spec.coef(w_old), spec.intercept(w_old),
                                iters=iters, hist=opts.hist, ls_max=opts.ls_max, nslots=opts.nslots)
    stats = op.stats.cpu().tolist()
    assert ref.evals > ref.accepted + 1  # the case really exercises retries
    assert stats[0] == ref.evals and stats[1] == ref.accepted, (stats, ref.evals, ref.accepted)
    assert abs(op.loss.item() - ref.loss) < 1e-3 * max(1.0, abs(ref.loss)), (op.loss.item(), ref.loss)
    delta = op.delta.cpu()
    scale = max(ref.delta_coef.abs().max().item(), 1e-6)
    assert (spec.coef(delta) - ref.delta_coef).abs().max().item() / scale < 2e-2


def test_persistent_consecutive_solves_with_many_slots(cuda):
    """nslots = 37 (> 32) with forced line-search retries, two solves in a row on
    one op: the second equals the same solve on a fresh op bitwise (the barrier
    words and the all-gather tags of consecutive solves never alias)."""
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(512, 1024, seed=5)
    g = torch.Generator().manual_seed(105)
    w1 = (torch.randn(spec.P, generator=g) * 8.0).to(cuda)
    w2 = (torch.randn(spec.P, generator=g) * 8.0).to(cuda)
    opts = SolverOptions(iters=6, ls_max=6, persist=True)
    assert opts.nslots > 32
    ring = _ring_with(ds, 1024, 37, 512, cuda)
    op = LocalSolveOp(spec, 1024, cuda, opts)
    # (w1 is test_line_search_retries_run_in_tail's seed-5 start: its solve retries)
    op.run(ring, 512, 37, w2)
    op.run(ring, 512, 37, w1)
    fresh = LocalSolveOp(spec, 1024, cuda, opts)
    fresh.run(ring, 512, 37, w1)
    torch.cuda.synchronize()
    assert bool(op._native.persistent)
    assert op.stats.cpu().tolist()[0] > op.stats.cpu().tolist()[1] + 1  # retries happened
    assert torch.equal(op.delta, fresh.delta) and op.loss.item() == fresh.loss.item()


def test_graph_and_eager_agree(cuda):
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(512, seed=5)
    ring = _ring_with(ds, 1024, 100, 512, cuda)
    w = _rand_w(spec, 2, 0.02).to(cuda)
    outs = []
    for g in (True, False):
        op = LocalSolveOp(spec, 1024, cuda, SolverOptions(use_graph=g))
        for _ in range(3):  # replays must be identical
            op.run(ring, 512, 100, w)
        torch.cuda.synchronize()
        outs.append(op.delta.clone())
    # the gradient sums use fp32 atomics (arrival order varies), so replays agree
    # to rounding, not bitwise
    scale = outs[0].abs().max().item()
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-4 * scale


def test_confusion_matches_cpu(cuda):
    spec = ModelSpec(1024, 6)
    te = synth_finefood(4877, seed=9)
    w = _rand_w(spec, 3, 0.5)
    gpu = EvalSet(spec, te.X, te.y, cuda)
    cpu = EvalSet(spec, te.X, te.y, "cpu")
    frag = Fragments(spec, cuda)
    wd = w.to(cuda)
    frag.refresh(wd)
    cg = torch.zeros(256, dtype=torch.int32, device=cuda)
    cc = torch.zeros(256, dtype=torch.int32)
    gpu.confusion_async(frag, wd, cg)
    cpu.confusion_async(None, w, cc)
    torch.cuda.synchronize()
    diff = (cg.cpu() - cc).abs().sum().item()
    assert cg.sum().item() == 4877
    assert diff <= 4, diff  # argmax ties at bf16/fp32 boundaries


def test_eval_to_pinned_slot(cuda):
    """The slot path (kernel writes counts + loss into pinned host memory and
    publishes a sequence number) matches the CPU confusion, repeatedly (the
    private accumulator must come back to zero after each call)."""
    from psx.ops.lr import EvalScratch
    from psx.utils.logsink import LogSink

    spec = ModelSpec(1024, 6)
    te = synth_finefood(4877, seed=9)
    gpu = EvalSet(spec, te.X, te.y, cuda)
    cpu = EvalSet(spec, te.X, te.y, "cpu")
    log = LogSink(spec.K, cuda, pool=4)
    scratch = EvalScratch(cuda)
    frag = Fragments(spec, cuda)
    rows = []
    for seed in (3, 4, 5):
        w = _rand_w(spec, seed, 0.5)
        wd = w.to(cuda)
        frag.refresh(wd)
        loss = torch.tensor([float(seed)], device=cuda)
        log.worker_eval(gpu, frag, wd, scratch, loss, 0, seed, 0)
        cc = torch.zeros(256, dtype=torch.int32)
        cpu.confusion_async(None, w, cc)
        rows.append(cc)
    book = log.book
    log.close()
    from psx.utils.metrics import metrics_from_confusion

    for r, cc in zip(book.worker, rows):
        f1, acc = metrics_from_confusion(cc.view(16, 16)[:6, :6].numpy())
        assert abs(r[5] - acc) <= 4 / 4877 and r[3] == float(r[2])
    assert scratch.acc.abs().sum().item() == 0 and scratch.ticket.abs().sum().item() == 0


def test_server_apply(cuda):
    spec = ModelSpec(1024, 6)
    w = _rand_w(spec, 4).to(cuda)
    d = _rand_w(spec, 5).to(cuda)
    ref = w + 0.25 * d
    frag = Fragments(spec, cuda)
    server_apply(spec, w, d, 0.25, frag)
    torch.cuda.synchronize()
    assert torch.allclose(w, ref, atol=1e-6)
    assert torch.allclose(frag.b[: spec.K], spec.intercept(ref), atol=1e-6)


def test_ring_ingest_strided_wrap(cuda):
    ds = synth_finefood(300, seed=6).to(cuda)
    ring = DeviceRing(64, ds.Fp, cuda)
    ring.ingest(ds.X, ds.y, 3, 4, 50, 40)  # rows 3,7,...  into slots 40..63,0..25
    torch.cuda.synchronize()
    src = torch.arange(50) * 4 + 3
    dst = (torch.arange(50) + 40) % 64
    assert torch.equal(ring.X.cpu()[dst], ds.X.cpu()[src])
    assert torch.equal(ring.y.cpu()[dst], ds.y.cpu()[src])
    assert torch.equal(ring.XT.cpu(), ring.X.cpu().t())


def test_paired_eval_matches_single(cuda):
    """Two models in one fragment buffer (columns [0,K) and [16-K,16)) evaluated in
    one pass give exactly the confusion counts of two separate passes."""
    from psx.ops.lr import EvalScratch
    from psx.utils.logsink import LogSink

    spec = ModelSpec(1024, 6)
    te = synth_finefood(4877, seed=11)
    ev = EvalSet(spec, te.X, te.y, cuda)
    wa, wb = _rand_w(spec, 21, 0.5).to(cuda), _rand_w(spec, 22, 0.5).to(cuda)
    shared_b = Fragments(spec, cuda, coff=16 - spec.K)
    shared_a = Fragments(spec, cuda, coff=0, share=shared_b)
    shared_a.refresh(wa)
    shared_b.refresh(wb)
    fa, fb = Fragments(spec, cuda), Fragments(spec, cuda)
    fa.refresh(wa)
    fb.refresh(wb)
    log = LogSink(spec.K, cuda)
    scratch = EvalScratch(cuda)
    loss = torch.tensor([1.5], device=cuda)
    log.pair_eval(ev, shared_a, wa, loss, 0, 7, 100, shared_b, wb, 6, 1234, scratch)
    log.worker_eval(ev, fa, wa, scratch, loss, 0, 7, 100)
    log.server_eval(ev, fb, wb, scratch, 6, ts=1234)
    book = log.book
    log.close()
    (wr1, wr2), (sr1, sr2) = book.worker, book.server
    assert wr1[1:] == wr2[1:] and sr1 == sr2 and sr1[0] == 1234
    assert scratch.acc.abs().sum().item() == 0


@pytest.mark.parametrize("ndeltas,server_row", [(1, True), (3, True), (1, False)])
def test_eval_apply_fused(cuda, ndeltas, server_row):
    """Worker row + previous server row + the server update in ONE launch: rows
    exactly those of separate evaluations, update == server_apply_n, and the new
    fragments land in the other buffer (the one read stays untouched)."""
    from psx.ops.lr import EvalScratch
    from psx.utils.logsink import LogSink

    spec = ModelSpec(1024, 6)
    te = synth_finefood(4877, seed=12)
    ev = EvalSet(spec, te.X, te.y, cuda)
    wa, ws = _rand_w(spec, 23, 0.5).to(cuda), _rand_w(spec, 24, 0.5).to(cuda)
    deltas = [_rand_w(spec, 50 + i, 0.2).to(cuda) for i in range(ndeltas)]
    fa = Fragments(spec, cuda)
    fa.refresh(wa)
    cur, nxt = Fragments(spec, cuda, coff=16 - spec.K), Fragments(spec, cuda, coff=16 - spec.K)
    cur.refresh(ws)
    cur_hi = cur.hi.clone()
    w_srv = ws.clone()
    ref = ws + 0.25 * sum(deltas)
    log = LogSink(spec.K, cuda)
    scratch = EvalScratch(cuda)
    loss = torch.tensor([0.75], device=cuda)
    log.pair_eval(ev, fa, wa, loss, 0, 9, 100, cur, w_srv, 8 if server_row else None, 4321, scratch,
                  apply=(w_srv, deltas, 0.25, nxt))
    fb = Fragments(spec, cuda, coff=16 - spec.K)
    fb.refresh(ws)
    log.worker_eval(ev, fa, wa, scratch, loss, 0, 9, 100)
    if server_row:
        log.server_eval(ev, fb, ws, scratch, 8, ts=4321)
    book = log.book
    log.close()
    torch.cuda.synchronize()
    assert len(book.worker) == 2 and book.worker[0][1:] == book.worker[1][1:]
    if server_row:
        assert len(book.server) == 2 and book.server[0] == book.server[1]
    else:
        assert not book.server
    assert torch.allclose(w_srv, ref, atol=1e-6)
    fr = Fragments(spec, cuda, coff=16 - spec.K)
    fr.refresh(ref)
    assert torch.equal(nxt.hi, fr.hi) and torch.equal(nxt.lo, fr.lo)
    assert torch.allclose(nxt.b[16 - spec.K:], spec.intercept(ref), atol=1e-6)
    assert torch.equal(cur.hi, cur_hi)
    assert scratch.acc.abs().sum().item() == 0


def test_server_apply_n_matches_sum(cuda):
    from psx import _native
    from psx.ops.lr import stream_handle

    spec = ModelSpec(1024, 6)
    w = _rand_w(spec, 31).to(cuda)
    deltas = [_rand_w(spec, 40 + i, 0.1).to(cuda) for i in range(5)]
    ref = w + 0.2 * sum(deltas)
    frag = Fragments(spec, cuda, coff=3)
    _native.hip().server_apply_n(spec.K, spec.F, spec.Fp, w.data_ptr(), [d.data_ptr() for d in deltas], 0.2,
                                 frag.hi.data_ptr(), frag.lo.data_ptr(), frag.b.data_ptr(), stream_handle(cuda), 3)
    torch.cuda.synchronize()
    assert torch.allclose(w, ref, atol=1e-6)
    assert torch.allclose(frag.b[3:3 + spec.K], spec.intercept(ref), atol=1e-6)


@pytest.mark.parametrize("graph", [True, False])
@pytest.mark.parametrize("n,B,pre", [(64, 512, 900), (200, 128, 300), (256, 1024, 1000), (1, 1, 0)])
def test_fused_ingest_matches_separate(cuda, graph, n, B, pre):
    """Rows ingested by the solve's first kernel == a separate ring_ingest + solve
    (ring contents bitwise, delta to fp32-atomic rounding); covers ring wrap and
    windows shorter than the ingest."""
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(4000, seed=7).to(cuda)
    w = _rand_w(spec, 3, 0.02).to(cuda)
    cap = 1024
    dst = (pre + 37) % cap  # the new rows end the window and wrap the ring
    start = (dst + n - B) % cap
    outs, rings = [], []
    for defer in (True, False):
        ring = DeviceRing(cap, ds.Fp, cuda, defer=defer)
        ring.ingest(ds.X, ds.y, 0, 1, min(cap, pre + 37), 0)  # older rows, launched on their own
        ring.flush()
        ring.ingest(ds.X, ds.y, 2000, 3, n, dst)
        assert (ring.pending is not None) == defer
        op = LocalSolveOp(spec, cap, cuda, SolverOptions(use_graph=graph))
        op.run(ring, B, start, w)
        assert ring.pending is None
        torch.cuda.synchronize()
        outs.append(op.delta.clone())
        rings.append((ring.X.cpu(), ring.XT.cpu(), ring.y.cpu()))
    for a, b in zip(*rings):
        assert torch.equal(a, b)
    assert torch.equal(rings[0][1], rings[0][0].t())
    scale = outs[1].abs().max().item()
    assert (outs[0] - outs[1]).abs().max().item() <= 2e-4 * scale


def test_deferred_ingest_not_ending_window_is_flushed(cuda):
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(1000, seed=8).to(cuda)
    ring = DeviceRing(256, ds.Fp, cuda, defer=True)
    ring.ingest(ds.X, ds.y, 0, 1, 64, 0)
    op = LocalSolveOp(spec, 256, cuda, SolverOptions())
    op.run(ring, 32, 0, torch.zeros(spec.P, device=cuda))  # window [0,32) does not end at slot 63
    torch.cuda.synchronize()
    assert ring.pending is None and torch.equal(ring.X.cpu()[:64], ds.X.cpu()[:64])


@pytest.mark.parametrize("n,B,pre", [(64, 512, 900), (200, 128, 300), (256, 1024, 1000), (1, 1, 0)])
def test_persistent_solve_matches_chain(cuda, n, B, pre):
    """The one-launch persistent solve (tile-resident, sc1 hand-offs) == the launch
    chain: same ring contents after the fused ingest (bitwise), same solve up to
    summation order; repeated runs are bitwise reproducible."""
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(4000, seed=7).to(cuda)
    w = _rand_w(spec, 3, 0.02).to(cuda)
    cap = 1024
    dst = (pre + 37) % cap
    start = (dst + n - B) % cap
    outs, rings, stats = [], [], []
    for persist in (True, False):
        ring = DeviceRing(cap, ds.Fp, cuda, defer=True)
        ring.ingest(ds.X, ds.y, 0, 1, min(cap, pre + 37), 0)
        ring.flush()
        ring.ingest(ds.X, ds.y, 2000, 3, n, dst)
        op = LocalSolveOp(spec, cap, cuda, SolverOptions(use_graph=False, persist=persist))
        op.run(ring, B, start, w)
        torch.cuda.synchronize()
        assert bool(op._native.persistent) == persist
        outs.append((op.delta.clone(), op.loss.item()))
        stats.append(op.stats.cpu().tolist())
        rings.append((ring.X.cpu(), ring.XT.cpu(), ring.y.cpu()))
        if persist:  # replays: bitwise identical
            for _ in range(3):
                op.run(ring, B, start, w)
            torch.cuda.synchronize()
            assert torch.equal(op.delta, outs[0][0])
    for a, b in zip(*rings):
        assert torch.equal(a, b)
    assert stats[0][:4] == stats[1][:4] and stats[0][4] == 0, stats
    scale = outs[1][0].abs().max().item()
    assert (outs[0][0] - outs[1][0]).abs().max().item() <= 2e-3 * scale
    assert abs(outs[0][1] - outs[1][1]) <= 1e-4 * max(1.0, abs(outs[1][1]))


@pytest.mark.parametrize("ls_max,iters", [(4, 2), (1, 3), (4, 1)])
def test_inplace_finalisation_matches_tail(cuda, monkeypatch, ls_max, iters):
    """The bwd_update launch that ends the solve finalises its feature slice in
    place (PSX_FIN_INPLACE, default on); the tail launch then writes only the
    scalars.  Bitwise the same delta, loss, model fragments and statistics as the
    tail's finalisation -- also when the line search needs the tail's extra slots
    (ls_max 1 / several iterations exercise both exits)."""
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(2048, seed=21).to(cuda)
    cap = 1024
    outs = []
    for fin in ("1", "0"):
        monkeypatch.setenv("PSX_FIN_INPLACE", fin)
        ring = DeviceRing(cap, ds.Fp, cuda)
        ring.place(ds.X[:cap], ds.y[:cap])
        runs = []
        for seed, sc in ((3, 0.05), (4, 0.05), (5, 8.0)):  # large weights: line-search retries in the tail
            w = _rand_w(spec, seed, sc).to(cuda)
            op = LocalSolveOp(spec, cap, cuda, SolverOptions(use_graph=False, iters=iters, ls_max=ls_max))
            op.run(ring, cap, 0, w)
            torch.cuda.synchronize()
            runs.append((op.delta.clone(), op.loss.item(), op.stats.cpu().tolist(), op.frag.hi.clone(),
                         op.frag.lo.clone(), op.frag.b.clone()))
        outs.append(runs)
    for a, b in zip(*outs):
        assert torch.equal(a[0], b[0])
        assert a[1] == b[1] and a[2] == b[2] and a[2][4] == 0
        assert torch.equal(a[3], b[3]) and torch.equal(a[4], b[4]) and torch.equal(a[5], b[5])


@pytest.mark.parametrize("B,start", [(1024, 0), (700, 96), (1020, 40)])  # (1020, 40): 33 tiles -> spread form
def test_solve_placement_variants_agree(cuda, B, start):
    """Where the cooperating workgroups run must not change the result: the
    persistent solve on XCD 0, on XCD 3 and spread over the XCDs (xcd = -1), and
    the chain with its backward slices on one XCD or spread, are each bitwise
    identical (fixed-order reductions everywhere); persistent vs chain agree up to
    summation order.  Placement: blockIdx % 8 == XCD (tools/xcd_probe.hip)."""
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(B, seed=11)
    cap = 1024
    ring = _ring_with(ds, cap, start, B, cuda)
    w = _rand_w(spec, 5, 0.03).to(cuda)
    outs = {}
    for persist in (True, False):
        for xcd in (0, 3, -1):
            op = LocalSolveOp(spec, cap, cuda, SolverOptions(use_graph=False, persist=persist, xcd=xcd))
            for _ in range(2):  # a replay on the same solver as well
                op.run(ring, B, start, w)
            torch.cuda.synchronize()
            assert bool(op._native.persistent) == persist
            assert op.barrier_errors() == 0
            outs[(persist, xcd)] = (op.delta.clone(), op.loss.item())
    for persist in (True, False):
        ref = outs[(persist, 0)]
        for xcd in (3, -1):
            assert torch.equal(outs[(persist, xcd)][0], ref[0]), (persist, xcd)
            assert outs[(persist, xcd)][1] == ref[1]
    a, b = outs[(True, 0)][0], outs[(False, 0)][0]
    assert (a - b).abs().max().item() <= 2e-3 * b.abs().max().item()
