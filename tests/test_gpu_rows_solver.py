"""Large-window ("rows") local solver on MI355X: every evaluation is ONE
row-parallel pass over the window (fused forward + backward per LDS tile, the
backward operand read transposed with ds_read_b64_tr_b16), partial gradients
reduced in a fixed order.  Checked against the float64 oracle of the
reference's fit (LogisticRegressionTaskSpark.java:179-184), and at 1M rows by
duplication invariance (the mean objective of 16 copies of a 64k window is the
64k window's)."""
import pytest
import torch

from psx import _native
from psx.models.logreg import ModelSpec
from psx.models.reference import local_solve_reference
from psx.ops.lr import LocalSolveOp, SolverOptions
from psx.runtime.buffer import DeviceRing
from psx.utils.data import synth_finefood

pytestmark = pytest.mark.gpu


def _rand_w(spec, seed, scale=0.05):
    g = torch.Generator().manual_seed(seed)
    return spec.pack(torch.randn(spec.K, spec.F, generator=g) * scale, torch.randn(spec.K, generator=g) * scale)


def _check(op, ds, spec, w_old, opts, tol=2e-2):
    ref = local_solve_reference(ds.float_features(), ds.y.long(), spec.coef(w_old), spec.intercept(w_old),
                                iters=opts.iters, hist=opts.hist, ls_max=opts.ls_max, nslots=opts.nslots,
                                mode=opts.mode, gd_lr=opts.gd_lr)
    delta = op.delta.cpu()
    stats = op.stats.cpu().tolist()
    scale = max(ref.delta_coef.abs().max().item(), 1e-6)
    err = (spec.coef(delta) - ref.delta_coef).abs().max().item() / scale
    errb = (spec.intercept(delta) - ref.delta_intercept).abs().max().item() / max(
        ref.delta_intercept.abs().max().item(), 1e-6)
    assert abs(op.loss.item() - ref.loss) < 1e-3 * max(1.0, abs(ref.loss)), (op.loss.item(), ref.loss, stats)
    assert err < tol and errb < tol, (err, errb, stats, ref.evals, ref.accepted)
    assert stats[1] == ref.accepted and stats[4] == 0, (stats, ref.accepted)


@pytest.mark.parametrize("B,start,F,iters", [(700, 900, 1024, 2), (1024, 1000, 1024, 4), (300, 5, 256, 2),
                                             (1024, 0, 2048, 2)])
def test_rows_mode_forced_small_window(cuda, monkeypatch, B, start, F, iters):
    """The rows path on small rings (forced) against the oracle, wrapped windows included."""
    monkeypatch.setenv("PSX_SOLVER_ROWS", "1")
    spec = ModelSpec(F, 6)
    ds = synth_finefood(B, F, seed=11)
    ring = DeviceRing(1024, spec.Fp, cuda)
    assert ring.rows_mode and ring.XT is None
    ring.place(ds.X[:B], ds.y[:B], start)
    opts = SolverOptions(iters=iters, ls_max=6)
    op = LocalSolveOp(spec, ring.cap, cuda, opts)
    w_old = _rand_w(spec, 3)
    op.run(ring, B, start, w_old.to(cuda))
    torch.cuda.synchronize()
    assert op._native.rows_mode
    _check(op, ds, spec, w_old, opts)


def test_rows_mode_64k_window_matches_reference(cuda):
    B = 65536
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(B, seed=12)
    ring = DeviceRing(B, spec.Fp, cuda)
    assert ring.rows_mode  # > kRowsModeMinCap rows: the default for such rings
    ring.place(ds.X, ds.y, 0)
    opts = SolverOptions(iters=2)
    op = LocalSolveOp(spec, ring.cap, cuda, opts)
    w_old = _rand_w(spec, 4)
    op.run(ring, B, 0, w_old.to(cuda))
    torch.cuda.synchronize()
    _check(op, ds, spec, w_old, opts)


def test_rows_mode_1m_window_duplication_invariant(cuda):
    """A 1,048,576-row window holding 16 copies of a 64k window (rotated start,
    so the window wraps the ring) has the same mean objective: its solve must
    match the 64k solve."""
    b, reps = 65536, 16
    spec = ModelSpec(1024, 6)
    ds = synth_finefood(b, seed=13)
    w_old = _rand_w(spec, 5).to(cuda)
    opts = SolverOptions(iters=2)
    small = DeviceRing(b, spec.Fp, cuda)
    small.place(ds.X, ds.y, 0)
    op_s = LocalSolveOp(spec, small.cap, cuda, opts)
    op_s.run(small, b, 0, w_old)
    big = DeviceRing(b * reps + 4096, spec.Fp, cuda)
    start = 7 * 32 + 5
    for r in range(reps):
        big.place(ds.X, ds.y, start + r * b)
    op_b = LocalSolveOp(spec, big.cap, cuda, opts)
    op_b.run(big, b * reps, start, w_old)
    torch.cuda.synchronize()
    ds_, db_ = op_s.delta, op_b.delta
    scale = ds_.abs().max().item()
    # std over n-1 rows differs by (n-1)/(N-1) ~ 1e-5 relative; the rest is rounding
    assert (ds_ - db_).abs().max().item() < 2e-3 * scale, ((ds_ - db_).abs().max().item(), scale)
    assert abs(op_s.loss.item() - op_b.loss.item()) < 1e-4 * abs(op_s.loss.item())
    assert op_b.stats[4].item() == 0


def test_rows_mode_engine_large_buffer(cuda):
    """End to end: a worker with a 32k-row buffer (rows solver) trains through the
    in-process engine and the global model learns."""
    from psx.runtime.config import PSConfig
    from psx.runtime.engine import LocalEngine

    train, test = synth_finefood(40000, seed=0), synth_finefood(2000, seed=1)
    cfg = PSConfig(num_workers=1, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=4096, epochs=100, max_iters=12, min_buffer_size=128, max_buffer_size=32768)
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    out = eng.run()
    assert out["rounds"] == 12
    assert eng.workers[0].ring.rows_mode
    accs = [r[3] for r in eng.log.book.server]
    assert accs[-1] > 0.35, accs
    assert _native.hip_loaded_path() is not None


@pytest.mark.parametrize("B,start,F", [(1024, 1000, 1024), (700, 3, 300), (20000, 77, 1024)])
def test_fp32_rows_match_reference(cuda, B, start, F):
    """--dtype fp32: fp32 ring rows (hi + lo bf16 MFMA operands) against the float64
    oracle on the SAME fp32 rows, tighter than the bf16 path's tolerance."""
    spec = ModelSpec(F, 6)
    ds = synth_finefood(B, F, seed=21, dtype="fp32")
    assert ds.X.dtype == torch.float32
    cap = max(1024, B)
    ring = DeviceRing(cap, spec.Fp, cuda, dtype="fp32")
    assert ring.rows_mode and ring.X.dtype == torch.float32
    ring.place(ds.X[:B], ds.y[:B], start)
    opts = SolverOptions(iters=2)
    op = LocalSolveOp(spec, ring.cap, cuda, opts)
    w_old = _rand_w(spec, 8)
    op.run(ring, B, start, w_old.to(cuda))
    torch.cuda.synchronize()
    assert op._native.rows_mode
    _check(op, ds, spec, w_old, opts, tol=5e-3)


def test_fp32_rows_differ_from_bf16_rows(cuda):
    """The fp32 path really consumes the fp32 bits: on rows that bf16 cannot
    represent its result is closer to the fp32 oracle than the bf16 path's."""
    spec = ModelSpec(1024, 6)
    ds32 = synth_finefood(2048, seed=22, dtype="fp32")
    ds16 = ds32.as_dtype("bf16")
    w_old = _rand_w(spec, 9)
    opts = SolverOptions(iters=2)
    ref = local_solve_reference(ds32.float_features(), ds32.y.long(), spec.coef(w_old), spec.intercept(w_old),
                                iters=2, hist=opts.hist, ls_max=opts.ls_max, nslots=opts.nslots)
    errs = {}
    for name, ds in (("fp32", ds32), ("bf16", ds16)):
        ring = DeviceRing(2048, spec.Fp, cuda, dtype=name)
        ring.place(ds.X, ds.y, 0)
        op = LocalSolveOp(spec, ring.cap, cuda, opts)
        op.run(ring, 2048, 0, w_old.to(cuda))
        torch.cuda.synchronize()
        errs[name] = (spec.coef(op.delta.cpu()) - ref.delta_coef).abs().max().item()
    assert errs["fp32"] < 0.5 * errs["bf16"], errs


def test_fp32_engine_bench_path(cuda):
    from psx.runtime.config import PSConfig
    from psx.runtime.engine import LocalEngine

    train, test = synth_finefood(20000, seed=0, dtype="fp32"), synth_finefood(1000, seed=1)
    cfg = PSConfig(num_workers=1, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=128, epochs=100, max_iters=30, dtype="fp32")
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    out = eng.run()
    assert out["rounds"] == 30 and eng.workers[0].ring.X.dtype == torch.float32
    assert eng.log.book.server[-1][3] > 0.3
