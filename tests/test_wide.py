"""Wide / sparse logistic-regression path (BASELINE.json configs 4 and 5).

CPU tests pin the oracle path (subspace solve == dense solve on the densified
window, sparse delta <-> dense delta, server apply, evaluation); GPU tests
compare the HIP kernels (csrc/kernels/wide_kernels.hip) against it.
"""
import math

import pytest
import torch

from psx.models.reference import local_solve_reference
from psx.models.wide import WideSpec
from psx.ops.lr import EvalScratch, SolverOptions
from psx.ops.sparse import (SparseDelta, SparseRing, WideEvalSet, WideSolveOp, nz_capacity, wide_logits,
                            wide_server_apply)
from psx.utils.data import load_libsvm, save_libsvm, synth_sparse


def _problem(F=3000, rows=400, labels="finefood", seed=0):
    ds = synth_sparse(rows, num_features=F, labels=labels, nnz_mean=20, max_nnz=48, seed=seed, vocab=4 * F,
                      class_vocab=200, signal=0.3)
    K = 1 if labels == "binary" else 6
    return ds, WideSpec(F, K)


def _fill_ring(ds, cap, NZ, device, start=0, n=None):
    ring = SparseRing(cap, NZ, device)
    n = ds.rows if n is None else n
    ring.ingest_from(ds.to(device), 0, 1, n, start)
    return ring


def test_synth_sparse_shape_and_norm():
    ds, spec = _problem()
    assert ds.rows == 400 and ds.indptr[-1] == ds.nnz
    assert int(ds.idx.min()) >= 0 and int(ds.idx.max()) < spec.F
    rows = ds.dense(range(5))
    assert torch.allclose(rows.norm(dim=1), torch.ones(5), atol=2e-2)
    assert set(ds.y.tolist()) <= {1, 2, 3, 4, 5}
    b, _ = _problem(labels="binary")
    assert set(b.y.tolist()) <= {0, 1}


def test_libsvm_roundtrip(tmp_path):
    ds, spec = _problem(rows=50)
    p = str(tmp_path / "d.svm")
    save_libsvm(ds, p)
    back = load_libsvm(p, num_features=spec.F)
    assert torch.equal(back.indptr, ds.indptr) and torch.equal(back.idx, ds.idx)
    assert torch.equal(back.val.view(torch.int16), ds.val.view(torch.int16)) and torch.equal(back.y, ds.y)


def test_libsvm_parser_edge_cases(tmp_path):
    p = tmp_path / "e.svm"
    p.write_text("# header comment\n3 1:0.5 7:-2 # trailing comment\n\n1\n  5 2:0 4:1e-1\r\n2 3:1.5")
    ds = load_libsvm(str(p))
    assert ds.y.tolist() == [3, 1, 5, 2] and ds.num_features == 7
    assert ds.indptr.tolist() == [0, 2, 2, 3, 4]  # empty row kept, explicit zero dropped
    assert ds.idx.tolist() == [0, 6, 3, 2]  # 1-based on disk
    assert torch.allclose(ds.val.float(), torch.tensor([0.5, -2.0, 0.1, 1.5]), atol=1e-3)
    z = load_libsvm(str(p), zero_based=True)
    assert z.idx.tolist() == [1, 7, 4, 3] and z.num_features == 8
    with pytest.raises(ValueError):
        load_libsvm(str(p), num_features=4)
    bad = tmp_path / "bad.svm"
    for body in ("1 3:x\n", "a 1:1\n", "1 0:1\n", "1 3\n"):
        bad.write_text(body)
        with pytest.raises(RuntimeError):
            load_libsvm(str(bad))


def test_nz_capacity():
    assert nz_capacity(3) == 8 and nz_capacity(48) == 48 and nz_capacity(49) == 56
    with pytest.raises(ValueError):
        nz_capacity(513)


def test_ring_wraps_and_truncates():
    ds, _ = _problem(rows=30)
    ring = SparseRing(16, 8, "cpu")
    ring.ingest_from(ds, 0, 1, 30, 5)  # wraps; rows longer than 8 entries are cut
    assert int(ring.trunc) == int(((ds.indptr[1:] - ds.indptr[:-1]) > 8).sum())
    # slot (5 + 29) % 16 = 2 holds row 29
    a = int(ds.indptr[29])
    k = int(ring.nnz[2])
    assert torch.equal(ring.idx[2, :k], ds.idx[a:a + k]) and int(ring.y[2]) == int(ds.y[29])


@pytest.mark.parametrize("labels", ["finefood", "binary"])
def test_cpu_subspace_solve_matches_dense_solve(labels):
    """The wide op solves in the window's feature subspace; on the full feature
    space the reference gives the same coefficients for the touched features."""
    ds, spec = _problem(F=400, rows=120, labels=labels)
    opts = SolverOptions(standardize=False, zero_const=False)
    ring = _fill_ring(ds, 128, 48, "cpu")
    g = torch.Generator().manual_seed(1)
    w_old = spec.init("random", seed=3)
    op = WideSolveOp(spec, 128, 48, "cpu", opts, dense_delta=True)
    op.run(ring, 120, 0, w_old)
    # dense oracle on all F features (untouched ones have zero gradient)
    X = ds.dense().double()
    coef = spec.coef(w_old).double()
    b = spec.intercept(w_old).double()
    res = local_solve_reference(X, ds.y.long(), coef, b, standardize=False, zero_const=False)
    dense = spec.pack(res.delta_coef, res.delta_intercept)
    touched = torch.zeros(spec.F, dtype=torch.bool)
    touched[ds.idx.long()] = True
    mask = torch.zeros(spec.P, dtype=torch.bool)
    mask[: spec.F * spec.KP].view(spec.F, spec.KP)[touched] = True
    mask[spec.F * spec.KP:] = True
    if spec.K >= 2:  # centring also moves the untouched features' coefficients in the dense solve
        assert torch.allclose(op.delta[mask], dense[mask], atol=1e-4), (op.delta - dense).abs().max()
    else:
        assert torch.allclose(op.delta, dense, atol=1e-5), (op.delta - dense).abs().max()
    assert math.isclose(float(op.loss), res.loss, rel_tol=1e-5)
    del g


def test_sparse_delta_and_server_apply_cpu():
    ds, spec = _problem(F=500, rows=64)
    ring = _fill_ring(ds, 64, 48, "cpu")
    op = WideSolveOp(spec, 64, 48, "cpu", SolverOptions(), dense_delta=True)
    w = spec.init("random", seed=1)
    op.run(ring, 64, 0, w)
    sd = op.sparse_delta()
    assert torch.allclose(sd.to_dense(), op.delta)
    w1 = w.clone()
    wide_server_apply(spec, w1, sd, 0.5)
    w2 = w.clone()
    wide_server_apply(spec, w2, op.delta, 0.5)
    assert torch.allclose(w1, w2)


def test_eval_cpu_matches_manual():
    ds, spec = _problem(F=300, rows=200)
    ev = WideEvalSet(spec, ds, "cpu")
    w = spec.init("random", seed=2, scale=1.0)
    z = ds.dense() @ spec.coef(w).t() + spec.intercept(w)
    pred = z.argmax(1)
    conf = ev.confusion_cpu(w).view(16, 16)
    for t, p in zip(ds.y.tolist()[:50], pred.tolist()[:50]):
        assert conf[t, p] > 0
    assert int(conf.sum()) == ds.rows


# ---------------------------------------------------------------------------
# GPU: HIP kernels vs the CPU oracle
def _gpu_vs_cpu(cuda, labels, opts, F=3000, rows=300, cap=320, start=250):
    ds, spec = _problem(F=F, rows=rows, labels=labels)
    NZ = nz_capacity(ds.max_nnz)
    w = spec.init("random", seed=5, scale=0.05)
    out = {}
    for dev in ("cpu", cuda):
        ring = _fill_ring(ds, cap, NZ, dev, start=start)
        op = WideSolveOp(spec, cap, NZ, dev, opts, dense_delta=True)
        op.run(ring, rows, start, w.to(dev))
        if dev != "cpu":
            torch.cuda.synchronize()
            assert op.host_count() == int(torch.unique(ds.idx).numel())
        out[dev] = (op.delta.cpu(), float(op.loss), op.stats.cpu().tolist(), op)
    (dc, lc, sc, _), (dg, lg, sg, opg) = out["cpu"], out[cuda]
    assert sc[0] == sg[0] and sc[1] == sg[1], (sc, sg)  # evaluations and accepted steps
    assert math.isclose(lc, lg, rel_tol=1e-4), (lc, lg)
    scale = dc.abs().max().item()
    assert (dc - dg).abs().max().item() <= 2e-3 * scale + 1e-6, ((dc - dg).abs().max().item(), scale)
    return spec, ds, opg, w


@pytest.mark.gpu
@pytest.mark.parametrize("labels,std", [("finefood", True), ("finefood", False), ("binary", True), ("binary", False)])
def test_gpu_wide_solve_matches_oracle(cuda, labels, std):
    _gpu_vs_cpu(cuda, labels, SolverOptions(standardize=std, zero_const=False))


@pytest.mark.gpu
def test_gpu_wide_solve_gd_and_no_graph(cuda):
    _gpu_vs_cpu(cuda, "finefood", SolverOptions(mode="gd", gd_lr=0.5, use_graph=False))


@pytest.mark.gpu
def test_gpu_wide_solve_repeated_windows(cuda):
    """Back-to-back solves reuse the feature map (reset by the next solve's first kernel)."""
    ds, spec = _problem(F=2000, rows=600)
    NZ = nz_capacity(ds.max_nnz)
    cap = 256
    opts = SolverOptions(zero_const=False)
    gring, cring = SparseRing(cap, NZ, cuda), SparseRing(cap, NZ, "cpu")
    gop = WideSolveOp(spec, cap, NZ, cuda, opts, dense_delta=True)
    cop = WideSolveOp(spec, cap, NZ, "cpu", opts, dense_delta=True)
    w = spec.init("random", seed=9, scale=0.05)
    wg = w.to(cuda)
    dsg = ds.to(cuda)
    for it in range(4):
        first = it * 100
        gring.ingest_from(dsg, first, 1, 200, first % cap)
        cring.ingest_from(ds, first, 1, 200, first % cap)
        gop.run(gring, 200, first % cap, wg)
        cop.run(cring, 200, first % cap, w)
        wide_server_apply(spec, wg, gop.sparse_delta(), 0.5)
        wide_server_apply(spec, w, cop.delta, 0.5)
    torch.cuda.synchronize()
    assert (wg.cpu() - w).abs().max().item() < 2e-3 * w.abs().max().item()


@pytest.mark.gpu
def test_gpu_wide_eval_and_logits(cuda):
    from psx.utils.logsink import LogSink

    ds, spec = _problem(F=1000, rows=500)
    w = spec.init("random", seed=4, scale=1.0)
    zc = wide_logits(spec, ds, w)
    zg = wide_logits(spec, ds.to(cuda), w.to(cuda)).cpu()
    assert torch.allclose(zc, zg, atol=1e-4)
    ev_c, ev_g = WideEvalSet(spec, ds, "cpu"), WideEvalSet(spec, ds, cuda)
    sinks = []
    for ev, dev in ((ev_c, "cpu"), (ev_g, cuda)):
        log = LogSink(spec.eval_classes, dev)
        log.server_eval(ev, None, w.to(dev), EvalScratch(dev), 0)
        sinks.append(log.book.server[0])
        log.close()
    assert abs(sinks[0][2] - sinks[1][2]) < 1e-9 and abs(sinks[0][3] - sinks[1][3]) < 1e-9


@pytest.mark.gpu
def test_gpu_wide_eval_overlay(cuda):
    """Worker rows evaluate the local model = pulled weights overlaid with the subspace solution."""
    from psx.utils.logsink import LogSink

    spec, ds, opg, w = _gpu_vs_cpu(cuda, "finefood", SolverOptions(zero_const=False))
    ev = WideEvalSet(spec, ds, cuda)
    log = LogSink(spec.eval_classes, cuda)
    log.worker_eval(ev, opg, w.to(cuda), EvalScratch(cuda), opg.loss, 0, 0, 0)
    row = log.book.worker[0]
    log.close()
    ref = WideEvalSet(spec, ds, "cpu").confusion_cpu(w + opg.delta.cpu()).view(16, 16)[:6, :6].double()
    acc = float(ref.trace() / ref.sum())
    assert abs(row[5] - acc) < 2e-3


@pytest.mark.gpu
def test_gpu_wide_paired_eval(cuda):
    """The worker's local model (overlay) and the global model it was trained from,
    evaluated in one pass == two separate passes (exact confusion counts)."""
    from psx.utils.logsink import LogSink

    spec, ds, opg, w = _gpu_vs_cpu(cuda, "finefood", SolverOptions(zero_const=False))
    ev = WideEvalSet(spec, ds, cuda)
    wg = w.to(cuda)
    sc = EvalScratch(cuda)
    log = LogSink(spec.eval_classes, cuda)
    log.pair_eval(ev, opg, wg, opg.loss, 0, 5, 77, None, wg, 4, 999, sc)
    log.worker_eval(ev, opg, wg, sc, opg.loss, 0, 5, 77)
    log.server_eval(ev, None, wg, sc, 4, ts=999)
    book = log.book
    log.close()
    (w1, w2), (s1, s2) = book.worker, book.server
    assert w1[1:] == w2[1:] and s1 == s2 and s1[0] == 999
    assert sc.acc.abs().sum().item() == 0


@pytest.mark.gpu
def test_gpu_sparse_ring_ingest(cuda):
    ds, _ = _problem(rows=100)
    NZ = 16
    rc, rg = SparseRing(64, NZ, "cpu"), SparseRing(64, NZ, cuda)
    rc.ingest_from(ds, 3, 2, 40, 50)
    rg.ingest_from(ds.to(cuda), 3, 2, 40, 50)
    torch.cuda.synchronize()
    assert torch.equal(rc.nnz, rg.nnz.cpu()) and torch.equal(rc.y, rg.y.cpu()) and int(rc.trunc) == int(rg.trunc)
    for s in range(64):
        k = int(rc.nnz[s])
        assert torch.equal(rc.idx[s, :k], rg.idx[s, :k].cpu())


# ---------------------------------------------------------------------------
# engines
def _wide_cfg(N, c, device_iters=6, sigmoid=False):
    from psx.runtime.config import PSConfig

    return PSConfig(num_workers=N, consistency_model=c, producer_time_per_event=0, stream_mode="per_iter",
                    rows_per_iter=64, epochs=50, max_iters=device_iters, min_buffer_size=64, max_buffer_size=256,
                    init="random", sigmoid=sigmoid, solver=SolverOptions(zero_const=False))


@pytest.mark.parametrize("c,N", [(0, 1), (0, 2), (-1, 2), (2, 3)])
def test_engine_wide_cpu(c, N):
    from psx.runtime.engine import LocalEngine

    ds, spec = _problem(F=2000, rows=1200)
    te, _ = _problem(F=2000, rows=300, seed=7)
    eng = LocalEngine(_wide_cfg(N, c), "cpu", train=ds, test=te)
    assert isinstance(eng.spec, WideSpec) and eng.spec.K == 6
    out = eng.run()
    assert out["updates"] >= 6 * N if c == 0 else out["updates"] >= 6
    book = eng.log.book
    assert book.server and book.worker
    if c > 0:
        assert out["max_vc_gap"] <= c


def test_engine_wide_binary_cpu():
    from psx.runtime.engine import LocalEngine

    ds, _ = _problem(F=1500, rows=800, labels="binary")
    te, _ = _problem(F=1500, rows=300, labels="binary", seed=3)
    eng = LocalEngine(_wide_cfg(1, 0, 10, sigmoid=True), "cpu", train=ds, test=te)
    out = eng.run()
    assert eng.spec.K == 1 and out["rounds"] == 10
    assert out["final_server_acc"] > 0.55  # planted signal is learnable


@pytest.mark.gpu
@pytest.mark.parametrize("c,N", [(0, 1), (0, 2), (-1, 2)])
def test_engine_wide_gpu(cuda, c, N):
    from psx.runtime.engine import LocalEngine

    ds, spec = _problem(F=2000, rows=1200)
    te, _ = _problem(F=2000, rows=300, seed=7)
    cfg = _wide_cfg(N, c, 8)
    outs = {}
    for dev in ("cpu", cuda):
        eng = LocalEngine(_wide_cfg(N, c, 8), dev, train=ds, test=te)
        outs[dev] = (eng.run(), eng.server.w.cpu())
    if c == 0:  # BSP is deterministic up to float rounding
        wc, wg = outs["cpu"][1], outs[cuda][1]
        assert (wc - wg).abs().max().item() < 5e-3 * wc.abs().max().item()
    assert outs[cuda][0]["server_rows"] >= 1
    del cfg


def test_wide_lanes_selection_cpu():
    """The one-launch wide rounds are a GPU schedule: CPU engines, one worker, tracing and
    injected faults keep the per-worker schedulers (engine.py _wide_lanes_ok)."""
    from psx.runtime.engine import LocalEngine

    ds, _ = _problem(F=800, rows=400)
    te, _ = _problem(F=800, rows=100, seed=7)
    eng = LocalEngine(_wide_cfg(3, -1, 2), "cpu", train=ds, test=te)
    assert not eng._wide_lanes_ok()
    out = eng.run()
    assert "wide_lanes" not in out and out["updates"] >= 2


def test_ingest_batch_groups_jobs():
    """IngestBatch collects every ring's deliveries of a round (one launch on the GPU);
    a different geometry or dataset starts a new batch."""
    from psx.ops.sparse import IngestBatch

    ds, _ = _problem(F=500, rows=64)
    rings = [SparseRing(32, 48, "cpu") for _ in range(3)]
    b = IngestBatch()
    flushed = []
    b.flush = lambda device: (flushed.append(list(b.jobs)), setattr(b, "jobs", []), setattr(b, "ds", None),
                              setattr(b, "geom", None))
    for i, r in enumerate(rings):
        b.add(r, ds, i, 3, 8, 5)
    assert len(b.jobs) == 3 and b.geom == (32, 48) and not flushed
    assert [j[:4] for j in b.jobs] == [[0, 3, 8, 5], [1, 3, 8, 5], [2, 3, 8, 5]]
    b.add(SparseRing(16, 48, "cpu"), ds, 0, 1, 4, 0)  # another geometry: the open batch goes first
    assert len(flushed) == 1 and len(flushed[0]) == 3 and len(b.jobs) == 1


def _wide_lanes_run(dev, N, c, iters=8, env=None):
    import os

    from psx.runtime.engine import LocalEngine

    ds, spec = _problem(F=2000, rows=1600)
    te, _ = _problem(F=2000, rows=300, seed=7)
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        eng = LocalEngine(_wide_cfg(N, c, iters), dev, train=ds, test=te)
        out = eng.run(close_log=False)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    book = eng.log.book
    eng.log.close()
    return eng, out, book, te


@pytest.mark.gpu
@pytest.mark.parametrize("c,overlay", [(0, "1"), (-1, "1"), (2, "1"), (-1, "0")])
def test_gpu_wide_lanes_match_cpu_rounds(cuda, c, overlay):
    """Several wide workers in ONE solve launch per round (WideLanes, one XCD each):
    every round's solves start from the same server weights and the pushes are applied
    in order, so BSP, SSP and ASP all land on the weights of the CPU engine's BSP rounds
    (whose workers solve with the float64-oracle path, ops/sparse.py _run_cpu).
    overlay "1": the evaluation reads the overlay table and the pushes are applied in
    one launch over it; "0": bitmaps + table probes and one launch per push."""
    N, iters = 4, 8
    eng, out, book, te = _wide_lanes_run(cuda, N, c, iters, env={"PSX_WIDE_EVAL_OVERLAY": overlay,
                                                                   "PSX_WIDE_LANES": "1"})
    assert out.get("wide_lanes") == N, out  # the one-launch path ran
    assert out["updates"] == N * iters
    assert len(book.worker) == N * iters and len(book.server) == iters
    assert all(math.isfinite(r[3]) and r[3] > 0 for r in book.worker), "worker rows carry the solve loss"
    ref, _, _, _ = _wide_lanes_run("cpu", N, 0, iters)
    wc, wg = ref.server.w.cpu(), eng.server.w.cpu()
    assert (wc - wg).abs().max().item() < 5e-3 * wc.abs().max().item()
    # the last server row (the flush pass) evaluates the final global model
    conf = WideEvalSet(ref.spec, te, "cpu").confusion_cpu(wg).view(16, 16)[:6, :6].double()
    assert abs(book.server[-1][3] - float(conf.trace() / conf.sum())) < 2e-3


@pytest.mark.gpu
def test_gpu_wide_lanes_rows_equal_separate_passes(cuda):
    """The multi-model evaluation pass: every worker row equals the worker's local model
    evaluated on its own (the overlay pass of test_gpu_wide_eval_overlay)."""
    from psx.utils.logsink import LogSink

    N = 3
    eng, out, book, te = _wide_lanes_run(cuda, N, -1, 1, env={"PSX_WIDE_LANES": "1"})
    assert out.get("wide_lanes") == N
    # one round from the initial weights: rebuild them and evaluate each local model alone
    w0 = eng.spec.init("random", seed=eng.cfg.seed, device=cuda)
    ev = WideEvalSet(eng.spec, te, cuda)
    log = LogSink(eng.spec.eval_classes, cuda)
    for w in eng.workers:
        log.worker_eval(ev, w.solver, w0, EvalScratch(cuda), w.solver.loss, w.k, 0, 0)
    alone = log.book.worker
    log.close()
    rows = sorted(book.worker, key=lambda r: r[1])
    for a, b in zip(rows, sorted(alone, key=lambda r: r[1])):
        assert a[1] == b[1] and a[3:6] == b[3:6], (a, b)  # partition, loss, F1, accuracy


def test_cli_libsvm_inprocess(tmp_path):
    """ServerAppRunner on LIBSVM files picks the wide model (reference CLI flags + new ones)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tr, _ = _problem(F=4000, rows=600)
    te, _ = _problem(F=4000, rows=100, seed=3)
    save_libsvm(tr, str(tmp_path / "train.svm"))
    save_libsvm(te, str(tmp_path / "test.svm"))
    cmd = [sys.executable, "-m", "psx.apps.server_app_runner", "-training", str(tmp_path / "train.svm"), "-test",
           str(tmp_path / "test.svm"), "--inprocess", "--device", "cpu", "-p", "0", "--num_workers", "2", "-c", "2",
           "--max_iters", "4", "-l", "--log_dir", str(tmp_path / "logs")]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    srows = (tmp_path / "logs" / "logs-server.csv").read_text().strip().split("\n")
    wrows = (tmp_path / "logs" / "logs-worker.csv").read_text().strip().split("\n")
    assert srows[0] == "timestamp;partition;vectorClock;loss;fMeasure;accuracy" and len(srows) >= 4
    assert wrows[0].endswith(";numTuplesSeen") and len(wrows) >= 9


@pytest.mark.gpu
@pytest.mark.parametrize("std", [True, False])
def test_gpu_wide_retry_slots_in_tail(cuda, std):
    """Line searches that need more than one trial run in the persistent tail
    launch (grid barriers); results still match the oracle.  A large initial
    model makes first trial steps fail the Wolfe tests (CPU oracle: 8-9
    evaluations for 4 accepted steps)."""
    ds, spec = _problem(F=2000, rows=300, labels="finefood", seed=4)
    NZ = nz_capacity(ds.max_nnz)
    w = spec.init("random", seed=7, scale=30.0)
    outs = []
    for dev in ("cpu", cuda):
        ring = _fill_ring(ds, 320, NZ, dev)
        op = WideSolveOp(spec, 320, NZ, dev, SolverOptions(zero_const=False, iters=4, standardize=std),
                         dense_delta=True)
        op.run(ring, 300, 0, w.to(dev))
        outs.append((op.delta.cpu(), op.stats.cpu().tolist(), float(op.loss)))
    (dc, sc, lc), (dg, sg, lg) = outs
    assert sc[0] == sg[0] and sc[1] == sg[1], (sc, sg)
    assert sc[0] > 1 + sc[1], sc  # some line search needed a retry (tail slots ran)
    assert math.isclose(lc, lg, rel_tol=1e-3)
    assert (dc - dg).abs().max().item() <= 5e-3 * dc.abs().max().item() + 1e-6
