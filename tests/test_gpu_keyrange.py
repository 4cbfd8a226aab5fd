"""Key-range sharded server on one MI355X: the wide solver's pull mode
(csrc/solver/wide_solver.h plan() / finish()) and the native KeyRangeLoop
(csrc/runtime/keyrange_loop.h) at world 1."""
import pytest
import torch

from psx import _native
from psx.models.wide import WideSpec
from psx.ops.lr import SolverOptions, stream_handle
from psx.ops.sparse import SparseRing, WideEvalSet, WideSolveOp, nz_capacity, wide_server_apply
from psx.runtime.buffer import StreamSource
from psx.runtime.config import PSConfig
from psx.utils.data import synth_sparse

pytestmark = pytest.mark.gpu


def _data(F, rows=3000, seed=0):
    kw = dict(num_features=F, labels="binary", nnz_mean=24, max_nnz=48, vocab=50000, class_vocab=400, signal=0.3)
    return synth_sparse(rows, seed=seed, **kw)


def _pulled_solver(spec, ring, own_W, own_S, dev):
    """A pull-mode WideSolver on `ring` with its own output buffers."""
    h = _native.hip()
    o = SolverOptions()
    c = h.WideCfg()
    c.K, c.KP, c.F, c.cap, c.NZ = spec.K, spec.KP, spec.F, ring.cap, ring.NZ
    c.iters, c.hist, c.ls_max, c.nslots, c.mode, c.gd_lr, c.tol = o.iters, o.hist, o.ls_max, o.nslots, 0, o.gd_lr, o.tol
    c.standardize, c.center, c.zero_const = int(o.standardize), int(o.center), int(o.zero_const)
    c.pulled, c.own_W, c.own_S = 1, own_W, own_S
    umax = min(spec.F, ring.cap * ring.NZ)
    pl = spec.KP + umax * spec.KP
    bufs = dict(dloc=torch.zeros(pl, device=dev), wloc=torch.zeros(pl, device=dev),
                loss=torch.zeros(1, device=dev), stats=torch.zeros(8, dtype=torch.int32, device=dev),
                uniq=torch.zeros(umax, dtype=torch.int32, device=dev), w_pull=torch.zeros(umax * spec.KP, device=dev),
                b=torch.zeros(spec.KP, device=dev))
    s = h.WideSolver(c, ring.idx.data_ptr(), ring.val.data_ptr(), ring.nnz.data_ptr(), ring.y.data_ptr(), 0,
                     bufs["dloc"].data_ptr(), bufs["wloc"].data_ptr(), bufs["loss"].data_ptr(),
                     bufs["stats"].data_ptr(), bufs["uniq"].data_ptr(), 0, True, bufs["w_pull"].data_ptr(),
                     bufs["b"].data_ptr())
    return s, bufs


@pytest.mark.parametrize("own_W", [1, 3])
def test_pulled_solve_equals_dense_solve(cuda, own_W):
    """plan -> pull the planned features' weights -> finish == the dense-mode
    solve from the whole vector; with own_W owners the local ids come grouped
    by owner (counts per owner)."""
    F = 200_000
    spec = WideSpec(F, 1)
    ds = _data(F, rows=600)
    w = spec.init("random", seed=5, scale=0.3, device=cuda)
    w[spec.F * spec.KP:] = 0.2
    ring = SparseRing(512, nz_capacity(ds.max_nnz), cuda)
    ring.ingest_from(ds.to(cuda), 0, 1, 512, 0)
    dense = WideSolveOp(spec, ring.cap, ring.NZ, cuda, SolverOptions())
    dense.run(ring, 500, 3, w)
    S = -(-F // own_W)
    s, b = _pulled_solver(spec, ring, own_W, S, cuda)
    st = stream_handle(cuda)
    s.plan(500, 3, st)
    v = s.read_plan(st)
    U = v[0]
    ids = b["uniq"][:U].long()
    if own_W > 1:
        owner = torch.clamp(ids // S, max=own_W - 1)
        assert bool((owner[1:] >= owner[:-1]).all())  # grouped by owner
        assert torch.bincount(owner, minlength=own_W).tolist() == v[1:1 + own_W]
    b["w_pull"][:U] = w[ids]  # the pull (KP = 1)
    b["b"].copy_(w[spec.F:])
    s.finish(st)
    torch.cuda.synchronize()
    assert U == dense.host_count()
    got = torch.zeros(spec.P, device=cuda)
    got[ids] = b["dloc"][1:1 + U]
    got[spec.F:] = b["dloc"][:1]
    ud = dense.host_count()
    ref = torch.zeros(spec.P, device=cuda)
    ref[dense.uniq[:ud].long()] = dense.dloc[1:1 + ud]
    ref[spec.F:] = dense.dloc[:1]
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 1e-4 * scale + 1e-7
    assert abs(b["loss"].item() - dense.loss.item()) <= 1e-5 * abs(dense.loss.item())


def _wide_solver(spec, ring, dev, persist, pulled=0):
    h = _native.hip()
    o = SolverOptions()
    c = h.WideCfg()
    c.K, c.KP, c.F, c.cap, c.NZ = spec.K, spec.KP, spec.F, ring.cap, ring.NZ
    c.iters, c.hist, c.ls_max, c.nslots, c.mode, c.gd_lr, c.tol = o.iters, o.hist, o.ls_max, o.nslots, 0, o.gd_lr, o.tol
    c.standardize, c.center, c.zero_const = int(o.standardize), int(o.center), int(o.zero_const)
    c.persist = int(persist)
    umax = min(spec.F, ring.cap * ring.NZ)
    pl = spec.KP + umax * spec.KP
    bufs = dict(dloc=torch.zeros(pl, device=dev), wloc=torch.zeros(pl, device=dev),
                loss=torch.zeros(1, device=dev), stats=torch.zeros(8, dtype=torch.int32, device=dev),
                uniq=torch.zeros(umax, dtype=torch.int32, device=dev))
    return bufs, c


@pytest.mark.parametrize("K", [1, 6])
def test_persistent_wide_solve_equals_chain(cuda, K):
    """The one-launch persistent wide solve (grid barriers between the phases)
    == the launch chain, over consecutive solves on different windows."""
    F = 300_000
    spec = WideSpec(F, K)
    labels = "binary" if K == 1 else "finefood"
    ds = synth_sparse(1200, num_features=F, labels=labels, nnz_mean=24, max_nnz=48, seed=3, vocab=50000,
                      class_vocab=400, signal=0.3)
    w = spec.init("random", seed=5, scale=0.2, device=cuda)
    ring = SparseRing(1024, nz_capacity(ds.max_nnz), cuda)
    ring.ingest_from(ds.to(cuda), 0, 1, 1024, 0)
    h = _native.hip()
    outs = []
    for persist in (False, True):
        bufs, c = _wide_solver(spec, ring, cuda, persist)
        s = h.WideSolver(c, ring.idx.data_ptr(), ring.val.data_ptr(), ring.nnz.data_ptr(), ring.y.data_ptr(),
                         w.data_ptr(), bufs["dloc"].data_ptr(), bufs["wloc"].data_ptr(), bufs["loss"].data_ptr(),
                         bufs["stats"].data_ptr(), bufs["uniq"].data_ptr(), 0, True)
        assert s.kernels_per_solve == 1 if persist else s.kernels_per_solve > 5
        res = []
        for B, start in ((1000, 5), (700, 300), (1024, 0)):
            s.run(B, start, stream_handle(cuda))
            torch.cuda.synchronize()
            U = s.ucount_host
            dense = torch.zeros(spec.P, device=cuda)
            dense.view(-1)[spec.F * spec.KP:] = bufs["dloc"][:spec.KP]
            dense[: spec.F * spec.KP].view(spec.F, spec.KP)[bufs["uniq"][:U].long()] = \
                bufs["dloc"][spec.KP: spec.KP + U * spec.KP].view(U, spec.KP)
            res.append((dense, bufs["loss"].item(), bufs["stats"][:4].tolist(), int(bufs["stats"][4].item())))
        outs.append(res)
    for (da, la, sa, ea), (db, lb, sb, eb) in zip(*outs):
        assert ea == 0 and eb == 0 and sa == sb
        scale = da.abs().max().item()
        assert (da - db).abs().max().item() <= 1e-4 * scale + 1e-7
        assert abs(la - lb) <= 1e-5 * abs(la)


def _replicated_gpu(spec, train, cfg, rounds, dev):
    """Oracle: one worker, the whole vector, dense-mode solves, w += lr * delta."""
    ring = SparseRing(cfg.max_buffer_size, nz_capacity(train.max_nnz), dev)
    win = _native.host.SlidingWindow(cfg.min_buffer_size, cfg.max_buffer_size, cfg.buffer_size_coefficient, 500,
                                     ring.cap)
    src = StreamSource(train, 0, 1, ring, win, mode="per_iter", rows_per_iter=cfg.rows_per_iter, epochs=cfg.epochs)
    op = WideSolveOp(spec, ring.cap, ring.NZ, dev, cfg.solver)
    w = spec.init(cfg.init, seed=cfg.seed, device=dev)
    for _ in range(rounds):
        src.poll()
        op.run(ring, int(win.size), int(win.start), w)
        wide_server_apply(spec, w, op.sparse_delta(), cfg.lr)
    torch.cuda.synchronize()
    return w


def test_keyrange_world1_matches_replicated_and_logs(cuda):
    from psx.parallel.keyrange import KeyRangeEngine

    F = 2_000_000
    train, test = _data(F, rows=6000), _data(F, rows=800, seed=1)
    cfg = PSConfig(consistency_model=0, producer_time_per_event=0, stream_mode="per_iter", rows_per_iter=128,
                   epochs=100, max_iters=12, min_buffer_size=128, max_buffer_size=512, init="random", model="wide",
                   sigmoid=True, bsp_schedule="keyrange")
    eng = KeyRangeEngine(cfg, 0, 1, cuda, train=train.to(cuda), test=test.to(cuda))
    out = eng.run()
    assert out["rounds"] == 12 and eng.lo == 0 and eng.hi == F
    k = out["keyrange"]
    assert k["weight_bytes"] == (F + 2) * 4 and k["model_bytes"] == 0  # world 1: every exchange is local
    assert 0 < k["last_u"] <= 512 * 48
    ref = _replicated_gpu(eng.spec, train.to(cuda), cfg, 12, cuda)
    got = torch.cat([eng.shard[:F], eng.b])
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 1e-4 * scale, (got - ref).abs().max().item()
    book = eng.log.book
    assert [r[1] for r in book.server] == list(range(12)) and len(book.worker) == 12
    assert all(r[3] > 0 for r in book.worker)  # the solver's loss rides in the worker rows
    conf = WideEvalSet(eng.spec, test, "cpu").confusion_cpu(got.cpu()).view(16, 16)[:2, :2].double()
    assert abs(book.server[-1][3] - float(conf.trace() / conf.sum())) <= 1.0 / 800 + 1e-9


def test_keyrange_worker_row_is_the_local_model(cuda):
    """The worker row (previous margins + the window overlay of the delta +
    the local intercept) == a direct evaluation of pulled weights + delta."""
    from psx.parallel.keyrange import KeyRangeEngine

    F = 300_000
    train, test = _data(F, rows=3000), _data(F, rows=600, seed=1)
    cfg = PSConfig(consistency_model=0, producer_time_per_event=0, stream_mode="per_iter", rows_per_iter=128,
                   epochs=100, max_iters=1, min_buffer_size=128, max_buffer_size=256, init="random", model="wide",
                   sigmoid=True, bsp_schedule="keyrange")
    eng = KeyRangeEngine(cfg, 0, 1, cuda, train=train.to(cuda), test=test.to(cuda))
    w0 = torch.cat([eng.shard[:F], eng.b]).clone()
    eng._run_bsp()
    torch.cuda.synchronize()
    so = eng.solver
    U = eng.last_u
    local = w0.clone()
    ids = so.uniq[:U].long()
    local[ids] += so.dloc[1:1 + U]
    local[F:] += so.dloc[:1]
    conf = WideEvalSet(eng.spec, test, "cpu").confusion_cpu(local.cpu()).view(16, 16)[:2, :2].double()
    row = eng.log.book.worker[0]
    assert row[1] == 0 and row[2] == 0
    assert abs(row[5] - float(conf.trace() / conf.sum())) <= 1.0 / 600 + 1e-9
    eng.log.close()
