"""Native RCCL communicator (csrc/comm/rccl_comm.h) on one MI355X: world size 1
in-process (the multi-rank path runs in the driver's 8-GPU bench; RCCL refuses
two ranks on one device)."""
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture
def pg(cuda):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device(cuda))
    yield
    dist.destroy_process_group()


def test_native_comm_world1(cuda, pg):
    from psx.parallel.comm import make_comm

    comm = make_comm(0, 1, cuda)
    assert comm is not None and comm.c.size == 1 and comm.c.rank == 0
    x = torch.arange(1000, dtype=torch.float32, device=cuda)
    ref = x.clone()
    comm.all_reduce(x)
    comm.reduce(x, 0)
    comm.broadcast(x, 0)
    i = torch.arange(64, dtype=torch.int32, device=cuda)
    comm.all_reduce(i)
    out = torch.empty(1000, dtype=torch.float32, device=cuda)
    comm.reduce_scatter(out, x)
    g = torch.zeros(1000, dtype=torch.float32, device=cuda)
    comm.all_gather(g, out)
    # side stream between fork / join, overlapping compute on the current stream
    y = torch.ones(1 << 20, device=cuda)
    comm.fork()
    comm.all_reduce(y, side=True)
    z = (x * 2).sum()
    comm.join()
    y += 1
    torch.cuda.synchronize()
    assert torch.equal(x, ref) and torch.equal(g, ref) and torch.equal(i.cpu(), torch.arange(64, dtype=torch.int32))
    assert torch.all(y == 2) and z.item() == 2 * ref.sum().item()
    comm.close()


def test_dist_engine_native_vs_torch_collectives(cuda, pg, monkeypatch):
    """The BSP loop gives the same model through the native communicator and through torch.distributed."""
    from psx.parallel.dist import DistEngine
    from psx.runtime.config import PSConfig
    from psx.utils.data import synth_finefood

    train, test = synth_finefood(4000, seed=0), synth_finefood(500, seed=1)
    monkeypatch.setenv("PSX_NATIVE_LANES", "0")  # (one worker per rank: the collectives' own comparison)
    ws = {}
    for native in ("1", "0"):
        for sched in ("allreduce", "reduce_bcast", "sharded"):
            monkeypatch.setenv("PSX_NATIVE_RCCL", native)
            cfg = PSConfig(num_workers=1, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                           rows_per_iter=64, epochs=100, max_iters=8, init="random", bsp_schedule=sched,
                           min_buffer_size=256, max_buffer_size=256)
            eng = DistEngine(cfg, 0, 1, cuda, train=train, test=test)
            out = eng.run()
            assert out["rounds"] == 8
            ws[(native, sched)] = eng.server.w.cpu()
    base = ws[("0", "allreduce")]
    for k, w in ws.items():
        assert torch.allclose(w, base, atol=1e-4 * max(1.0, base.abs().max().item())), k


def test_dist_engine_native_bsp_loop_world1(cuda, pg, monkeypatch):
    """The allreduce rank body in the native BSP loop (RCCL all-reduce + update
    launch per round, rows riding in the solves) == the Python rank loop: same
    model, same rows."""
    from psx.parallel.dist import DistEngine
    from psx.runtime.config import PSConfig
    from psx.utils.data import synth_finefood

    train, test = synth_finefood(4000, seed=0), synth_finefood(500, seed=1)
    res = []
    monkeypatch.setenv("PSX_NATIVE_LANES", "0")  # (the single-worker BspLoop against the Python loop)
    for native in ("1", "0"):
        monkeypatch.setenv("PSX_NATIVE_BSP", native)
        cfg = PSConfig(num_workers=1, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                       rows_per_iter=64, epochs=100, max_iters=12, init="random", bsp_schedule="allreduce",
                       min_buffer_size=256, max_buffer_size=256)
        eng = DistEngine(cfg, 0, 1, cuda, train=train, test=test)
        out = eng.run()
        assert out["rounds"] == 12
        assert hasattr(eng, "native_host_us_per_round") == (native == "1")
        torch.cuda.synchronize()
        book = eng.log.book
        res.append((eng.server.w.cpu(), sorted((r[1], r[2], r[3]) for r in book.server),
                    sorted((r[1], r[2], r[3], r[4], r[5], r[6]) for r in book.worker), eng.server.updates))
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1] and [r[0] for r in res[0][1]] == list(range(12))
    assert res[0][2] == res[1][2] and res[0][3] == res[1][3]


def test_rccl_p2p_self_world1(cuda, pg):
    """RcclComm send / recv to self inside group_start / group_end for every piece
    shape the native SSP/ASP server sends (dense weights; sparse pull: ids int32 +
    values f32, split in two ring-log halves)."""
    from psx.parallel.comm import make_comm

    comm = make_comm(0, 1, cuda)
    c, s = comm.c, torch.cuda.current_stream().cuda_stream
    w = torch.randn(6150, device=cuda)
    ids = torch.randint(0, 1 << 20, (700,), dtype=torch.int32, device=cuda)
    vals = torch.randn(700 * 8, device=cuda)
    pieces = [w, ids[:300], vals[:300 * 8], ids[300:], vals[300 * 8:]]
    outs = [torch.zeros_like(t) for t in pieces]
    c.group_start()
    for t, o in zip(pieces, outs):
        dt = 1 if t.dtype == torch.int32 else 0
        c.send(t.data_ptr(), t.numel(), dt, 0, s)
        c.recv(o.data_ptr(), o.numel(), dt, 0, s)
    c.group_end()
    torch.cuda.synchronize()
    assert all(torch.equal(t, o) for t, o in zip(pieces, outs))
    comm.close()


@pytest.mark.parametrize("sched", ["reduce_bcast", "allreduce"])
def test_dist_lanes_world1_matches_local(cuda, pg, sched):
    """A rank of the multi-lane loop with RCCL (4 workers per rank: lane sum -> reduce
    to the server -> update -> broadcast, or all-reduce into every replica) gives the
    in-process engine's model and server rows."""
    from psx.parallel.dist import DistEngine
    from psx.runtime.config import PSConfig
    from psx.runtime.engine import LocalEngine
    from psx.utils.data import synth_finefood

    train, test = synth_finefood(20000, seed=0), synth_finefood(1000, seed=1)
    kw = dict(consistency_model=0, producer_time_per_event=0, stream_mode="per_iter", rows_per_iter=512,
              epochs=100, max_iters=10, init="random", min_buffer_size=512, max_buffer_size=512)
    cfg = PSConfig(num_workers=4, workers_per_rank=4, bsp_schedule=sched, **kw)
    eng = DistEngine(cfg, 0, 1, cuda, train=train, test=test)
    out = eng.run()
    assert out["rounds"] == 10 and getattr(eng, "_lanes", None) is not None
    ref = LocalEngine(PSConfig(num_workers=4, **kw), cuda, train=train, test=test)
    ref.run()
    torch.cuda.synchronize()
    scale = ref.server.w.abs().max().item()
    assert torch.allclose(eng.server.w, ref.server.w, atol=1e-5 * scale), (eng.server.w - ref.server.w).abs().max()
    a = [(r[1], round(r[2], 6)) for r in eng.log.book.server]
    b = [(r[1], round(r[2], 6)) for r in ref.log.book.server]
    assert [r[0] for r in a] == list(range(10)) and len(eng.log.book.worker) == 40
    assert sum(x != y for x, y in zip(a, b)) <= 2  # (argmax ties may flip with last-bit differences)


def test_dist_lanes_unbounded_run_stops_by_vote(cuda, pg):
    """max_iters 0 (the CLI default) runs natively too: chunks of the lanes loop with
    a collective stop vote -- by the wall clock, or when the data is exhausted."""
    from psx.parallel.dist import DistEngine
    from psx.runtime.config import PSConfig
    from psx.utils.data import synth_finefood

    train, test = synth_finefood(8000, seed=0), synth_finefood(500, seed=1)
    kw = dict(consistency_model=0, producer_time_per_event=0, stream_mode="per_iter", rows_per_iter=256,
              init="random", min_buffer_size=256, max_buffer_size=512, max_iters=0, num_workers=2,
              workers_per_rank=2, bsp_schedule="allreduce")
    eng = DistEngine(PSConfig(epochs=1000, max_wallclock_s=1.0, **kw), 0, 1, cuda, train=train, test=test)
    out = eng.run()
    assert getattr(eng, "_lanes", None) is not None and out["rounds"] >= 256 and out["rounds"] % 256 == 0
    assert [r[1] for r in eng.log.book.server] == list(range(out["rounds"]))
    # data exhausted (1 epoch = 4000 rows per worker = 16 rounds of deliveries), then idle_exit_s
    eng = DistEngine(PSConfig(epochs=1, idle_exit_s=0.3, **kw), 0, 1, cuda, train=train, test=test)
    out = eng.run()
    assert getattr(eng, "_lanes", None) is not None and out["rounds"] >= 256
    assert eng.workers[0].source.exhausted


def test_local_lanes_unbounded_run_stops_when_data_is_exhausted(cuda):
    from psx.runtime.config import PSConfig
    from psx.runtime.engine import LocalEngine
    from psx.utils.data import synth_finefood

    train, test = synth_finefood(8000, seed=0), synth_finefood(500, seed=1)
    cfg = PSConfig(consistency_model=0, producer_time_per_event=0, stream_mode="per_iter", rows_per_iter=256,
                   init="random", min_buffer_size=256, max_buffer_size=512, max_iters=0, num_workers=2, epochs=1,
                   idle_exit_s=0.3)
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    out = eng.run()
    assert out.get("lanes") == 2 and out["rounds"] >= 16
    assert all(w.source.exhausted for w in eng.workers)


def test_lanes_loop_dedicated_server_rank_world1(cuda, pg):
    """The dedicated server rank's body of the lanes loop (no lanes: a zero
    contribution reduced to itself, the update, the broadcast of the weights, the
    global model's evaluation rows) through the native RCCL communicator."""
    from psx import _native
    from psx.models.logreg import ModelSpec
    from psx.ops.lr import EvalSet, Fragments, SolverOptions, stream_handle
    from psx.parallel.comm import make_comm
    from psx.utils.data import synth_finefood
    from psx.utils.logsink import LogSink

    comm = make_comm(0, 1, cuda)
    h, host = _native.hip(), _native.host
    spec = ModelSpec(1024, 6)
    te = synth_finefood(1000, seed=1)
    ev = EvalSet(spec, te.X, te.y, cuda)
    o = SolverOptions()
    sc = h.SolverCfg()
    sc.K, sc.F, sc.Fp, sc.P, sc.cap = spec.K, spec.F, spec.Fp, spec.P, 1024
    sc.iters, sc.hist, sc.ls_max, sc.mode = o.iters, o.hist, o.ls_max, 0
    sc.center, sc.zero_const, sc.nslots, sc.gd_lr, sc.tol = 1, 1, o.nslots, o.gd_lr, o.tol
    w = spec.init("random", seed=2, device=cuda)
    w0 = w.clone()
    frags = [Fragments(spec, cuda), Fragments(spec, cuda)]
    sink = LogSink(spec.eval_classes, cuda)
    d = dict(scfg=sc, N=4, p_ms=1.0, k=[], w=w.data_ptr(), lr=0.25, api=host.capi(), server_rank=0,
             shi=[f.hi.data_ptr() for f in frags], slo=[f.lo.data_ptr() for f in frags],
             sb=[f.b.data_ptr() for f in frags], Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=ev.T,
             sink=sink.native.handle, log_server=1, log_workers=0)
    lp = h.LanesLoop(d, comm.c)
    assert lp.run(5, 0, stream_handle(cuda)) == 5
    lp.flush(stream_handle(cuda))
    torch.cuda.synchronize()
    sink.drain(block=True)
    assert torch.equal(w, w0)  # nothing pushed: w += lr * 0
    assert [r[1] for r in sink.book.server] == list(range(5)) and not sink.book.worker
    f1 = [r[2] for r in sink.book.server]
    assert max(f1) - min(f1) < 1e-9 and f1[0] > 0  # the same (unchanged) global model every round
    del lp
    comm.close()


def test_dist_lanes_cli_defaults_producer_clock_and_cadence(cuda, pg):
    """ServerAppRunner's defaults on the multi-rank engine: the producer clock (-p), the
    fresh-window cadence (iter_new_frac 0.5) and an unbounded run that stops by the
    wall clock -- all inside the native lanes loop (4-round chunks + stop vote)."""
    import time

    from psx.parallel.dist import DistEngine
    from psx.runtime.config import PSConfig, new_tuples_needed
    from psx.utils.data import synth_finefood

    train, test = synth_finefood(40000, seed=0), synth_finefood(1000, seed=1)
    cfg = PSConfig(consistency_model=0, producer_time_per_event=0.5, iter_new_frac=0.5, iter_new_cap=128,
                   max_iters=0, max_wallclock_s=2.0, num_workers=2, workers_per_rank=2, bsp_schedule="allreduce",
                   init="random")
    eng = DistEngine(cfg, 0, 1, cuda, train=train, test=test)
    t0 = time.time()
    out = eng.run()
    took = time.time() - t0
    assert getattr(eng, "_lanes", None) is not None, "the lanes loop did not run"
    assert out["rounds"] >= 3 and took < 2.0 + 3.0, (out["rounds"], took)
    book = eng.log.book
    assert [r[1] for r in book.server] == list(range(out["rounds"]))
    for k in (0, 1):
        seen = [r[-1] for r in book.worker if r[1] == k]
        assert len(seen) == out["rounds"]
        assert all(b - a >= min(new_tuples_needed(cfg, 128), 64) for a, b in zip(seen, seen[1:])), seen
