"""Key-range sharded parameter server (psx/parallel/keyrange.py) on CPU ranks
(gloo, world 4): each rank stores only its key range, a round moves only the
window's ids / values, and the result equals the replicated dense schedule."""
import gc
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


BASE = dict(consistency_model=0, producer_time_per_event=0, stream_mode="per_iter", rows_per_iter=64, epochs=100,
            max_iters=6, min_buffer_size=64, max_buffer_size=128, init="random", model="wide", sigmoid=True,
            server_colocated=True)


def _data(F):
    from psx.utils.data import synth_sparse

    kw = dict(num_features=F, labels="binary", nnz_mean=16, max_nnz=32, vocab=20000, class_vocab=300)
    return synth_sparse(1200, seed=0, **kw), synth_sparse(150, seed=1, **kw)


def _rank_main(rank, world, port, kw, F, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from psx.parallel.dist import DistEngine, init_from_env
    from psx.runtime.config import PSConfig

    torch.set_num_threads(2)
    r, w, dev = init_from_env(cpu=True)
    cfg = PSConfig(**kw)
    train, test = _data(F)
    eng = DistEngine(cfg, r, w, dev, train=train, test=test)
    out = eng.run()
    res = {"out": {k: v for k, v in out.items() if k in ("rounds", "keyrange", "updates")}}
    if "keyrange" in out:
        gc.collect()
        # the largest float32 tensor alive in this rank: its shard, nothing P-sized
        res["max_f32"] = max(t.numel() for t in gc.get_objects()
                             if torch.is_tensor(t) and t.dtype == torch.float32)
        res["shard_numel"] = eng.shard.numel()
        parts = [None] * w
        dist.all_gather_object(parts, (eng.lo, eng.hi, eng.shard.numpy().copy(), eng.b.numpy().copy()))
        res["parts"] = parts if r == 0 else None
    else:
        res["w"] = eng.server.w.numpy().copy() if r == 0 else None
    res["server"] = list(eng.log.book.server) if r == 0 else None
    res["worker"] = list(eng.log.book.worker) if r == 0 else None
    out_q.put((r, res))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, kw, F):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, kw, F, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _assemble(parts, F, KP):
    w = torch.zeros(F * KP + KP)
    for lo, hi, shard, b in parts:
        w[lo * KP:hi * KP] = torch.from_numpy(shard[: (hi - lo) * KP])
        w[F * KP:] = torch.from_numpy(b)
    return w


def test_key_range_partition():
    from psx.parallel.keyrange import key_range

    F = 1_000_003
    rs = [key_range(F, 4, r) for r in range(4)]
    assert rs[0][0] == 0 and rs[-1][1] == F
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    assert max(hi - lo for lo, hi, _ in rs) - min(hi - lo for lo, hi, _ in rs) <= 3


def test_shard_csr_margins_sum_to_full():
    """Partial margins of the shards of a CSR set sum to the full margins."""
    from psx.models.wide import WideSpec
    from psx.parallel.keyrange import _csr_mm, key_range, shard_csr

    train, test = _data(50_000)
    spec = WideSpec(50_000, 1)
    w = spec.init("random", seed=2, scale=1.0)
    full = _csr_mm(test, w[: spec.F].view(spec.F, 1))
    tot = torch.zeros_like(full)
    for r in range(3):
        lo, hi, _ = key_range(spec.F, 3, r)
        s = shard_csr(test, lo, hi)
        tot += _csr_mm(s, spec.init_range("random", 2, lo, hi, scale=1.0)[: hi - lo].view(hi - lo, 1))
    assert torch.allclose(tot, full, atol=1e-5)


def _replicated(F, W, rounds):
    """Oracle: BSP with a full dense replica -- every worker's round-r window
    (one delivery per round), its solve from the whole model, w += lr * sum."""
    from psx.models.wide import WideSpec
    from psx.ops.lr import SolverOptions
    from psx.ops.sparse import SparseRing, WideSolveOp, nz_capacity
    from psx.runtime.buffer import StreamSource
    from psx import _native

    train, _ = _data(F)
    spec = WideSpec(F, 1)
    w = spec.init("random", seed=0)
    nz = nz_capacity(train.max_nnz)
    ws = []
    for k in range(W):
        ring = SparseRing(BASE["max_buffer_size"], nz, "cpu")
        win = _native.host.SlidingWindow(BASE["min_buffer_size"], BASE["max_buffer_size"], 0.3, 500, ring.cap)
        src = StreamSource(train, k, W, ring, win, mode="per_iter", rows_per_iter=BASE["rows_per_iter"], epochs=100)
        ws.append((ring, win, src, WideSolveOp(spec, ring.cap, nz, "cpu", SolverOptions())))
    for _ in range(rounds):
        tot = torch.zeros_like(w)
        for ring, win, src, op in ws:
            src.poll()
            op.run(ring, int(win.size), int(win.start), w)
            tot += op.sparse_delta().to_dense()
        w += tot / W
    return w


@pytest.mark.timeout(600)
def test_keyrange_world4_matches_replicated_and_stores_a_quarter(tmp_path):
    F, KP = 1_000_000, 1
    kr = _run(4, dict(BASE, bsp_schedule="keyrange", logging=True, log_dir=str(tmp_path)), F)
    # the same BSP model as applying the summed deltas to a full replica
    w_kr = _assemble(kr[0]["parts"], F, KP)
    w_ref = _replicated(F, 4, BASE["max_iters"])
    assert torch.allclose(w_kr, w_ref, atol=2e-6, rtol=1e-5), (w_kr - w_ref).abs().max()
    # per-rank weight memory ~ P / 4, and nothing P-sized anywhere in the process
    P = F * KP + KP
    for r in range(4):
        k = kr[r]["out"]["keyrange"]
        assert k["weight_bytes"] <= (P // 4 + 2 * KP + 1) * 4
        assert kr[r]["max_f32"] == kr[r]["shard_numel"] <= P // 4 + KP + 1
    # rows: one server row per round (rank 0), one worker row per worker per round
    assert [s[1] for s in kr[0]["server"]] == list(range(6))
    assert [x[1] for x in kr[0]["worker"]] == [0] * 6  # rank 0's own worker rows
    lines = (tmp_path / "logs-worker.csv").read_text().splitlines()
    assert lines[0].startswith("timestamp;partition;vectorClock") and len(lines) == 1 + 6 * 4
    assert sorted({int(x.split(";")[1]) for x in lines[1:]}) == [0, 1, 2, 3]
    assert len((tmp_path / "logs-server.csv").read_text().splitlines()) == 1 + 6
    # the last server row evaluates the final model
    from psx.models.wide import WideSpec
    from psx.ops.sparse import WideEvalSet

    conf = WideEvalSet(WideSpec(F, 1), _data(F)[1], "cpu").confusion_cpu(w_kr).view(16, 16)[:2, :2].double()
    assert abs(kr[0]["server"][-1][3] - float(conf.trace() / conf.sum())) < 1e-9


@pytest.mark.timeout(600)
def test_keyrange_bytes_follow_the_window_not_the_model():
    """Model traffic per round is set by the window's distinct features: an 8x
    wider model moves the same bytes (and far fewer than one dense vector)."""
    outs = {}
    for F in (500_000, 4_000_000):
        res = _run(4, dict(BASE, bsp_schedule="keyrange", max_iters=3), F)
        outs[F] = [res[r]["out"]["keyrange"] for r in range(4)]
    for F, ks in outs.items():
        for k in ks:
            U = k["last_u"]
            bound = 4 * 4 + 8 * U + 8 * U * 1 + 4
            assert 0 < k["last_round_bytes"] <= bound, (F, k)
            assert k["last_round_bytes"] < (F + 1) * 4 / 50
    a = sum(k["last_round_bytes"] for k in outs[500_000])
    b = sum(k["last_round_bytes"] for k in outs[4_000_000])
    assert 0.8 < b / a < 1.25, (a, b)
