"""The native SSP/ASP server loop (csrc/runtime/async_server.h) on one MI355X,
over the same-process transport (LocalP2P) with stand-in workers: protocol,
tracker decisions, update + evaluation kernels and the server rows, checked
exactly (every worker's delta is fixed, so the final weights are known)."""
import pytest
import torch

from psx.parallel.async_local import LocalAsyncHarness
from psx.utils.data import synth_finefood

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,c", [(1, -1), (4, -1), (4, 2), (3, 0)])
def test_native_async_server_applies_every_delta(cuda, n, c):
    test = synth_finefood(600, seed=1)
    hs = LocalAsyncHarness(n, c, test=test, device=cuda)
    try:
        iters = 40
        out = hs.run(iters)
        assert out["updates"] == n * iters
        want = sum(hs.deltas) * (hs.lr * iters)
        d = (hs.w - want).abs().max().item()
        assert d < 1e-4 * max(1e-3, want.abs().max().item()), d
        # server rows follow worker 0's deltas (ServerProcessor.java:154-165)
        rows = hs.log.book.server
        assert len(rows) == iters and [r[1] for r in rows] == list(range(iters))
        assert all(0.0 <= r[3] <= 1.0 for r in rows)
        if c > 0:
            assert out["max_vc_gap"] <= c + 1
        if c == 0:
            assert out["max_vc_gap"] <= 1
        # the fragments of the evaluation follow w (refreshed by the update kernel)
        assert torch.isfinite(hs.w).all()
    finally:
        hs.close()


def test_native_async_server_two_runs(cuda):
    """A second run of the same server continues at the tracked clocks (the
    stand-in workers of the second run start where the tracker is)."""
    hs = LocalAsyncHarness(2, -1, test=synth_finefood(300, seed=1), device=cuda)
    try:
        out = hs.run(10)
        assert out["updates"] == 20 and hs.server.updates == 20
        # every worker finished (retired) at the end of run 1: run 2 revives them
        out = hs.run(7)
        assert out["updates"] == 14 and hs.server.updates == 34
        assert [hs.tracker.clock(k) for k in range(2)] == [17, 17]
    finally:
        hs.close()


@pytest.mark.parametrize("n,c", [(1, -1), (4, -1), (4, 2)])
def test_native_wide_sparse_pull(cuda, n, c):
    """Wide model, sparse pushes + sparse pulls through the native loop: every
    push applied, the pull log appended and shipped (far fewer floats than dense
    pulls), the weights exact."""
    from psx.parallel.async_local import LocalAsyncWideHarness

    hs = LocalAsyncWideHarness(n, c, device=cuda)
    try:
        iters = 30
        out = hs.run(iters)
        assert out["updates"] == n * iters
        want = hs.expected(iters)
        d = (hs.w - want).abs().max().item()
        assert d < 1e-4 * max(1e-3, want.abs().max().item()), d
        assert out["sparse_pulls"] > 0 and out["feeder_sparse"] == out["sparse_pulls"]
        assert out["pull_floats"] < (out["sparse_pulls"] + out["dense_pulls"]) * hs.P / 4
    finally:
        hs.close()


def test_log_append_apply_kernels(cuda):
    """Worker-side apply of logged pushes (atomic adds; ids repeat across entries)
    equals applying the pushes one by one; the log ring wraps."""
    from psx import _native

    h = _native.hip()
    F, KP, U = 5000, 8, 700
    cap = 3 * (U + 1) + 5  # entries 3.. wrap
    g = torch.Generator().manual_seed(3)
    lids = torch.zeros(cap, dtype=torch.int32, device=cuda)
    lvals = torch.zeros(cap * KP, device=cuda)
    w = torch.zeros(F * KP + KP, device=cuda)
    ref = torch.zeros_like(w)
    pos = 0
    s = torch.cuda.current_stream().cuda_stream
    entries = []
    for e in range(5):
        uniq = torch.randperm(F, generator=g)[:U].to(torch.int32).to(cuda)
        dl = (torch.randn((U + 1) * KP, generator=g)).to(cuda)
        h.log_append(uniq.data_ptr(), dl.data_ptr(), U, F, KP, lids.data_ptr(), lvals.data_ptr(), pos % cap, cap, s)
        entries.append((pos, uniq, dl))
        pos += U + 1
        ref[F * KP:] += 0.5 * dl[:KP]
        idx = (uniq.long() * KP).unsqueeze(1) + torch.arange(KP, device=cuda).unsqueeze(0)
        ref.index_add_(0, idx.reshape(-1), 0.5 * dl[KP:])
    # apply the last 2 entries (they wrap) from the ring, the first 3 by hand
    first3 = entries[2][0] + U + 1
    for p0, uniq, dl in entries[:3]:
        w[F * KP:] += 0.5 * dl[:KP]
        idx = (uniq.long() * KP).unsqueeze(1) + torch.arange(KP, device=cuda).unsqueeze(0)
        w.index_add_(0, idx.reshape(-1), 0.5 * dl[KP:])
    m = pos - first3
    start = first3 % cap
    l1 = min(m, cap - start)
    ids = torch.cat([lids[start:start + l1], lids[: m - l1]])
    vals = torch.cat([lvals[start * KP:(start + l1) * KP], lvals[: (m - l1) * KP]])
    h.log_apply(w.data_ptr(), ids.data_ptr(), vals.data_ptr(), m, KP, 0.5, s)
    torch.cuda.synchronize()
    assert (w - ref).abs().max().item() < 1e-5 * ref.abs().max().item()
