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
