"""End-to-end parameter-server runs on one MI355X (in-process engine)."""
import pytest
import torch

from psx import _native
from psx.ops.lr import SolverOptions
from psx.runtime.config import PSConfig
from psx.runtime.engine import LocalEngine
from psx.utils.data import synth_finefood

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    base = dict(num_workers=1, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                rows_per_iter=128, epochs=1000, max_iters=30, init="zeros")
    base.update(kw)
    return PSConfig(**base)


def test_bsp_single_worker_learns(cuda):
    train, test = synth_finefood(20000, seed=0), synth_finefood(2000, seed=1)
    eng = LocalEngine(_cfg(max_iters=150), cuda, train=train, test=test)
    out = eng.run()
    assert out["rounds"] == 150
    accs = [r[3] for r in eng.log.book.server]
    assert accs[-1] > 0.33, accs[-10:]  # well above the 0.2 prior
    assert _native.hip_loaded_path() is not None


@pytest.mark.parametrize("c", [-1, 2])
def test_async_two_workers_threads(cuda, c):
    train, test = synth_finefood(8000, seed=0), synth_finefood(1000, seed=1)
    cfg = _cfg(num_workers=2, consistency_model=c, max_iters=20,
               inject_worker_delay_ms={1: 5.0})
    eng = LocalEngine(cfg, cuda, train=train, test=test)
    out = eng.run()
    assert out["updates"] >= 40
    if c > 0:
        assert out["max_vc_gap"] <= c + 1
    ws = eng.log.book.worker
    assert {r[1] for r in ws} == {0, 1}


def test_gd_solver_mode(cuda):
    train, test = synth_finefood(4000, seed=0), synth_finefood(500, seed=1)
    eng = LocalEngine(_cfg(max_iters=10, solver=SolverOptions(mode="gd", gd_lr=2.0, iters=3)), cuda,
                      train=train, test=test)
    out = eng.run()
    assert out["rounds"] == 10
    torch.cuda.synchronize()
