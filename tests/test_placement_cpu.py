"""Engine-side choice of the solve's placement and launch form (CPU-checkable
parts; the kernels themselves: tests/test_gpu_kernels.py)."""
import torch

from psx.ops.lr import SolverOptions
from psx.runtime.config import PSConfig
from psx.runtime.engine import LocalEngine
from psx.utils.data import synth_finefood


def _cfg(n):
    return PSConfig(num_workers=n, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                    rows_per_iter=64, epochs=10, max_iters=1, init="zeros")


def test_workers_xcd_placement():
    train, test = synth_finefood(600, seed=0), synth_finefood(100, seed=1)
    one = LocalEngine(_cfg(1), "cpu", train=train, test=test)
    assert one.workers[0].solver.opts.xcd == 0  # a lone solver: its workgroups on XCD 0
    many = LocalEngine(_cfg(3), "cpu", train=train, test=test)
    assert all(w.solver.opts.xcd == -1 for w in many.workers)  # concurrent solvers: spread


def test_solver_options_defaults():
    o = SolverOptions()
    assert o.persist is None and o.xcd == 0 and o.tail is True


def test_bench_chain_flag():
    import bench

    a = bench.parse(["--chain"])
    cfg = bench.build_cfg(a, 1)
    assert cfg.solver.persist is False
    a = bench.parse(["--persist"])
    assert bench.build_cfg(a, 1).solver.persist is True
    assert bench.build_cfg(bench.parse([]), 1).solver.persist is None  # the engine decides
    assert torch.device("cpu").type == "cpu"
