"""Host cost of one in-process BSP round (bench.py's headline engine) on one GPU:
enqueue a short burst of rounds right after a device sync (the launch queue never
fills, so the host time is the host's own cost), then sync and take the wall time
of the burst (GPU-bound when the device time exceeds the host time).
Usage: python tools/host_cost.py [rounds] [extra bench flags...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from psx.runtime.engine import LocalEngine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    a = bench.parse(sys.argv[2:])
    train, test = bench.make_data(a, "cuda:0")
    cfg = bench.build_cfg(a, a.workers)
    cfg.max_iters = 200
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    eng.run()
    print(f"graph={cfg.solver.use_graph}")
    sync = torch.cuda.synchronize
    # host time inside the solver launches alone
    from psx.ops import lr as lrmod
    acc = {"run": 0.0, "n": 0}
    orig_run = lrmod.LocalSolveOp.run

    def timed_run(self, *a, **k):
        t = time.perf_counter()
        try:
            return orig_run(self, *a, **k)
        finally:
            acc["run"] += time.perf_counter() - t
            acc["n"] += 1

    lrmod.LocalSolveOp.run = timed_run
    for _ in range(5):
        eng.cfg.max_iters = n
        eng.log = bench._fresh_log(eng)  # run() closes its sink
        sync()
        torch.cuda.synchronize = lambda *a, **k: None  # the engine's end-of-run sync
        try:
            t0 = time.perf_counter()
            eng.run()
            t1 = time.perf_counter()
        finally:
            torch.cuda.synchronize = sync
        sync()
        t2 = time.perf_counter()
        print(f"{n} rounds: host {1e6 * (t1 - t0) / n:.1f} us/round, wall {1e6 * (t2 - t0) / n:.1f} us/round, "
              f"solver launches {1e6 * acc['run'] / max(acc['n'], 1):.1f} us/solve", flush=True)
        acc.update(run=0.0, n=0)


if __name__ == "__main__":
    main()
