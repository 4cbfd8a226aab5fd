"""Where the Python around one BSP lanes call goes (bench.py's driver form): cProfile of
N timed calls after the warm-up, sorted by own time.  Native calls (LanesLoop.run) show
as single entries.

    python tools/run_overhead.py --steps 20 --warmup 5
"""
from __future__ import annotations

import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    import torch

    import bench
    from psx.runtime.engine import LocalEngine

    a = bench.parse(argv)
    train, test = bench.make_data(a, "cuda:0")
    cfg = bench.build_cfg(a, a.workers)
    cfg.max_iters = a.warmup
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    eng.run(close_log=False)
    eng.cfg.max_iters = a.steps
    torch.cuda.synchronize()
    times = []
    pr = cProfile.Profile()
    for i in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter_ns()
        if i >= 1:
            pr.enable()
        eng.run(close_log=False, summary=False)
        if i >= 1:
            pr.disable()
        eng.log.drain(block=True)
        torch.cuda.synchronize()
        times.append((time.perf_counter_ns() - t0) / 1000.0)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print("call_us", [round(t, 1) for t in times])
    print(s.getvalue())


if __name__ == "__main__":
    main()
