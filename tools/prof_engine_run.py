"""cProfile of one driver-form timed engine run (bench.py's dense default: 8 workers,
20 rounds after 5 warm-up rounds): where the Python around the native loop goes."""
import cProfile
import pstats
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402
from psx.runtime.engine import LocalEngine  # noqa: E402

import torch  # noqa: E402


def main():
    a = bench.parse(["--steps", "20", "--warmup", "5"])
    train, test = bench.make_data(a, "cuda:0")
    cfg = bench.build_cfg(a, a.workers)
    cfg.max_iters = a.warmup
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    eng.run(close_log=False)
    for rep in range(3):
        eng.cfg.max_iters = 20
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        eng.run(close_log=False, summary=False)
        eng.log.drain(block=True)
        torch.cuda.synchronize()
        pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
