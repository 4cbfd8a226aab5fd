"""Where the fixed per-run cost of the driver's short bench form goes: the default
bench engine is built, warmed up, then `eng.run()` of --steps rounds is timed
--reps times (the bench's timed region: run + log drain + synchronize) and the
last repetition runs under cProfile (host-side attribution; GPU waits show up
in the synchronising calls).

    python tools/short_form_profile.py --steps 20 --reps 5 > out.txt
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    o = ap.parse_args()
    a = bench.parse(["--steps", str(o.steps), "--warmup", "5"])
    from psx.runtime.engine import LocalEngine

    train, test = bench.make_data(a, "cuda:0")
    cfg = bench.build_cfg(a, a.workers)
    cfg.max_iters = a.warmup
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    eng.run(close_log=False)
    eng.cfg.max_iters = o.steps
    for rep in range(o.reps):
        prof = cProfile.Profile() if rep == o.reps - 1 else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if prof:
            prof.enable()
        eng.run(close_log=False)
        eng.log.drain(block=True)
        torch.cuda.synchronize()
        if prof:
            prof.disable()
        dt = time.perf_counter() - t0
        print(f"rep {rep}: {o.steps} rounds in {dt * 1e3:.3f} ms = {dt * 1e6 / o.steps:.1f} us/round", flush=True)
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(40)
    print(s.getvalue())
    eng.log.close()


if __name__ == "__main__":
    main()
