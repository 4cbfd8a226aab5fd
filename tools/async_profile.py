"""Per-update timeline of the asynchronous lanes loop (csrc/kernels/lanes_async.hip) on one
MI355X: the phases of every lane's last update from the device's s_memrealtime stamps
(100 MHz): the solve, the ticket, the serial slice updates, the
token and the lane's own evaluation row.

    PSX_LANES_STAMPS=1 python tools/async_profile.py [--consistency -1] [--iters 300]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--consistency", type=int, default=-1)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=300)
    a = ap.parse_args()
    import torch

    from psx.ops.lr import stream_handle
    from psx.runtime.config import PSConfig
    from psx.runtime.engine import LocalEngine
    from psx.utils.data import synth_finefood

    cfg = PSConfig(num_workers=a.workers, consistency_model=a.consistency, producer_time_per_event=0,
                   stream_mode="per_iter", rows_per_iter=1024, epochs=1000, max_iters=30, min_buffer_size=128,
                   max_buffer_size=1024, init="random", seed=0)
    eng = LocalEngine(cfg, "cuda:0", train=synth_finefood(90000, seed=0), test=synth_finefood(4877, seed=1))
    eng.run(close_log=False)  # warm-up
    eng.cfg.max_iters = a.iters
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = eng.run(close_log=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = {"consistency": a.consistency, "workers": a.workers, "updates_per_s": round(a.iters * a.workers / dt, 1),
           "async_lanes": bool(out.get("async_lanes"))}
    lp = eng._lanes
    if os.environ.get("PSX_LANES_STAMPS") and lp is not None:
        lanes = []
        for l in range(a.workers):
            st = lp.read_stamps(l, stream_handle("cuda:0"))
            T = lambda k: st[30 * 16 + k]
            us = lambda x, y: round((T(y) - T(x)) / 100.0, 2) if T(x) and T(y) else None
            ln = {"solve": us(0, 4), "ticket": us(4, 5), "apply": us(5, 6), "token": us(6, 7), "eval": us(7, 8),
                  # the last iteration's start: release record seen, the lane-wide barrier
                  "wait_release": us(9, 10), "barrier": us(10, 0),
                  # (its parts: the lane-wide barrier; the record read + the acquire fence;
                  # from there to the released stamp)
                  "barrier_wait": us(10, 11), "record+acquire": us(11, 12), "to_stamp": us(12, 0),
                  # (the solve's start: the pulled weights read, this workgroup's rows staged,
                  # every row workgroup staged)
                  "s.pull": us(0, 13), "s.stage": us(13, 14), "s.stage_barrier": us(14, 15)}
            # the solve's slots (the same stamps as the BSP round kernel: tools/lanes_profile.py)
            from lanes_profile import phases
            ends = [st[(24 + (w >> 4)) * 16 + (w & 15)] for w in range(32)]
            starts = [st[(26 + (w >> 4)) * 16 + (w & 15)] for w in range(32)]
            if all(ends) and all(starts) and T(7):
                ln["eval_wg_start_us"] = [round((x - T(7)) / 100.0, 2) for x in (min(starts), max(starts))]
                ln["eval_wg_end_us"] = [round((x - T(7)) / 100.0, 2) for x in (min(ends), max(ends))]
            ph = phases(st)
            ln["slots"] = ph.get("slots")
            lanes.append(ln)
        res["last_update_us"] = lanes
    eng.log.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
