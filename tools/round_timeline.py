"""Per-round device timeline of the BSP lanes loop in bench.py's configuration, from
the lanes kernels' own phase stamps (LanesLoop.set_trace): for every round of the
timed call, when its first lane started staging, how long the slowest lane's stage /
solve / update took, the start-to-start interval to the next round -- and where the
call's wall clock went outside the rounds (host start -> first round, last lane ->
the call's end).  The ring is armed on the cached loop after the warm-up and read
after the call, so the timed call itself runs exactly as in bench.py.

    python tools/round_timeline.py --steps 20 --warmup 5 > round_timeline.json
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    import torch

    import bench
    from psx.ops.lr import stream_handle
    from psx.runtime.engine import LocalEngine

    a = bench.parse(argv)
    train, test = bench.make_data(a, "cuda:0")
    cfg = bench.build_cfg(a, a.workers)
    cfg.max_iters = a.warmup
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    if a.warmup > 0:
        eng.run(close_log=False)
    lp = getattr(eng, "_lanes", None)
    if lp is None:
        raise SystemExit("round_timeline: the run did not take the BSP lanes loop")
    lp.set_trace(max(64, a.steps + 8))
    eng.cfg.max_iters = a.steps
    torch.cuda.synchronize()
    h0 = time.perf_counter_ns()
    out = eng.run(close_log=False, summary=False)
    h_run = time.perf_counter_ns()
    eng.log.drain(block=True)
    torch.cuda.synchronize()
    h1 = time.perf_counter_ns()
    stream = stream_handle(eng.device)
    rows = lp.trace_take(stream)
    ref = lp.clock_ref(stream)
    off_us = (ref[0] + ref[2]) / 2000.0 - ref[1] / 100.0  # device ticks (10 ns) -> host us

    def us(t):
        return off_us + t / 100.0

    rounds = {}
    for r in rows:
        if r[0] != 0 or min(r[4:8]) <= 0:
            continue
        d = rounds.setdefault(int(r[1]), {"start": us(r[4]), "end": us(r[7]), "ingest": 0.0, "solve": 0.0,
                                           "update": 0.0})
        d["start"] = min(d["start"], us(r[4]))
        d["end"] = max(d["end"], us(r[7]))
        d["ingest"] = max(d["ingest"], (r[5] - r[4]) / 100.0)
        d["solve"] = max(d["solve"], (r[6] - r[5]) / 100.0)
        d["update"] = max(d["update"], (r[7] - r[6]) / 100.0)
    rs = sorted(rounds)
    base = rounds[rs[0]]["start"]
    per = []
    for i, k in enumerate(rs):
        d = rounds[k]
        nxt = rounds[rs[i + 1]]["start"] - d["start"] if i + 1 < len(rs) else None
        per.append({"round": k, "start_us": round(d["start"] - base, 2), "ingest_us": round(d["ingest"], 2),
                    "solve_us": round(d["solve"], 2), "update_us": round(d["update"], 2),
                    "lanes_us": round(d["end"] - d["start"], 2), "to_next_us": round(nxt, 2) if nxt else None})
    h0u, h1u = h0 / 1000.0, h1 / 1000.0
    print(json.dumps({
        "steps": a.steps, "warmup": a.warmup, "rounds_seen": len(rs),
        "call_us": round(h1u - h0u, 2), "us_per_step": round((h1u - h0u) / a.steps, 3),
        "host_start_to_first_round_us": round(base - h0u, 2),
        "first_round_to_last_lane_end_us": round(rounds[rs[-1]]["end"] - base, 2),
        "last_lane_end_to_call_end_us": round(h1u - rounds[rs[-1]]["end"], 2),
        "run_returned_after_last_lane_us": round(h_run / 1000.0 - rounds[rs[-1]]["end"], 2),
        "host_start_to_lp_run_us": round(eng._t_lp_run_ns / 1000.0 - h0u, 2),
        "lp_run_to_first_round_us": round(base - eng._t_lp_run_ns / 1000.0, 2),
        "lp_run_returned_rel_last_lane_end_us": round(eng._t_lp_done_ns / 1000.0 - rounds[rs[-1]]["end"], 2),
        "phases_ms": out.get("phases_ms"),
        "rounds": per}))


if __name__ == "__main__":
    main()
