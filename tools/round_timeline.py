"""Per-round device timeline of the BSP lanes loop in bench.py's configuration, from
the lanes kernels' own phase stamps (LanesLoop.set_trace, the --trace path):
for every round of the timed call, when its first lane started staging (relative to
the call's first round), how long the slowest lane's stage / solve / update took,
and the start-to-start interval to the next round.  Shows where a short
(driver-form) call spends the time its steady-state rounds do not.

    python tools/round_timeline.py --steps 20 --warmup 5 > round_timeline.json
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    import torch

    import bench
    from psx.runtime.engine import LocalEngine

    a = bench.parse(argv)
    tmp = tempfile.mkdtemp(prefix="psx_rt_")
    train, test = bench.make_data(a, "cuda:0")
    cfg = bench.build_cfg(a, a.workers)
    cfg.trace_path = os.path.join(tmp, "trace.json")
    cfg.perf_log = True
    cfg.log_dir = tmp
    cfg.max_iters = a.warmup
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    if a.warmup > 0:
        eng.run(close_log=False)
    eng.cfg.max_iters = a.steps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(close_log=False, summary=False)
    eng.log.drain(block=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    eng.tracer.close()
    ev = json.load(open(cfg.trace_path))["traceEvents"]
    rounds = {}
    for e in ev:
        if e.get("tid") != "device" or "round" not in e.get("args", {}):
            continue
        r = rounds.setdefault(e["args"]["round"], {})
        name, ts, end = e["name"], e["ts"], e["ts"] + e["dur"]
        r["start"] = min(r.get("start", ts), ts) if name == "ingest" else r.get("start", ts)
        r[name] = max(r.get(name, 0.0), e["dur"])
        r["end"] = max(r.get("end", end), end)
    rs = sorted(rounds)[-a.steps:]
    base = rounds[rs[0]]["start"]
    out = []
    for i, k in enumerate(rs):
        r = rounds[k]
        nxt = rounds[rs[i + 1]]["start"] - r["start"] if i + 1 < len(rs) else None
        out.append({"round": k, "start_us": round(r["start"] - base, 2), "ingest_us": round(r.get("ingest", 0), 2),
                    "solve_us": round(r.get("solve", 0), 2), "update_us": round(r.get("server", 0), 2),
                    "lanes_us": round(r["end"] - r["start"], 2),
                    "to_next_us": round(nxt, 2) if nxt is not None else None})
    last = rounds[rs[-1]]
    print(json.dumps({"steps": a.steps, "warmup": a.warmup, "call_ms": round(dt * 1e3, 3),
                      "ms_per_step": round(dt * 1e3 / a.steps, 5),
                      "first_round_start_to_last_lane_end_us": round(last["end"] - base, 2),
                      "rounds": out}))


if __name__ == "__main__":
    main()
