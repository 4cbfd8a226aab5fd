"""Round time and per-lane phase timeline of the multi-lane BSP round kernel.

    PSX_LANES_STAMPS=1 python tools/lanes_profile.py --lanes 4 --rounds 400 [--no-eval]

Prints us per round (synchronised around `rounds` rounds after a warm-up) and, for
every lane, the phases of its last solve from the device's s_memrealtime stamps
(100 MHz): phase I (stage + ingest + column sums), the statistics barrier, prep
and first trial point, each slot (forward -> backward/controller), the
finalisation and the cross-lane update.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(L, rows, evaluate, dev):
    import torch

    from psx import _native
    from psx.models.logreg import ModelSpec
    from psx.ops.lr import EvalSet, Fragments, SolverOptions
    from psx.utils.data import synth_finefood
    from psx.utils.logsink import LogSink

    h, host = _native.hip(), _native.host
    spec = ModelSpec(1024, 6)
    train = synth_finefood(90000, seed=0).to(dev)
    te = synth_finefood(4877, seed=1)
    ev = EvalSet(spec, te.X, te.y, dev)
    o = SolverOptions()
    cap = 1024
    sc = h.SolverCfg()
    sc.K, sc.F, sc.Fp, sc.P, sc.cap = spec.K, spec.F, spec.Fp, spec.P, cap
    sc.iters, sc.hist, sc.ls_max, sc.mode = o.iters, o.hist, o.ls_max, 0
    sc.center, sc.zero_const, sc.nslots, sc.gd_lr, sc.tol = 1, 1, o.nslots, o.gd_lr, o.tol
    rings = [(torch.zeros(cap, spec.Fp, dtype=torch.bfloat16, device=dev),
              torch.zeros(cap, dtype=torch.int32, device=dev)) for _ in range(L)]
    wins = [host.SlidingWindow(cap, cap, 0.3, 500, cap) for _ in range(L)]
    frags = [Fragments(spec, dev), Fragments(spec, dev)]
    w = spec.init("random", seed=0, device=dev)
    log = LogSink(spec.K, dev) if evaluate else None
    d = dict(scfg=sc, dsX=train.X.data_ptr(), dsy=train.y.data_ptr(), ds_rows=int(train.rows), N=L,
             per_iter_rows=rows, epochs=1000, k=list(range(L)), X=[r[0].data_ptr() for r in rings],
             y=[r[1].data_ptr() for r in rings], window=[wn.handle for wn in wins], w=w.data_ptr(), lr=1.0 / L,
             shi=[f.hi.data_ptr() for f in frags], slo=[f.lo.data_ptr() for f in frags],
             sb=[f.b.data_ptr() for f in frags], Xt=ev.X.data_ptr(), yt=ev.y.data_ptr(), T=ev.T,
             sink=log.native.handle if log is not None else 0, api=host.capi())
    lp = h.LanesLoop(d, None)
    return lp, (train, ev, rings, wins, frags, w, log)


def phases(st):
    """Durations (us) of lane phases from a [32][16] stamp table (0: not written)."""
    T = lambda s, k: st[s * 16 + k]
    base = T(30, 0)
    if not base:
        return {}
    us = lambda a, b: round((b - a) / 100.0, 2) if a and b else None
    out = {"stage+sums": us(T(30, 0), T(30, 1)), "stats barrier": us(T(30, 1), T(30, 2)),
           "prep+barrier": us(T(30, 2), T(30, 3))}
    slots = []
    for s in range(30):
        if not T(s, 0):
            break
        slots.append({"fwd": us(T(s, 0), T(s, 2)), "bwd": us(T(s, 2), T(s, 8)),
                      "fwd_start_us": us(base, T(s, 0)),
                      # lane 0's workgroup 0: trial-point fragments + staging wait, forward MFMA,
                      # softmax + backward tile, row sums, partials store + barrier
                      "f.wfrag": us(T(s, 0), T(s, 9)), "f.mfma": us(T(s, 9), T(s, 10)),
                      "f.smax+bwd": us(T(s, 10), T(s, 11)), "f.sums": us(T(s, 11), T(s, 1)),
                      "f.gpf+barrier": us(T(s, 1), T(s, 2)),
                      # slice owner 0: partials reduce, gradient, dots + all-gather, controller,
                      # controller copy, apply + next trial point
                      "b.reduce": us(T(s, 2), T(s, 3)), "b.grad": us(T(s, 3), T(s, 4)),
                      "b.dots+gather": us(T(s, 4), T(s, 5)), "b.ctrl": us(T(s, 5), T(s, 6)),
                      "b.copy": us(T(s, 6), T(s, 7)), "b.apply+next": us(T(s, 7), T(s, 8)),
                      # finer: partials store issue / barrier wait; the dots' local part, the
                      # all-gather wait, the fixed-order sum
                      "f.gpf": us(T(s, 1), T(s, 15)), "f.barrier": us(T(s, 15), T(s, 2)),
                      "b.dots.local": us(T(s, 4), T(s, 12)), "b.gather": us(T(s, 12), T(s, 13)),
                      "b.dots.sum": us(T(s, 13), T(s, 14))})
    out["slots"] = slots
    out["slots_total"] = us(T(30, 3), T(30, 4))
    out["finalize"] = us(T(30, 4), T(30, 5))
    out["update"] = us(T(30, 5), T(30, 6))
    out["solve_total"] = us(T(30, 0), T(30, 6))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=400)
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--no-eval", dest="evaluate", action="store_false")
    a = ap.parse_args()
    import torch

    from psx.ops.lr import stream_handle

    dev = "cuda:0"
    lp, keep = build(a.lanes, a.rows, a.evaluate, dev)
    s = stream_handle(dev)
    lp.run(50, 0, s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp.run(a.rounds, 50, s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = {"lanes": a.lanes, "evaluate": a.evaluate, "us_per_round": round(dt / a.rounds * 1e6, 2),
           "updates_per_s": round(a.rounds * a.lanes / dt, 1), "host_us_per_round": round(lp.host_us_per_round, 2),
           "hand_off_scope": lp.hand_off_scope}
    if os.environ.get("PSX_LANES_STAMPS"):
        res["phases"] = [phases(lp.read_stamps(l, s)) for l in range(a.lanes)]
        # the riders of the last round, us from lane 0's phase-I start (its stamp 30/0)
        rs, base = lp.read_rider_stamps(s), lp.read_stamps(0, s)[30 * 16]
        if rs and base:
            rel = lambda t: round((t - base) / 100.0, 2) if 0 < t < (1 << 62) else None
            res["riders"] = {"kernel_first_entry": rel(rs[15]), "first_entry": rel(rs[12]), "last_entry": rel(rs[13]), "rider0_entry": rel(rs[0]),
                             "rider0_first_tile": rel(rs[1]), "rider0_items": [rel(rs[2 + i]) for i in range(4)],
                             "rider0_ticket": rel(rs[8]), "last_ticket": rel(rs[14]),
                             "publisher_known": rel(rs[10]), "published": rel(rs[11])}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
