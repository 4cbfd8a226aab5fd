"""Test accuracy / weighted F1 vs wall-clock (the reference's headline plots,
README.md:237-326, docs/plots/*.png), measured on one device with the
in-process engine: N workers stream their round-robin shards of the synthetic
fine-food data (64 new rows per worker per round, unthrottled producer) under a
consistency model; every server row (global model on the 4,877-row test set)
is timestamped.  Reports per N: rounds, updates/s, best/final F1, time to
reach F1 >= 0.40 / 0.42 / 0.44 (reference best: 124 s to 0.40 with 4 workers
at 10 tps) and accuracy at fixed times.

Usage: python tools/accuracy_wallclock.py [--workers 1 2 4 8] [--consistency 0]
                                          [--epochs 3] [--device cuda:0] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def first_time(rows, t0, thr):
    for ts, _vc, f1, _acc in rows:
        if f1 >= thr:
            return round((ts - t0) / 1000.0, 3)
    return None


def acc_at(rows, t0, sec):
    best = None
    for ts, _vc, _f1, acc in rows:
        if (ts - t0) / 1000.0 <= sec:
            best = acc
    return None if best is None else round(best, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--consistency", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--rows-per-iter", type=int, default=64)
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from psx.runtime.config import PSConfig
    from psx.runtime.engine import LocalEngine
    from psx.utils.data import synth_finefood

    train, test = synth_finefood(90000, seed=0), synth_finefood(4877, seed=1)
    out = []
    print(f"{'N':>3} {'c':>3} {'rounds':>7} {'wall_s':>7} {'upd/s':>9} {'best_f1':>8} {'final_f1':>8} "
          f"{'t_f1>=.40':>9} {'t_f1>=.42':>9} {'t_f1>=.44':>9} {'acc@0.1s':>8} {'acc@1s':>7}")
    for N in a.workers:
        cfg = PSConfig(num_workers=N, consistency_model=a.consistency, producer_time_per_event=0,
                       stream_mode="per_iter", rows_per_iter=a.rows_per_iter, epochs=a.epochs, max_iters=0,
                       idle_exit_s=0.0, init="zeros")
        eng = LocalEngine(cfg, a.device, train=train, test=test)
        res = eng.run()
        rows = eng.log.book.server
        t0 = min(r[0] for r in eng.log.book.worker)  # reference definition: first log row
        f1 = [r[2] for r in rows]
        rec = {"workers": N, "consistency": a.consistency, "rounds": res["rounds"], "wall_s": round(res["elapsed_s"], 3),
               "updates_per_s": round(res["updates_per_s"], 1), "best_f1": round(max(f1), 4),
               "final_f1": round(f1[-1], 4), "t_f1_040": first_time(rows, t0, 0.40),
               "t_f1_042": first_time(rows, t0, 0.42), "t_f1_044": first_time(rows, t0, 0.44),
               "acc_0.1s": acc_at(rows, t0, 0.1), "acc_1s": acc_at(rows, t0, 1.0)}
        out.append(rec)
        print(f"{N:>3} {a.consistency:>3} {rec['rounds']:>7} {rec['wall_s']:>7} {rec['updates_per_s']:>9} "
              f"{rec['best_f1']:>8} {rec['final_f1']:>8} {str(rec['t_f1_040']):>9} {str(rec['t_f1_042']):>9} "
              f"{str(rec['t_f1_044']):>9} {str(rec['acc_0.1s']):>8} {str(rec['acc_1s']):>7}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
