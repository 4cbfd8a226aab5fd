"""CPU simulation of the reference's single-worker streaming protocol at its
matched producer rate, on a synthetic data set -- used to check how learnable a
data set is under the reference's own algorithm (not the engine's speed).

Protocol (reference README.md:237-260, evaluation/logs/single-worker_5tps):
the producer bursts 128 rows, then emits 5 rows/s; the worker's window is the
last 128 rows (SlidingBuffer); each iteration is one local solve (2 L-BFGS
iterations from the current model, LogisticRegressionTaskSpark.java) whose
delta the server adds (one worker: w = w_new).  The reference managed 0.76
iterations/s, i.e. ~6.6 new rows per iteration; accuracy is reported on the
test set at given numbers of tuples seen.

    python tools/stream_sim.py [--rows-per-iter 7] [--marks 300,600,1500,3000,5449]
    python tools/stream_sim.py --variant zipf --signal 0.1 --class-zipf 1.0
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def simulate(tr, te, window=128, rows_per_iter=7, marks=(300, 600, 1500, 3000, 5449), workers=1,
             lr: float | None = None):
    """Returns [(tuples, test accuracy)] at each mark.  With workers > 1 every
    worker solves over its own partition's window from the same global model
    (sequential consistency: the server adds each delta with lr = 1/N,
    ServerProcessor.java:148-151)."""
    from psx.models.reference import local_solve_reference
    from psx.utils.metrics import confusion, metrics_from_confusion

    X = tr.float_features().double()
    y = tr.y.long()
    Xt = te.float_features().double()
    K, F = 6, X.shape[1]
    coef = torch.zeros(K, F, dtype=torch.float64)
    inter = torch.zeros(K, dtype=torch.float64)
    seen = window * workers
    out, mi = [], 0
    while mi < len(marks) and seen <= X.shape[0]:
        dc = torch.zeros_like(coef)
        di = torch.zeros_like(inter)
        for w in range(workers):
            # worker w's partition is every workers-th row (the producer's round robin)
            part = torch.arange(w, seen, workers)[-window:]
            r = local_solve_reference(X[part], y[part], coef, inter, iters=2)
            dc += r.coef - coef
            di += r.intercept - inter
        step = 1.0 / workers if lr is None else lr
        coef, inter = coef + step * dc, inter + step * di
        seen += rows_per_iter * workers
        while mi < len(marks) and seen >= marks[mi]:
            pred = (Xt @ coef.t() + inter).argmax(1)
            f1, acc = metrics_from_confusion(confusion(te.y.numpy(), pred.numpy(), K))
            out.append({"tuples": marks[mi], "acc": round(acc, 4), "f1": round(f1, 4)})
            mi += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-per-iter", type=int, default=7)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--window", type=int, default=128)
    ap.add_argument("--lr", type=float, default=None, help="server step (default 1/workers)")
    ap.add_argument("--marks", default="300,600,1500,3000,5449")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--train-rows", type=int, default=12000)
    ap.add_argument("--kw", default="{}", help="JSON keyword arguments for synth_finefood")
    a = ap.parse_args()
    from psx.utils.data import FINEFOOD_TEST_ROWS, synth_finefood

    torch.set_num_threads(a.threads)
    kw = json.loads(a.kw)
    tr = synth_finefood(a.train_rows, seed=0, **kw)
    te = synth_finefood(FINEFOOD_TEST_ROWS, seed=1, **kw)
    t = time.time()
    res = simulate(tr, te, window=a.window, rows_per_iter=a.rows_per_iter, workers=a.workers, lr=a.lr,
                   marks=tuple(int(m) for m in a.marks.split(",")))
    print(json.dumps({"kw": kw, "workers": a.workers, "curve": res, "s": round(time.time() - t, 1)}), flush=True)


if __name__ == "__main__":
    main()
