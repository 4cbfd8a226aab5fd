"""The bench protocol's global-model F1, round by round, under the float64 CPU
oracle of the reference's solver (psx/models/reference.py, pinned to sklearn):
N workers, each fitting 2 L-BFGS iterations on a fresh window of `window` rows of
its round-robin shard from the current model, the server adding (1/N) * sum of
the deltas (ServerProcessor.java:36,148-151), unthrottled producer.

Shows where the bench's round-to-round F1 swings come from: the same period-2
oscillation appears in the oracle, so it is the algorithm's, not the kernels'.

    python tools/f1_swing_sim.py [--rounds 40] [--workers 8] [--window 1024]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--window", type=int, default=1024)
    ap.add_argument("--train-rows", type=int, default=90000)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    from psx.models.reference import local_solve_reference
    from psx.utils.data import FINEFOOD_TEST_ROWS, synth_finefood
    from psx.utils.metrics import confusion, metrics_from_confusion

    torch.set_num_threads(a.threads)
    tr, te = synth_finefood(a.train_rows, seed=0), synth_finefood(FINEFOOD_TEST_ROWS, seed=1)
    X, y, Xt = tr.float_features().double(), tr.y.long(), te.float_features().double()
    N, win, K = a.workers, a.window, 6
    torch.manual_seed(0)
    coef = torch.randn(K, X.shape[1], dtype=torch.float64) * 0.01
    inter = torch.zeros(K, dtype=torch.float64)
    shard = a.train_rows // N
    for r in range(a.rounds):
        dc, di = torch.zeros_like(coef), torch.zeros_like(inter)
        for k in range(N):
            rows = k + (torch.arange(r * win, (r + 1) * win) % shard) * N
            res = local_solve_reference(X[rows], y[rows], coef, inter, iters=2)
            dc += res.coef - coef
            di += res.intercept - inter
        coef, inter = coef + dc / N, inter + di / N
        pred = (Xt @ coef.t() + inter).argmax(1)
        f1, acc = metrics_from_confusion(confusion(te.y.numpy(), pred.numpy(), K))
        print(json.dumps({"round": r, "f1": round(f1, 4), "acc": round(acc, 4), "epoch_pos": (r * win) % shard,
                          "predicted_per_class": torch.bincount(pred, minlength=K).tolist()}), flush=True)


if __name__ == "__main__":
    main()
