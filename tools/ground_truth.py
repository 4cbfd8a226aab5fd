"""Offline ground truth: full-batch multinomial logistic regression on the
whole training set, evaluated on the test set (weighted F1 + accuracy).

The reference's offline baseline is a datawig SimpleImputer notebook
(evaluation/python-ground-truth-algorithm.ipynb:55-104, report at :378-380,
accuracy / weighted F1 ~0.47 on fine-food reviews).  datawig/MXNet are not
available here; the model class that matters for the streaming comparison is
the same softmax regression the parameter server trains, so this fits it to
convergence (float64 L-BFGS in torch, standardised features, optional L2)
and reports the ceiling the streaming runs approach.

Usage:
  python tools/ground_truth.py --train data/train.csv --test data/test.csv
  python tools/ground_truth.py --synthetic [--rows 90000 --test_rows 4877]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from psx.utils.data import load_csv, synth_finefood  # noqa: E402
from psx.utils.metrics import confusion, metrics_from_confusion  # noqa: E402


def fit_full_batch(X: torch.Tensor, y: torch.Tensor, K: int, l2: float = 0.0, iters: int = 200):
    """Standardised full-batch softmax regression (float64 L-BFGS, strong Wolfe)."""
    X = X.double()
    mu = X.mean(0)
    sd = X.std(0, unbiased=True)
    live = sd > 0
    Xs = torch.where(live, (X - mu) / torch.where(live, sd, torch.ones_like(sd)), torch.zeros_like(X))
    W = torch.zeros(K, X.shape[1], dtype=torch.float64, requires_grad=True)
    b = torch.zeros(K, dtype=torch.float64, requires_grad=True)
    opt = torch.optim.LBFGS([W, b], lr=1.0, max_iter=iters, history_size=10, line_search_fn="strong_wolfe",
                            tolerance_grad=1e-9, tolerance_change=1e-12)

    def closure():
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(Xs @ W.t() + b, y) + 0.5 * l2 * (W * W).sum()
        loss.backward()
        return loss

    opt.step(closure)
    with torch.no_grad():
        loss = torch.nn.functional.cross_entropy(Xs @ W.t() + b, y) + 0.5 * l2 * (W * W).sum()
        coef = torch.where(live, W / torch.where(live, sd, torch.ones_like(sd)), torch.zeros_like(W))
        inter = b - coef @ mu
    return coef, inter, float(loss)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--train", default=None)
    ap.add_argument("--test", default=None)
    ap.add_argument("--synthetic", action="store_true", help="fine-food-shaped synthetic data (no CSV)")
    ap.add_argument("--rows", type=int, default=90000)
    ap.add_argument("--test_rows", type=int, default=4877)
    ap.add_argument("--features", type=int, default=1024)
    ap.add_argument("--l2", type=float, default=0.0)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args(argv)
    if a.synthetic or not a.train:
        tr = synth_finefood(a.rows, num_features=a.features, seed=0)
        te = synth_finefood(a.test_rows, num_features=a.features, seed=1)
    else:
        tr = load_csv(a.train)
        te = load_csv(a.test or a.train)
    K = int(max(int(tr.y.max()), int(te.y.max())) + 1)
    coef, inter, loss = fit_full_batch(tr.float_features(), tr.y.long(), K, a.l2, a.iters)
    pred = (te.float_features().double() @ coef.t() + inter).argmax(1)
    c = confusion(te.y.numpy(), pred.numpy(), K)
    f1, acc = metrics_from_confusion(c)
    out = {"train_rows": int(tr.rows), "test_rows": int(te.rows), "features": int(tr.num_features), "classes": K,
           "train_loss": round(loss, 6), "test_accuracy": round(acc, 4), "test_weighted_f1": round(f1, 4),
           "per_class_recall": np.round(np.diag(c) / np.maximum(c.sum(1), 1), 4).tolist()}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
