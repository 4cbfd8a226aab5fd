"""Calibrate the synthetic fine-food signal so full-batch LR reaches ~0.47 accuracy.

Usage: python tools/calibrate_synth.py [signal ...]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from psx.utils.data import synth_finefood  # noqa: E402


def offline_lr_accuracy(signal, train_rows=30000, test_rows=4877, iters=200):
    tr = synth_finefood(train_rows, seed=0, signal=signal)
    te = synth_finefood(test_rows, seed=1, signal=signal)
    X, y = tr.float_features(), tr.y.long()
    Xt, yt = te.float_features(), te.y.long()
    W = torch.zeros(6, X.shape[1], requires_grad=True)
    b = torch.zeros(6, requires_grad=True)
    opt = torch.optim.LBFGS([W, b], max_iter=iters, line_search_fn="strong_wolfe")

    def closure():
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(X @ W.t() + b, y)
        loss.backward()
        return loss

    opt.step(closure)
    with torch.no_grad():
        acc = ((Xt @ W.t() + b).argmax(1) == yt).float().mean().item()
    return acc


if __name__ == "__main__":
    sigs = [float(s) for s in sys.argv[1:]] or [0.2, 0.3, 0.4]
    for s in sigs:
        t = time.time()
        print(f"signal={s:.3f} test_acc={offline_lr_accuracy(s):.4f} ({time.time()-t:.1f}s)", flush=True)
