"""Full-batch learning curve of a dataset: the best test accuracy / weighted F1 a
converged softmax regression reaches from the first n training tuples.  At
matched producer rates a streaming run is data-arrival bound, so its accuracy
at time t is judged against this curve at n = tuples seen by t (the synthetic
fine-food set is absent from the reference, whose curves are on the real data).

    python tools/learning_curve.py [--ns 500,1000,...] [--out evaluation/learning_curve.json]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="500,1000,2000,3000,4000,6000,8000,12000,16000,24000,32000,90000")
    ap.add_argument("--out", default="evaluation/learning_curve.json")
    ap.add_argument("--threads", type=int, default=2)
    a = ap.parse_args()
    from ground_truth import fit_full_batch
    from psx.utils.data import FINEFOOD_TEST_ROWS, synth_finefood
    from psx.utils.metrics import confusion, metrics_from_confusion

    torch.set_num_threads(a.threads)
    ns = [int(x) for x in a.ns.split(",")]
    tr, te = synth_finefood(max(ns), seed=0), synth_finefood(FINEFOOD_TEST_ROWS, seed=1)
    rows = []
    for n in ns:
        coef, inter, _ = fit_full_batch(tr.float_features()[:n], tr.y[:n].long(), 6, 0.0, 150)
        pred = (te.float_features().double() @ coef.t() + inter).argmax(1)
        f1, acc = metrics_from_confusion(confusion(te.y.numpy(), pred.numpy(), 6))
        rows.append({"tuples": n, "test_accuracy": round(acc, 4), "test_weighted_f1": round(f1, 4)})
        print(json.dumps(rows[-1]), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
