"""Classification metrics with Spark MulticlassMetrics semantics.

Reference: Metrics.java:15-24 uses MulticlassClassificationEvaluator with metric
names "f1" (= weightedFMeasure) and "accuracy".  weightedFMeasure sums, over
the labels that occur in the data, (label count / total) * F1(label), where a
label's precision/recall is 0 when its denominator is 0.
"""
from __future__ import annotations

import numpy as np


def metrics_from_confusion(conf) -> tuple[float, float]:
    """(weighted F1, accuracy) from a confusion matrix [true][pred]."""
    c = np.asarray(conf, dtype=np.float64)
    total = c.sum()
    if total <= 0:
        return 0.0, 0.0
    tp = np.diag(c)
    true_count = c.sum(axis=1)
    pred_count = c.sum(axis=0)
    with np.errstate(divide="ignore", invalid="ignore"):
        prec = np.where(pred_count > 0, tp / pred_count, 0.0)
        rec = np.where(true_count > 0, tp / true_count, 0.0)
        f1 = np.where(prec + rec > 0, 2 * prec * rec / (prec + rec), 0.0)
    wf1 = float((true_count / total * f1).sum())
    acc = float(tp.sum() / total)
    return wf1, acc


def confusion(y_true, y_pred, num_classes: int) -> np.ndarray:
    y_true = np.asarray(y_true, dtype=np.int64)
    y_pred = np.asarray(y_pred, dtype=np.int64)
    m = np.zeros((num_classes, num_classes), dtype=np.int64)
    np.add.at(m, (y_true, y_pred), 1)
    return m
