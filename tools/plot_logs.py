"""Plots and summary tables from parameter-server CSV logs.

Reproduces the reference's evaluation notebooks (reference:
evaluation/plot-generation.ipynb, evaluation/evaluation-multipleDatasetsAtOnce.ipynb)
from logs in the shared schema (server: timestamp;partition;vectorClock;loss;
fMeasure;accuracy -- worker: ...;numTuplesSeen):

* per-run: worker train loss, weighted F1 and accuracy (server + workers) vs
  "overall tuples seen" (at vector clock v: the sum over workers of their
  numTuplesSeen at v, the notebook's x axis), truncated to the smallest
  maximum vector clock over all partitions (plot-generation.ipynb cell 5);
* per-run: iteration (vector clock) vs wall-clock per partition -- the
  consistency-model scatter of docs/plots/consistency_model_*.png;
* several runs at once: server accuracy / F1 curves overlaid
  (evaluation-multipleDatasetsAtOnce.ipynb);
* a markdown summary (rows, max vc, final/best server metrics, worker
  updates/s, max in-flight vector-clock gap between workers).

Usage:
  python tools/plot_logs.py PREFIX [PREFIX ...] [--out DIR] [--names a,b,...]
where PREFIX + "logs-server.csv" / PREFIX + "logs-worker.csv" are the files
(e.g. ./ for ./logs-server.csv, or /root/reference/evaluation/logs/sequential_).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import pandas as pd


def load(prefix: str):
    s = pd.read_csv(prefix + "logs-server.csv", sep=";")
    w = pd.read_csv(prefix + "logs-worker.csv", sep=";")
    return s, w


def tuples_curve(s: pd.DataFrame, w: pd.DataFrame):
    """Per-partition frames with the notebook's 'overall tuples seen' x axis."""
    parts = sorted(int(p) for p in w["partition"].unique())
    max_vc = min([int(w[w.partition == p].vectorClock.max()) for p in parts] + [int(s.vectorClock.max())])
    w = w[w.vectorClock <= max_vc]
    s = s[s.vectorClock <= max_vc]
    per_vc = w.groupby("vectorClock")["numTuplesSeen"].sum()
    overall = per_vc.reindex(range(max_vc + 1)).ffill().fillna(0)
    out = {}
    for p in parts:
        d = w[w.partition == p].sort_values("vectorClock").copy()
        d["overall"] = overall.loc[d.vectorClock.values].values
        out[p] = d
    ds = s.sort_values("vectorClock").copy()
    ds["overall"] = overall.loc[ds.vectorClock.values].values
    return out, ds, max_vc


def max_vc_gap(w: pd.DataFrame) -> int:
    """Largest difference between workers' latest vector clocks over time
    (the reference validates consistency models this way: README.md:299-321)."""
    w = w.sort_values("timestamp")
    latest, gap = {}, 0
    parts = w["partition"].unique()
    for p, vc in zip(w["partition"].values, w["vectorClock"].values):
        latest[p] = vc
        if len(latest) == len(parts):
            vals = list(latest.values())
            gap = max(gap, max(vals) - min(vals))
    return int(gap)


def summary(name: str, s: pd.DataFrame, w: pd.DataFrame) -> dict:
    span = (w.timestamp.max() - w.timestamp.min()) / 1000.0 if len(w) > 1 else float("nan")
    return {
        "run": name,
        "worker_rows": len(w),
        "server_rows": len(s),
        "workers": int(w.partition.nunique()),
        "max_vc": int(w.vectorClock.max()) if len(w) else 0,
        "final_server_acc": float(s.accuracy.iloc[-1]) if len(s) else float("nan"),
        "best_server_acc": float(s.accuracy.max()) if len(s) else float("nan"),
        "final_server_f1": float(s.fMeasure.iloc[-1]) if len(s) else float("nan"),
        "best_server_f1": float(s.fMeasure.max()) if len(s) else float("nan"),
        "worker_updates_per_s": len(w) / span if span and span > 0 else float("nan"),
        "max_worker_vc_gap": max_vc_gap(w),
    }


def plot_run(name: str, s, w, out_dir: str, plt):
    curves, ds, max_vc = tuples_curve(s, w)
    files = []
    for metric, col, title in (("loss", "loss", "Losses on train data (workers)"),
                               ("f1", "fMeasure", "weighted f1-score on test data"),
                               ("accuracy", "accuracy", "accuracy on test data")):
        fig = plt.figure(figsize=(8, 6), dpi=120)
        for p, d in curves.items():
            plt.plot(d["overall"], d[col], linewidth=0.6, alpha=0.5 if metric != "loss" else 0.8,
                     label=f"worker{p + 1}")
        if metric != "loss":
            plt.plot(ds["overall"], ds[col], linewidth=1.2, color="black", label="server")
        plt.title(f"{title} [{name}]")
        plt.xlabel("Overall num tuples seen")
        plt.ylabel(col)
        plt.legend(loc="best", ncol=2, fontsize=7)
        f = os.path.join(out_dir, f"{name}_{metric}.png")
        fig.savefig(f)
        plt.close(fig)
        files.append(f)
    fig = plt.figure(figsize=(8, 6), dpi=120)
    t0 = min(w.timestamp.min(), s.timestamp.min() if len(s) else w.timestamp.min())
    for p, d in w.groupby("partition"):
        plt.scatter((d.timestamp - t0) / 1000.0, d.vectorClock, s=3, label=f"partition {p + 1}")
    plt.title(f"iterations over time [{name}]")
    plt.xlabel("seconds")
    plt.ylabel("vector clock")
    plt.legend(loc="best", fontsize=7)
    f = os.path.join(out_dir, f"{name}_consistency.png")
    fig.savefig(f)
    plt.close(fig)
    files.append(f)
    return files


def plot_overlay(runs, out_dir: str, plt):
    files = []
    for col, title in (("accuracy", "server accuracy"), ("fMeasure", "server weighted f1")):
        fig = plt.figure(figsize=(8, 6), dpi=120)
        for name, s, w in runs:
            _, ds, _ = tuples_curve(s, w)
            plt.plot(ds["overall"], ds[col], linewidth=1.0, label=name)
        plt.title(title)
        plt.xlabel("Overall num tuples seen")
        plt.ylabel(col)
        plt.legend(loc="best", fontsize=7)
        f = os.path.join(out_dir, f"overlay_{col}.png")
        fig.savefig(f)
        plt.close(fig)
        files.append(f)
    return files


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("prefixes", nargs="+")
    ap.add_argument("--out", default="plots")
    ap.add_argument("--names", default=None, help="comma-separated run names (default: from the prefixes)")
    ap.add_argument("--no-plots", action="store_true", help="summary table only")
    a = ap.parse_args(argv)
    names = a.names.split(",") if a.names else [os.path.basename(p.rstrip("_/")) or "run" for p in a.prefixes]
    runs = [(n, *load(p)) for n, p in zip(names, a.prefixes)]
    rows = [summary(n, s, w) for n, s, w in runs]
    cols = list(rows[0].keys())
    print("| " + " | ".join(cols) + " |")
    print("|" + "---|" * len(cols))
    for r in rows:
        print("| " + " | ".join(f"{r[c]:.4g}" if isinstance(r[c], float) else str(r[c]) for c in cols) + " |")
    if not a.no_plots:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        os.makedirs(a.out, exist_ok=True)
        files = []
        for n, s, w in runs:
            files += plot_run(n, s, w, a.out, plt)
        if len(runs) > 1:
            files += plot_overlay(runs, a.out, plt)
        print(f"wrote {len(files)} plots to {a.out}", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
