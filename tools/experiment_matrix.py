"""The reference's 8-experiment matrix at MATCHED producer rates, plus the
side-by-side table against the reference's own logs.

Reference runs (evaluation/logs/*.csv, README.md:237-326):
  single-worker 5 tps; 4 workers at 0.5 / 2.5 / 5 / 10 tps per worker (c = 0);
  sequential (c=0), bounded delay 10 (c=10), eventual (c=-1) at run.sh's -p 200.
-p is the TOTAL rate (floor(1000/p) rows/s after a burst of N*128 rows,
CsvProducer.java:73-83), so "X tps per worker" with N workers is p = 1000/(X*N).

Each run is the in-process engine (server + N workers) via the ServerAppRunner
CLI, for --seconds of wall clock, writing the reference's log schema; the runs
are independent processes started together.  Metrics follow SURVEY.md
Appendix C: accuracy@t = last server row with ts - t0 <= t (t0 = first log row),
time to server F1 >= 0.40, peak server F1, updates/s = worker rows / span.

    python tools/experiment_matrix.py --device cpu --seconds 600 --out evaluation/psx_logs
    python tools/experiment_matrix.py --table-only --out evaluation/psx_logs
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/evaluation/logs"

# name, reference log prefix, workers, -p (ms per event, total rate), -c
RUNS = [
    ("single-worker_5tps", "single-worker_5tps", 1, 200.0, 0),
    ("4-workers_0-5tps", "4-workers_0-5tps", 4, 500.0, 0),
    ("4-workers_2-5tps", "4-workers_2-5tps", 4, 100.0, 0),
    ("4-workers_5tps", "4-workers_5tps", 4, 50.0, 0),
    ("4-workers_10tps", "4-workers_10tps", 4, 25.0, 0),
    ("sequential", "sequential", 4, 200.0, 0),
    ("bounded_delay_10", "bounded_delay_10", 4, 200.0, 10),
    ("eventual", "eventual", 4, 200.0, -1),
]
MARKS = (60, 120, 300, 600, 1200)


def ensure_data(out_dir: str):
    from psx.utils.data import FINEFOOD_TEST_ROWS, save_bin, synth_finefood

    os.makedirs(out_dir, exist_ok=True)
    tr, te = os.path.join(out_dir, "train.bin"), os.path.join(out_dir, "test.bin")
    if not os.path.exists(tr):
        save_bin(synth_finefood(90000, seed=0), tr)
        save_bin(synth_finefood(FINEFOOD_TEST_ROWS, seed=1), te)
    return tr, te


def launch(a, tr, te):
    """The selected runs as independent processes, at most a.max_concurrent at a time."""
    todo = [r for r in RUNS if not a.runs or r[0] in a.runs.split(",")]
    procs = []

    def start(name, n, p, c):
        d = os.path.join(a.out, name)
        os.makedirs(d, exist_ok=True)
        env = dict(os.environ, OMP_NUM_THREADS=str(a.threads), PYTHONPATH=ROOT)
        cmd = [sys.executable, "-m", "psx.apps.server_app_runner", "--inprocess", "--device", a.device,
               "-training", tr, "-test", te, "-p", str(p), "-c", str(c), "--num_workers", str(n), "-l",
               "--log_dir", d, "--max_wallclock_s", str(a.seconds), "--async_scheduler", "threads",
               "--iter_new_rows", str(a.iter_new_rows), "--iter_new_frac", str(a.iter_new_frac),
               "--iter_new_cap", str(a.iter_new_cap), "--iter_new_ramp", str(a.iter_new_ramp)]
        procs.append((name, subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=open(os.path.join(d, "run.out"), "w"),
                                             stderr=subprocess.STDOUT)))

    t0 = time.time()
    while todo or any(p.poll() is None for _, p in procs):
        while todo and sum(p.poll() is None for _, p in procs) < a.max_concurrent:
            name, _, n, p, c = todo.pop(0)
            start(name, n, p, c)
        time.sleep(15)
        print(f"[matrix] {time.time() - t0:.0f} s, running: {[n for n, p in procs if p.poll() is None]}", flush=True)
    return {n: p.returncode for n, p in procs}


def _log(prefix: str, kind: str) -> str:
    p = prefix + f"logs-{kind}.csv"
    return p if os.path.exists(p) else p + ".gz"  # committed logs are gzipped when large


def metrics(prefix: str) -> dict:
    import pandas as pd

    s = pd.read_csv(_log(prefix, "server"), sep=";")
    w = pd.read_csv(_log(prefix, "worker"), sep=";")
    t0 = min(s.timestamp.min(), w.timestamp.min())
    s = s.sort_values("timestamp")
    out = {"span_s": (max(s.timestamp.max(), w.timestamp.max()) - t0) / 1000.0}
    for t in MARKS:
        r = s[s.timestamp - t0 <= t * 1000]
        out[f"acc@{t}"] = float(r.accuracy.iloc[-1]) if len(r) and out["span_s"] >= t else None
    hit = s[s.fMeasure >= 0.40]
    out["t_f1_040"] = float((hit.timestamp.iloc[0] - t0) / 1000.0) if len(hit) else None
    out["peak_f1"] = float(s.fMeasure.max())
    out["peak_acc"] = float(s.accuracy.max())
    wspan = (w.timestamp.max() - w.timestamp.min()) / 1000.0
    out["updates_per_s"] = float(len(w) / wspan) if wspan > 0 else None
    out["tuples"] = int(w.groupby("partition").numTuplesSeen.max().sum())
    return out


def fmt(v, d=3):
    return "-" if v is None else (f"{v:.{d}f}" if isinstance(v, float) else str(v))


def table(out_dir: str) -> str:
    lines = ["| run | who | " + " | ".join(f"acc@{t}s" for t in MARKS) +
             " | time to F1>=0.40 | peak F1 | updates/s | tuples seen |",
             "|---|---|" + "---|" * (len(MARKS) + 4)]
    res = {}
    for name, ref, n, p, c in RUNS:
        for who, prefix in (("reference", os.path.join(REF, ref + "_")), ("psx", os.path.join(out_dir, name) + "/")):
            if not os.path.exists(_log(prefix, "server")):
                continue
            m = metrics(prefix)
            res[f"{name}/{who}"] = m
            lines.append(f"| {name} (N={n}, -p {p:g}, -c {c}) | {who} | " +
                         " | ".join(fmt(m[f'acc@{t}']) for t in MARKS) +
                         f" | {fmt(m['t_f1_040'], 1)} s | {fmt(m['peak_f1'])} | {fmt(m['updates_per_s'], 2)} |"
                         f" {m['tuples']} |")
    with open(os.path.join(out_dir, "matrix.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--seconds", type=float, default=600.0)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--out", default="evaluation/psx_logs")
    ap.add_argument("--table-only", action="store_true")
    ap.add_argument("--iter_new_frac", type=float, default=0.5,
                    help="worker cadence: iterate once this fraction of the window is new (the CLI default 0.5; "
                         "0: continuously)")
    ap.add_argument("--iter_new_cap", type=int, default=128, help="cap of the new tuples per iteration (CLI default)")
    ap.add_argument("--runs", default="", help="comma-separated run names (default: all 8)")
    ap.add_argument("--max-concurrent", dest="max_concurrent", type=int, default=8,
                    help="engines running at once (on one GPU every one is a process of its own)")
    ap.add_argument("--iter_new_ramp", type=int, default=0, help="first solves wait for R, 2R, 4R, ... new tuples")
    ap.add_argument("--iter_new_rows", type=int, default=0,
                    help="worker cadence: iterate after this many new tuples (0: continuously, the reference's way)")
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    os.makedirs(a.out, exist_ok=True)
    if not a.table_only:
        tr, te = ensure_data(os.path.join(ROOT, "data"))
        rcs = launch(a, tr, te)
        print("[matrix] exit codes", rcs, flush=True)
    t = table(a.out)
    with open(os.path.join(a.out, "matrix.md"), "w") as fh:
        fh.write(t + "\n")
    print(t)


if __name__ == "__main__":
    main()
