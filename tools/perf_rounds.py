"""Per-round host vs device time of the bench configuration (logs-perf.csv
summary): is the round host-bound or device-bound?
Usage: python tools/perf_rounds.py [--model dense] [--steps N]"""
import os
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    argv = sys.argv[1:]
    a = bench.parse(argv + (["--steps", "600"] if "--steps" not in argv else []))
    from psx.runtime.engine import LocalEngine

    d = tempfile.mkdtemp()
    train, test = bench.make_data(a, "cuda:0")
    cfg = bench.build_cfg(a, 1)
    cfg.max_iters = a.steps
    cfg.perf_log = True
    cfg.log_dir = d
    eng = LocalEngine(cfg, "cuda:0", train=train, test=test)
    eng.run()
    rows = [r.split(";") for r in open(os.path.join(d, "logs-perf.csv")).read().strip().split("\n")[1:]]
    rows = rows[100:]  # skip warm-up
    cols = ["host_round_us", "ingest_us", "solve_us", "comm_us", "server_us"]
    print(f"side_eval={os.environ.get('PSX_SIDE_EVAL', '1')} rounds={len(rows)}")
    for i, c in enumerate(cols):
        v = [float(r[2 + i]) for r in rows]
        print(f"  {c:14s} median {statistics.median(v):8.1f}  p90 {sorted(v)[int(0.9 * len(v))]:8.1f}")
    print(f"  updates/s (last row) {rows[-1][-1]}")


if __name__ == "__main__":
    main()
