"""Reference CSV log schema, Java double formatting, metrics."""
import numpy as np
import pytest

from psx._native import host
from psx.utils.metrics import confusion, metrics_from_confusion


@pytest.mark.parametrize(
    "v,s",
    [(1.4005257709290158, "1.4005257709290158"), (0.10724921907524179, "0.10724921907524179"), (-1.0, "-1.0"),
     (123.0, "123.0"), (0.0, "0.0"), (1e-4, "1.0E-4"), (1.25e7, "1.25E7"), (0.001, "0.001"), (9999999.0, "9999999.0"),
     (float("nan"), "NaN")],
)
def test_java_double(v, s):
    assert host.java_double(v) == s


def test_logger_files(tmp_path):
    w = tmp_path / "logs-worker.csv"
    s = tmp_path / "logs-server.csv"
    lw = host.CsvLogger(str(w), True, True)
    ls = host.CsvLogger(str(s), False, True)
    lw.log_worker(1584302430044, 1, 0, 1.4005257709290158, 0.10724921907524179, 0.2177568177158089, 98)
    ls.log_server(1584302444085, 0, 0.1418398830648744, 0.23846627024810335)
    lw.close()
    ls.close()
    assert w.read_text().splitlines() == [
        "timestamp;partition;vectorClock;loss;fMeasure;accuracy;numTuplesSeen",
        "1584302430044;1;0;1.4005257709290158;0.10724921907524179;0.2177568177158089;98",
    ]
    assert s.read_text().splitlines() == [
        "timestamp;partition;vectorClock;loss;fMeasure;accuracy",
        "1584302444085;-1;0;-1;0.1418398830648744;0.23846627024810335",
    ]


def test_logger_append_mode(tmp_path):
    p = tmp_path / "x.csv"
    a = host.CsvLogger(str(p), True, True)
    a.log_worker(1, 0, 0, 0.5, 0.5, 0.5, 1)
    a.close()
    b = host.CsvLogger(str(p), True, False, True)
    b.log_worker(2, 1, 0, 0.5, 0.5, 0.5, 1)
    b.close()
    lines = p.read_text().splitlines()
    assert len(lines) == 3 and lines[0].startswith("timestamp") and lines[2].startswith("2;1;")


def test_reference_log_parses_with_same_schema():
    path = "/root/reference/evaluation/logs/sequential_logs-worker.csv"
    try:
        head = open(path).readline().strip()
    except OSError:
        pytest.skip("reference logs not mounted")
    assert head == "timestamp;partition;vectorClock;loss;fMeasure;accuracy;numTuplesSeen"


def test_weighted_f1_matches_sklearn():
    sk = pytest.importorskip("sklearn.metrics")
    rng = np.random.default_rng(0)
    yt = rng.integers(1, 6, 500)
    yp = np.where(rng.random(500) < 0.4, yt, rng.integers(0, 6, 500))
    f1, acc = metrics_from_confusion(confusion(yt, yp, 6))
    assert f1 == pytest.approx(sk.f1_score(yt, yp, average="weighted", labels=np.unique(yt)), abs=1e-12)
    assert acc == pytest.approx((yt == yp).mean())


def test_metrics_empty():
    assert metrics_from_confusion(np.zeros((3, 3))) == (0.0, 0.0)


def test_native_metrics_match_numpy():
    import numpy as np

    from psx import _native
    from psx.utils.metrics import metrics_from_confusion

    rng = np.random.default_rng(0)
    for K in (2, 6, 16):
        c = np.zeros((16, 16), dtype=np.int32)
        c[:K, :K] = rng.integers(0, 50, size=(K, K))
        c[0, :] = 0  # a label absent from the data
        f1, acc = _native.host.weighted_f1_accuracy(c, K)
        rf1, racc = metrics_from_confusion(c[:K, :K])
        assert abs(f1 - rf1) < 1e-12 and abs(acc - racc) < 1e-12


def test_metrics_sink_cpu_rows(tmp_path):
    import torch

    from psx.models.logreg import ModelSpec
    from psx.ops.lr import EvalScratch, EvalSet
    from psx.utils.data import synth_finefood
    from psx.utils.logsink import LogSink
    from psx.utils.metrics import metrics_from_confusion

    spec = ModelSpec(64, 6)
    te = synth_finefood(300, 64, seed=2)
    ev = EvalSet(spec, te.X, te.y, "cpu")
    w = spec.init("random", seed=3)
    wp, sp = tmp_path / "w.csv", tmp_path / "s.csv"
    log = LogSink(spec.K, "cpu", str(wp), str(sp), pool=2)  # tiny pool: exercises slot reuse / back-pressure
    scratch = EvalScratch("cpu")
    loss = torch.tensor([0.25])
    for i in range(5):
        log.worker_eval(ev, None, w, scratch, loss, 0, i, 10 * i)
        log.server_eval(ev, None, w, scratch, i)
    book = log.book
    log.close()
    conf = torch.zeros(256, dtype=torch.int32)
    ev.confusion_async(None, w, conf)
    f1, acc = metrics_from_confusion(conf.view(16, 16)[:6, :6].numpy())
    assert len(book.worker) == 5 and len(book.server) == 5
    assert [r[2] for r in book.worker] == list(range(5))
    assert all(abs(r[4] - f1) < 1e-12 and abs(r[5] - acc) < 1e-12 and r[3] == 0.25 for r in book.worker)
    assert [r[1] for r in book.server] == list(range(5))
    wl = wp.read_text().strip().splitlines()
    sl = sp.read_text().strip().splitlines()
    assert wl[0] == "timestamp;partition;vectorClock;loss;fMeasure;accuracy;numTuplesSeen" and len(wl) == 6
    assert sl[0] == "timestamp;partition;vectorClock;loss;fMeasure;accuracy" and len(sl) == 6
    assert sl[1].split(";")[1:4] == ["-1", "0", "-1"]  # server rows: partition -1, loss -1


def test_plot_logs_reads_reference_logs(tmp_path):
    """tools/plot_logs.py consumes the reference's own evaluation logs (shared
    schema) and recovers its consistency behaviour: BSP gap 1, SSP(10) gap 11."""
    import os
    import sys

    ref = "/root/reference/evaluation/logs/"
    if not os.path.exists(ref + "sequential_logs-server.csv"):
        import pytest

        pytest.skip("reference logs not present")
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import plot_logs

    s, w = plot_logs.load(ref + "sequential_")
    assert plot_logs.max_vc_gap(w) == 1
    s2, w2 = plot_logs.load(ref + "bounded_delay_10_")
    assert plot_logs.max_vc_gap(w2) == 11
    assert plot_logs.main([ref + "sequential_", "--out", str(tmp_path), "--names", "seq"]) == 0
    assert (tmp_path / "seq_accuracy.png").exists() and (tmp_path / "seq_consistency.png").exists()


def test_perf_log_and_trace(tmp_path):
    import json

    from psx.runtime.config import PSConfig
    from psx.runtime.engine import LocalEngine
    from psx.utils.data import synth_finefood

    tr, te = synth_finefood(600, num_features=128, seed=0), synth_finefood(100, num_features=128, seed=1)
    cfg = PSConfig(num_workers=2, consistency_model=0, producer_time_per_event=0, stream_mode="per_iter",
                   rows_per_iter=32, epochs=5, max_iters=5, min_buffer_size=32, max_buffer_size=64,
                   log_dir=str(tmp_path), perf_log=True, trace_path=str(tmp_path / "t.json"))
    LocalEngine(cfg, "cpu", train=tr, test=te).run()
    rows = (tmp_path / "logs-perf.csv").read_text().strip().split("\n")
    assert rows[0].startswith("round;timestamp;host_round_us") and len(rows) == 6
    assert [int(r.split(";")[0]) for r in rows[1:]] == [0, 1, 2, 3, 4]
    ev = json.loads((tmp_path / "t.json").read_text())["traceEvents"]
    assert {"ingest", "solve", "server"} <= {e["name"] for e in ev}


def test_tracer_lane_rows(tmp_path):
    """Tracer.lane_rows (the lanes loops' device phase stamps, 100 MHz ticks) -> device
    trace spans on the host timeline and one perf row per round / per update."""
    import json

    from psx.utils.trace import Tracer

    tr = Tracer(str(tmp_path / "t.json"), perf_path=str(tmp_path / "logs-perf.csv"))
    ref = (2_000_000_000, 1_000_000, 2_000_010_000)  # host ns around the probe, device ticks
    base = 1_000_000
    bsp = []
    for rnd in (4, 5):
        for lane in range(2):
            t0 = base + rnd * 10_000 + lane * 10
            bsp.append([0, rnd, lane, lane, t0, t0 + 1500, t0 + 6500 + lane * 100, t0 + 7000 + lane * 100])
    bsp.append([0, 6, 0, 0, 0, 0, 0, 0])  # a round the kernel never stamped: skipped
    tr.lane_rows(bsp, ref, ups=123.0)
    tr.lane_rows([[1, 9, 1, 3, base, base + 4000, base + 4500, 0]], ref, ups=7.0)
    tr.close()
    rows = [r.split(";") for r in (tmp_path / "logs-perf.csv").read_text().strip().split("\n")[1:]]
    assert [int(r[0]) for r in rows] == [4, 5, 9]
    # round 4: ingest 15 us, solve = the slower lane's 51 us, server 5 us, span 71.1 us
    assert float(rows[0][3]) == pytest.approx(15.0) and float(rows[0][4]) == pytest.approx(51.0)
    assert float(rows[0][6]) == pytest.approx(5.0) and float(rows[0][2]) == pytest.approx(71.1)
    assert float(rows[2][4]) == pytest.approx(40.0) and float(rows[2][6]) == pytest.approx(5.0)
    ev = json.loads((tmp_path / "t.json").read_text())["traceEvents"]
    dev = [e for e in ev if e.get("tid") == "device"]
    assert len(dev) == 2 * 2 * 3 + 2
    off_us = (ref[0] + ref[2]) / 2000.0 - ref[1] / 100.0
    s4 = [e for e in dev if e["name"] == "solve" and e["args"].get("round") == 4 and e["args"]["lane"] == 0][0]
    assert s4["ts"] == pytest.approx(off_us + (base + 40_000 + 1500) / 100.0) and s4["dur"] == pytest.approx(50.0)
