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
