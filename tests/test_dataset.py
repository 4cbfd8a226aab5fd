"""CSV ingest, binary cache, synthetic data and the producer arrival schedule."""
import math
import os

import numpy as np
import pytest
import torch

from psx._native import host
from psx.utils import data

MOCK = "/root/reference/mockData/sample_input_data.csv"


def test_mock_csv_width_and_header_inference():
    if not os.path.exists(MOCK):
        pytest.skip("reference mock data not mounted")
    ds = data.load_csv(MOCK)
    assert ds.rows == 50 and ds.num_features == 99 and ds.Fp == 128
    assert set(ds.y.tolist()) <= {0, 1}
    raw = np.loadtxt(MOCK, delimiter=",")
    assert np.array_equal(ds.float_features().numpy(), raw[:, :-1].astype(np.float32))
    assert ds.y.tolist() == raw[:, -1].astype(int).tolist()
    assert ds.X[:, 99:].abs().sum() == 0  # zero padding


def test_header_csv_roundtrip(tmp_path):
    ds = data.synth_finefood(300, num_features=64, seed=3)
    p = tmp_path / "t.csv"
    data.write_csv(ds, str(p), header=True)
    info = host.csv_probe(str(p), 0)
    assert info.header and info.rows == 300 and info.cols == 65
    assert info.names[-1] == "Score"
    back = data.load_csv(str(p))
    assert torch.equal(back.y, ds.y)
    err = (back.float_features() - ds.float_features()).abs().max().item()
    assert err < 1e-2  # %.6g text + bf16 re-rounding


def test_binary_cache_roundtrip(tmp_path):
    ds = data.synth_finefood(100, seed=4)
    p = tmp_path / "d.psxb"
    data.save_bin(ds, str(p))
    back = data.load_any(str(p))
    assert torch.equal(back.X.view(torch.int16), ds.X.view(torch.int16)) and torch.equal(back.y, ds.y)


def test_malformed_row_is_an_error(tmp_path):
    p = tmp_path / "bad.csv"
    p.write_text("1,2,3\n4,5\n")
    with pytest.raises(Exception):
        data.load_csv(str(p))
    p.write_text("1,2,3\n4,x,1\n")
    with pytest.raises(Exception):
        data.load_csv(str(p), header="no")


def java_producer_times(rows, n_workers, p_ms):
    """Literal simulation of CsvProducer.runProducer's sleep schedule (no network latency)."""
    q = 1000 // int(p_ms)
    t = 0.0
    out = []
    count = 0
    for _ in range(rows):
        out.append(t)
        count += 1
        if count >= n_workers * 128 and count % q == 0:
            t += 1000.0
    return out


@pytest.mark.parametrize("n,p", [(4, 200), (1, 200), (4, 100), (2, 7)])
def test_arrival_schedule_matches_reference_loop(n, p):
    ref = java_producer_times(3000, n, p)
    got = [host.arrival_time_ms(r, n, p) for r in range(3000)]
    assert got == ref


def test_unthrottled_and_slow_rates():
    assert host.arrival_time_ms(10**6, 4, 0) == 0.0
    assert host.arrival_time_ms(4 * 128 + 9, 4, 2000) == 10 * 2000.0  # p > 1000: one row per p ms (Q5 fix)


def test_due_rows_round_robin_shard():
    n, p = 3, 100
    total = 5000
    # worker 1 owns rows 1, 4, 7, ...
    cnt, times = host.due_rows(1, n, p, total, 0, 2500.0, 10**6)
    expect = [r for r in range(1, total, n) if host.arrival_time_ms(r, n, p) <= 2500.0]
    assert cnt == len(expect)
    assert list(times[:cnt]) == [host.arrival_time_ms(r, n, p) for r in expect]


def test_synthetic_finefood_shape():
    ds = data.synth_finefood(5000, seed=0)
    assert ds.num_features == 1024 and ds.Fp == 1024
    y = ds.y.numpy()
    assert set(np.unique(y)) == {1, 2, 3, 4, 5}
    frac2 = (y == 2).mean()
    assert 0.13 < frac2 < 0.18  # 14.8k of 94.8k
    norms = ds.float_features().norm(dim=1)
    assert torch.allclose(norms, torch.ones_like(norms), atol=2e-2)


def test_bf16_conversion_rne():
    for v in [1.0, 1.00390625, 1.01171875, -3.5, 1e-3]:
        b = host.f32_to_bf16(v)
        ref = torch.tensor([v], dtype=torch.float32).to(torch.bfloat16).view(torch.int16).item() & 0xFFFF
        assert b == ref
    assert math.isnan(torch.tensor([host.f32_to_bf16(float("nan"))], dtype=torch.int32).to(torch.int16)
                      .view(torch.bfloat16).float().item())
