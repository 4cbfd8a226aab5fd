"""Local solver: the device control state machine (host build) vs the independent
two-loop L-BFGS reference, plus Spark-semantics properties."""
import numpy as np
import pytest
import torch

from psx._native import host
from psx.models.logreg import ModelSpec, from_reference_layout, to_reference_layout
from psx.models.reference import feature_std, local_solve_reference, multinomial_loss_grad
from psx.utils.data import synth_binary, synth_finefood


def emulate_device(X, y, coef_old, b_old, iters=2, hist=10, ls_max=4, mode="lbfgs", gd_lr=1.0, center=True,
                   zero_const=True, tol=1e-6):
    """Float64 emulation of the kernel chain prep -> [eval, reduce, update] x slots -> finalize,
    driving the REAL device state machine (solver_ctrl.h compiled for the host)."""
    X = X.double()
    y = y.long()
    K, F = coef_old.shape
    P = K * F + K
    cfg = host.SolverCfg()
    cfg.K, cfg.F, cfg.Fp, cfg.P, cfg.cap = K, F, F, P, X.shape[0]
    cfg.iters, cfg.hist, cfg.ls_max = iters, hist, ls_max
    cfg.mode = 1 if mode == "gd" else 0
    cfg.center, cfg.zero_const, cfg.gd_lr, cfg.tol = int(center), int(zero_const), gd_lr, tol
    cfg.nslots = 1 + iters * (1 if mode == "gd" else ls_max)
    ctrl = host.SolverCtrl()
    sd = feature_std(X)
    live = sd > 0
    inv = torch.where(live, 1.0 / torch.where(live, sd, torch.ones_like(sd)), torch.zeros_like(sd))
    w_old = coef_old.double()
    wfix = torch.zeros_like(w_old) if zero_const else torch.where(live, torch.zeros_like(w_old), w_old)
    x = torch.cat([(w_old * sd).reshape(-1), b_old.double()])
    d = torch.zeros(P, dtype=torch.float64)
    g_c = torch.zeros(P, dtype=torch.float64)
    S = torch.zeros(hist, P, dtype=torch.float64)
    Y = torch.zeros(hist, P, dtype=torch.float64)
    t_trial = 0.0
    for slot in range(cfg.nslots):
        if ctrl.phase == host.kPhDone:
            break
        v = x + t_trial * d
        c, b = v[: K * F].view(K, F), v[K * F:]
        f, gc_, gb = multinomial_loss_grad(X, y, c * inv + wfix, b)
        g_t = torch.cat([(gc_ * inv).reshape(-1), gb])
        m, head = ctrl.m, ctrl.head
        dots = [float(g_t @ g_t), float(g_t @ d), float(g_t @ g_c)] + [0.0] * (2 * hist)
        for i in range(hist):
            valid = m > 0 and (m == hist or ((i - (head - m + 1)) % hist) < m)
            if valid:
                dots[3 + i] = float(S[i] @ g_t)
                dots[3 + hist + i] = float(Y[i] @ g_t)
        ctrl.step(cfg, float(f), dots, slot)
        if ctrl.action_slot != slot:
            continue
        a = ctrl.action
        if a == host.kActDone:
            break
        if a == host.kActInit:
            g_c = g_t.clone()
            d = ctrl.cg * g_c
        elif a in (host.kActAccept, host.kActAcceptDone):
            dold = d
            x = x + ctrl.t_acc * dold
            if a == host.kActAcceptDone:
                break
            if ctrl.push_slot >= 0:
                S[ctrl.push_slot] = ctrl.t_acc * dold
                Y[ctrl.push_slot] = g_t - g_c
            g_c = g_t.clone()
            cs, cy = ctrl.cs, ctrl.cy
            d = ctrl.cg * g_c
            for i in range(hist):
                if cs[i] != 0.0:
                    d = d + cs[i] * S[i]
                if cy[i] != 0.0:
                    d = d + cy[i] * Y[i]
        t_trial = ctrl.t
    c, b = x[: K * F].view(K, F), x[K * F:]
    coef = torch.where(live, c * inv, wfix)
    if center:
        coef = coef - coef.mean(0, keepdim=True)
        b = b - b.mean()
    return coef, b, ctrl


CASES = [
    dict(iters=2), dict(iters=8), dict(iters=15, hist=3), dict(iters=3, mode="gd", gd_lr=0.7),
    dict(iters=4, zero_const=False), dict(iters=2, center=False), dict(iters=6, ls_max=2),
]


@pytest.mark.parametrize("kw", CASES)
def test_device_state_machine_matches_two_loop_reference(kw):
    ds = synth_finefood(400, num_features=96, seed=11)
    spec = ModelSpec(96, 6)
    g = torch.Generator().manual_seed(1)
    coef_old = torch.randn(6, 96, generator=g) * 0.05
    b_old = torch.randn(6, generator=g) * 0.05
    X = ds.float_features()
    X[:, 5] = 0.25  # a constant feature (std 0) exercises the zero_const path
    ref = local_solve_reference(X, ds.y, coef_old, b_old, **kw)
    coef, b, ctrl = emulate_device(X, ds.y, coef_old, b_old, **kw)
    scale = max(ref.coef.abs().max().item(), 1e-9)
    assert (coef.float() - ref.coef).abs().max().item() / scale < 1e-5
    assert (b.float() - ref.intercept).abs().max().item() < 1e-5 * max(1.0, ref.intercept.abs().max().item())
    assert ctrl.nacc == ref.accepted and ctrl.evals == ref.evals
    assert ctrl.f_c == pytest.approx(ref.loss, rel=1e-6)  # gd_lr travels as float32
    if spec and kw.get("zero_const", True):
        assert ref.coef[:, 5].abs().max() == 0  # Spark: zero-variance feature -> coefficient 0


def test_two_iterations_reduce_loss_and_center():
    ds = synth_finefood(800, num_features=128, seed=2)
    X, y = ds.float_features(), ds.y
    coef0, b0 = torch.zeros(6, 128), torch.zeros(6)
    res = local_solve_reference(X, y, coef0, b0, iters=2)
    sd = feature_std(X.double())
    live = sd > 0
    loss0, _, _ = multinomial_loss_grad(X.double(), y.long(), coef0.double(), b0.double())
    assert res.loss < float(loss0)
    assert res.accepted == 2
    assert torch.allclose(res.coef.sum(0), torch.zeros(128), atol=1e-5)  # centred across classes
    assert abs(float(res.intercept.sum())) < 1e-5
    assert torch.allclose(res.delta_coef, res.coef - coef0)


def test_binary_labels_mock_shape():
    ds = synth_binary(50, 99, seed=0)
    res = local_solve_reference(ds.float_features(), ds.y, torch.zeros(2, 99), torch.zeros(2), iters=10)
    pred = (ds.float_features() @ res.coef.t() + res.intercept).argmax(1)
    assert (pred == ds.y.long()).float().mean() > 0.8


def test_reference_layout_roundtrip():
    spec = ModelSpec(1024, 6)
    assert spec.P_ref == 6150  # LogisticRegressionTaskSpark.java:101
    w = spec.init("random", seed=3)
    ref = to_reference_layout(spec, w)
    # flat index k <-> class k % K, feature k // K (column-major 6 x 1024)
    coef = spec.coef(w)
    assert ref[7].item() == coef[7 % 6, 7 // 6].item()
    assert torch.equal(from_reference_layout(spec, ref), w)


def test_solver_ctrl_rejects_short_dots():
    cfg = host.SolverCfg()
    cfg.hist = 10
    with pytest.raises(Exception):
        host.SolverCtrl().step(cfg, 1.0, [0.0] * 5, 0)
