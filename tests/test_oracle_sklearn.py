"""The float64 solve oracle (psx/models/reference.py) checked against libraries
that share none of its code.

The GPU kernels are tested against that oracle (tests/test_gpu_kernels.py), so
a misreading of the reference worker's Spark fit
(LogisticRegressionTaskSpark.java:142-221: multinomial LR, standardisation,
regParam 0, intercepts, centring) common to both would pass those tests.  Here
the oracle's pieces are pinned independently:

* the objective and its gradient against sklearn's ``log_loss`` and torch
  autograd;
* the optimum the L-BFGS iterations head to: run to convergence, the oracle's
  class probabilities must match sklearn's unregularised multinomial
  ``LogisticRegression`` (a different solver -- scipy's L-BFGS-B -- on the
  unstandardised problem; with regParam 0 the optimum is the same in the
  original feature space, which is exactly what standardisation must preserve);
* centring: the returned coefficients sum to 0 over the classes per feature,
  and so do the intercepts, as Spark's multinomial fit without
  regularisation leaves them.

Spark's 2-iteration trajectory itself (Breeze's line-search details) stays
"parity unpinned": no Spark here and no fixture in the reference holds it.
"""
import numpy as np
import pytest
import torch

from psx.models.reference import local_solve_reference, multinomial_loss_grad, predict

sklearn = pytest.importorskip("sklearn")
from sklearn.linear_model import LogisticRegression  # noqa: E402
from sklearn.metrics import log_loss  # noqa: E402


def _data(n=3000, F=12, K=4, seed=0):
    """Non-separable multinomial data (labels drawn from a softmax model) with
    features of different scales and offsets, so standardisation matters."""
    g = np.random.default_rng(seed)
    scale = g.uniform(0.2, 5.0, size=F)
    mu = g.normal(size=F) * 2.0 * scale
    X = g.normal(size=(n, F)) * scale + mu
    W = g.normal(size=(K, F)) / scale * 0.4
    b = g.normal(size=K) * 0.5
    z = (X - mu) @ W.T + b
    p = np.exp(z - z.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    y = np.array([g.choice(K, p=pi) for pi in p])
    return X, y


def test_loss_and_gradient_match_sklearn_and_autograd():
    X, y = _data(n=500, F=7, K=3, seed=1)
    g = np.random.default_rng(2)
    c = torch.tensor(g.normal(size=(3, 7)) * 0.3)
    b = torch.tensor(g.normal(size=3) * 0.3)
    Xt, yt = torch.tensor(X), torch.tensor(y)
    loss, gc, gb = multinomial_loss_grad(Xt, yt, c, b)
    p = torch.softmax(Xt @ c.t() + b, dim=1).numpy()
    assert float(loss) == pytest.approx(log_loss(y, p, labels=[0, 1, 2]), rel=1e-12)
    c2, b2 = c.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(Xt @ c2.t() + b2, yt)
    ref.backward()
    torch.testing.assert_close(gc, c2.grad, rtol=1e-10, atol=1e-12)
    torch.testing.assert_close(gb, b2.grad, rtol=1e-10, atol=1e-12)


def test_binary_loss_matches_sklearn():
    X, y = _data(n=400, F=5, K=2, seed=3)
    g = np.random.default_rng(4)
    c = torch.tensor(g.normal(size=(1, 5)) * 0.3)
    b = torch.tensor([0.1])
    loss, _, _ = multinomial_loss_grad(torch.tensor(X), torch.tensor(y), c, b)
    p1 = torch.sigmoid(torch.tensor(X) @ c[0] + b).numpy()
    assert float(loss) == pytest.approx(log_loss(y, np.stack([1 - p1, p1], 1)), rel=1e-12)


def test_converged_oracle_matches_sklearn_optimum():
    # standardize=True is the worker's setting; without it this badly scaled
    # problem (offsets, scales 0.2..5) is still 0.006 away after 400 iterations
    K, F = 4, 12
    standardize = True
    X, y = _data(K=K, F=F)
    res = local_solve_reference(torch.tensor(X), torch.tensor(y), torch.zeros(K, F, dtype=torch.float64),
                                torch.zeros(K, dtype=torch.float64), iters=400, ls_max=20, tol=0.0,
                                standardize=standardize, zero_const=True)
    sk = LogisticRegression(penalty=None, solver="lbfgs", tol=1e-12, max_iter=5000).fit(X, y)
    Xt = torch.tensor(X)
    res.coef, res.intercept = res.coef.double(), res.intercept.double()
    p_ours = torch.softmax(Xt @ res.coef.t() + res.intercept, dim=1).numpy()
    p_sk = sk.predict_proba(X)
    assert np.abs(p_ours - p_sk).max() < 2e-4
    # the same optimum in parameter space once sklearn's solution is centred the same way
    coef_sk = sk.coef_ - sk.coef_.mean(0, keepdims=True)
    icpt_sk = sk.intercept_ - sk.intercept_.mean()
    np.testing.assert_allclose(res.coef.numpy(), coef_sk, atol=2e-3 * np.abs(coef_sk).max())
    np.testing.assert_allclose(res.intercept.numpy(), icpt_sk, atol=2e-3 * np.abs(icpt_sk).max())
    assert (predict(Xt, res.coef, res.intercept).numpy() == sk.predict(X)).mean() > 0.999


def test_two_iteration_solve_is_centred_and_descends():
    """The reference's actual call (setMaxIter(2)) from a non-zero pulled model:
    the loss goes down, the result is centred over classes, and delta is
    w_new - w_old (LogisticRegressionTaskSpark.java:195-218)."""
    K, F = 4, 12
    X, y = _data(K=K, F=F, seed=5)
    g = np.random.default_rng(6)
    c0 = torch.tensor(g.normal(size=(K, F)) * 0.05)
    b0 = torch.tensor(g.normal(size=K) * 0.05)
    Xt, yt = torch.tensor(X), torch.tensor(y)
    res = local_solve_reference(Xt, yt, c0, b0, iters=2, zero_const=True)
    for k in ("coef", "intercept", "delta_coef", "delta_intercept"):
        setattr(res, k, getattr(res, k).double())
    l0 = float(multinomial_loss_grad(Xt, yt, c0, b0)[0])
    l1 = float(multinomial_loss_grad(Xt, yt, res.coef, res.intercept)[0])
    assert l1 < l0
    torch.testing.assert_close(res.coef.sum(0), torch.zeros(F, dtype=torch.float64), atol=1e-6, rtol=0)
    assert abs(float(res.intercept.sum())) < 1e-6  # the oracle hands back fp32 (the device weights' dtype)
    torch.testing.assert_close(res.delta_coef, res.coef - c0)
    torch.testing.assert_close(res.delta_intercept, res.intercept - b0)
    assert res.accepted == 2
