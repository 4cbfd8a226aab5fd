"""PyTorch CPU reference of the worker local solve (test oracle + CPU plumbing path).

Semantics re-derived from the reference worker's Spark call
(LogisticRegressionTaskSpark.java:142-221: ``setMaxIter(2)``, initial model =
pulled weights, default ``standardization=true``, ``regParam=0``, ``tol=1e-6``)
and Spark 3.0's multinomial training:

* features are scaled by 1/std (sample std over the buffer); a feature whose
  std is 0 is excluded from the margins and its final coefficient is 0;
* L-BFGS (history 10) with a strong-Wolfe line search (c1=1e-4, c2=0.9, first
  step 1/||d||, bracket growth x1.5, cubic zoom);
* no regularisation -> coefficients are centred per feature across classes and
  the intercepts are centred;
* the worker returns delta = w_new - w_old (:195-218).

This file is an INDEPENDENT implementation of the same algorithm as the device
state machine in ``csrc/kernels/solver_ctrl.h``: it uses the textbook two-loop
recursion instead of the compact representation, and float64 throughout.  The
two are compared in tests.  Spark itself is not available here, so bitwise
parity with Spark is "parity unpinned"; the rules above are matched exactly.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch


@dataclass
class SolveResult:
    coef: torch.Tensor  # [K, F] new coefficients (centred)
    intercept: torch.Tensor  # [K]
    delta_coef: torch.Tensor
    delta_intercept: torch.Tensor
    loss: float
    evals: int
    accepted: int
    ls_fail: int


def feature_std(X: torch.Tensor) -> torch.Tensor:
    n = X.shape[0]
    if n < 2:
        return torch.zeros(X.shape[1], dtype=X.dtype)
    return X.var(dim=0, unbiased=True).clamp_min(0).sqrt()


def multinomial_loss_grad(X, y, coef_eff, b):
    """Mean cross entropy and gradients w.r.t. the effective coefficients / intercepts.

    One coefficient row (K == 1) is the binary sigmoid model with labels {0, 1}."""
    z = X @ coef_eff.t() + b
    if coef_eff.shape[0] == 1:
        zz = z[:, 0]
        yy = (y > 0).to(z.dtype)
        loss = (torch.nn.functional.softplus(zz) - yy * zz).mean()
        r = (torch.sigmoid(zz) - yy).view(-1, 1)
        n = X.shape[0]
        return loss, (r.t() @ X) / n, r.sum(0) / n
    lse = torch.logsumexp(z, dim=1)
    loss = (lse - z.gather(1, y.view(-1, 1)).squeeze(1)).mean()
    p = torch.softmax(z, dim=1)
    p[torch.arange(X.shape[0]), y] -= 1.0
    n = X.shape[0]
    return loss, (p.t() @ X) / n, p.sum(0) / n


def _interp(lt, lf, ld, rt, rf, rd):
    if lt > rt:
        lt, lf, ld, rt, rf, rd = rt, rf, rd, lt, lf, ld
    w = rt - lt
    lb, ub = lt + 0.1 * w, lt + 0.9 * w
    d1 = ld + rd - 3.0 * (lf - rf) / (lt - rt) if lt != rt else float("nan")
    rad = d1 * d1 - ld * rd
    if not (rad >= 0.0) or not (w > 0.0):
        t = lt + 0.5 * w
    else:
        d2 = math.sqrt(rad)
        den = rd - ld + 2.0 * d2
        t = rt - w * (rd + d2 - d1) / den if den != 0.0 else lt + 0.5 * w
        if t != t:
            t = lt + 0.5 * w
    return min(max(t, lb), ub)


def local_solve_reference(
    X: torch.Tensor,
    y: torch.Tensor,
    coef_old: torch.Tensor,
    intercept_old: torch.Tensor,
    *,
    iters: int = 2,
    hist: int = 10,
    ls_max: int = 4,
    nslots: int | None = None,
    mode: str = "lbfgs",
    gd_lr: float = 1.0,
    center: bool = True,
    zero_const: bool = True,
    tol: float = 1e-6,
    standardize: bool = True,
) -> SolveResult:
    """Run the worker's local solve on a buffer (X: [B, F] float, y: [B] int)."""
    X = X.double()
    y = y.long()
    K, F = coef_old.shape
    if nslots is None:
        nslots = 1 + iters * (1 if mode == "gd" else ls_max)
    w_old = coef_old.double()
    b_old = intercept_old.double()
    sd = feature_std(X) if standardize else torch.ones(X.shape[1], dtype=X.dtype)
    live = sd > 0
    inv = torch.where(live, 1.0 / torch.where(live, sd, torch.ones_like(sd)), torch.zeros_like(sd))
    wfix = torch.zeros_like(w_old) if zero_const else torch.where(live, torch.zeros_like(w_old), w_old)

    def unpack(v):
        return v[: K * F].view(K, F), v[K * F :]

    def fg(v):
        c, b = unpack(v)
        loss, gc, gb = multinomial_loss_grad(X, y, c * inv + wfix, b)
        return float(loss), torch.cat([(gc * inv).reshape(-1), gb])

    x = torch.cat([(w_old * sd).reshape(-1), b_old])
    evals = 0
    accepted = 0
    ls_fail = 0
    slot = 0

    f_c, g_c = fg(x)
    evals += 1
    slot += 1
    S, Yh = [], []
    gnorm = float(g_c.norm())
    it = 0
    if math.isfinite(f_c) and gnorm > 0 and iters > 0:
        d = -g_c.clone()
        dg0 = float(g_c @ d)
        t = gd_lr if mode == "gd" else 1.0 / gnorm
        while True:
            # ---- one line search (or one GD step) ----
            lo = (0.0, f_c, dg0)
            hi = None
            zoom = False
            ls_i = 0
            accepted_t = None
            done = False
            while True:
                x_t = x + t * d
                f_t, g_t = fg(x_t)
                evals += 1
                slot_now = slot
                slot += 1
                if mode == "gd":
                    accepted_t = t
                    break
                dd = float(g_t @ d)
                ls_i += 1
                finite = math.isfinite(f_t)
                armijo = finite and f_t <= f_c + 1e-4 * t * dg0
                tn = t
                if not zoom:
                    if not finite:
                        tn = t * 0.5
                    elif (not armijo) or (f_t >= lo[1] and ls_i > 1):
                        hi = (t, f_t, dd)
                        zoom = True
                        tn = _interp(*lo, *hi)
                    elif abs(dd) <= 0.9 * abs(dg0):
                        accepted_t = t
                        break
                    elif dd >= 0:
                        hi = lo
                        lo = (t, f_t, dd)
                        zoom = True
                        tn = _interp(*lo, *hi)
                    else:
                        lo = (t, f_t, dd)
                        tn = t * 1.5
                else:
                    if (not armijo) or f_t >= lo[1]:
                        hi = (t, f_t, dd)
                    else:
                        if abs(dd) <= 0.9 * abs(dg0):
                            accepted_t = t
                            break
                        if dd * (hi[0] - lo[0]) >= 0:
                            hi = lo
                        lo = (t, f_t, dd)
                    tn = _interp(*lo, *hi)
                out_of_slots = slot_now + 1 >= nslots
                if ls_i >= ls_max or out_of_slots:
                    ls_fail += 1
                    if armijo and f_t < f_c:
                        accepted_t = t
                        if out_of_slots:
                            done = True
                    else:
                        done = True
                    break
                t = tn
            if accepted_t is None:
                break  # no step
            # ---- accept ----
            t = accepted_t
            s_new = t * d
            y_new = g_t - g_c
            x = x + s_new
            it += 1
            accepted += 1
            f_prev, f_c = f_c, f_t
            gn = float(g_t.norm())
            fscale = max(abs(f_t), 1.0)
            if it >= iters or done:
                break
            if mode == "lbfgs" and (gn <= tol * fscale or abs(f_prev - f_t) <= tol * fscale):
                break
            g_c = g_t
            if mode == "gd":
                d = -g_c
                dg0 = float(g_c @ d)
                t = gd_lr
                if slot >= nslots:
                    break
                continue
            sy = float(s_new @ y_new)
            yy = float(y_new @ y_new)
            if sy > 1e-10 * (yy if yy > 0 else 1.0) and yy > 0:
                S.append(s_new)
                Yh.append(y_new)
                if len(S) > hist:
                    S.pop(0)
                    Yh.pop(0)
            # two-loop recursion
            if S:
                q = g_c.clone()
                alphas = []
                for s_i, y_i in zip(reversed(S), reversed(Yh)):
                    rho = 1.0 / float(s_i @ y_i)
                    a = rho * float(s_i @ q)
                    alphas.append((rho, a))
                    q -= a * y_i
                gamma = float(S[-1] @ Yh[-1]) / float(Yh[-1] @ Yh[-1])
                r = gamma * q
                for (s_i, y_i), (rho, a) in zip(zip(S, Yh), reversed(alphas)):
                    beta = rho * float(y_i @ r)
                    r += s_i * (a - beta)
                d = -r
            else:
                d = -g_c
            dg0 = float(g_c @ d)
            if not dg0 < 0:
                S.clear()
                Yh.clear()
                d = -g_c
                dg0 = float(g_c @ d)
            t = 1.0
            if slot >= nslots:
                break
    c, b = unpack(x)
    coef = torch.where(live, c * inv, wfix)
    if center and K >= 2:
        coef = coef - coef.mean(0, keepdim=True)
        b = b - b.mean()
    return SolveResult(
        coef=coef.float(),
        intercept=b.float(),
        delta_coef=(coef - w_old).float(),
        delta_intercept=(b - b_old).float(),
        loss=f_c,
        evals=evals,
        accepted=accepted,
        ls_fail=ls_fail,
    )


def predict(X: torch.Tensor, coef: torch.Tensor, intercept: torch.Tensor) -> torch.Tensor:
    return (X.float() @ coef.float().t() + intercept.float()).argmax(1)
