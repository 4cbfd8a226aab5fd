"""Wide (sparse-input) logistic regression: model spec and weight layout.

BASELINE.json configs 4 and 5 scale the reference model
(LogisticRegressionTaskSpark.java:32-35, 98-140: multinomial LR over 1024
hashed features) to 10^6 .. 10^8 hashed features.  The weights stay a dense
vector (the server owns it; config 5 shards it by key range), but feature rows
are sparse CSR and the worker solves in the subspace its window touches
(csrc/kernels/wide_kernels.h).

Device layout (``P = F*KP + KP`` floats):
  * coefficient (feature f, class c) at ``f*KP + c`` -- feature-major, which is
    the reference's own flat order (``w[k]`` = class ``k % K``, feature
    ``k // K``; LogisticRegressionTaskSpark.java:122-140) with K padded to KP so
    one non-zero gathers its KP weights with 16-B loads;
  * the KP intercepts at ``F*KP + c``;
  * classes ``c >= K`` are padding and stay zero.

``K == 1`` is the binary sigmoid / cross-entropy model (one logit, labels
{0, 1}); ``K >= 2`` is the multinomial model with the reference's phantom
class 0 when labels are 1..5.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


def padded_classes(K: int) -> int:
    for kp in (1, 2, 4, 8, 16):
        if K <= kp:
            return kp
    raise ValueError(f"at most 16 classes supported (got {K})")


@dataclass(frozen=True)
class WideSpec:
    num_features: int  # F
    num_classes: int  # K (1 = binary sigmoid)

    @property
    def F(self) -> int:
        return self.num_features

    @property
    def K(self) -> int:
        return self.num_classes

    @property
    def KP(self) -> int:
        return padded_classes(self.num_classes)

    @property
    def P(self) -> int:
        return self.F * self.KP + self.KP

    @property
    def eval_classes(self) -> int:
        """Classes of the confusion matrix (binary model: 2)."""
        return 2 if self.K == 1 else self.K

    # ---- views -------------------------------------------------------------
    def coef(self, w: torch.Tensor) -> torch.Tensor:
        """[K, F] view (copy) of the coefficients of a device-layout vector."""
        return w[: self.F * self.KP].view(self.F, self.KP)[:, : self.K].t()

    def intercept(self, w: torch.Tensor) -> torch.Tensor:
        return w[self.F * self.KP : self.F * self.KP + self.K]

    def pack(self, coef: torch.Tensor, intercept: torch.Tensor, device=None) -> torch.Tensor:
        dev = device if device is not None else coef.device
        w = torch.zeros(self.P, dtype=torch.float32, device=dev)
        w[: self.F * self.KP].view(self.F, self.KP)[:, : self.K] = coef.t().to(dev, torch.float32)
        w[self.F * self.KP : self.F * self.KP + self.K] = intercept.to(dev, torch.float32)
        return w

    INIT_CHUNK = 1 << 22  # features per generator chunk of the random init

    def init(self, kind: str = "zeros", seed: int = 0, scale: float = 0.01, device=None) -> torch.Tensor:
        """Zeros (reference quirk Q6) or N(0, scale^2) coefficients.  Random
        init is drawn by CPU generators (identical on every device and rank), one
        per chunk of INIT_CHUNK features, and streamed to the target device
        (10^8 x KP floats)."""
        return self.init_range(kind, seed, 0, self.F, scale, device)

    def init_range(self, kind: str, seed: int, lo: int, hi: int, scale: float = 0.01, device=None) -> torch.Tensor:
        """The coefficients of features [lo, hi) of :meth:`init` followed by KP
        zero intercepts: ``[(hi - lo)*KP + KP]`` (a key-range shard, or with
        lo = 0, hi = F the whole vector).  Only the chunks overlapping the range
        are generated, so a rank draws its own shard alone."""
        dev = torch.device(device) if device is not None else torch.device("cpu")
        n = hi - lo
        w = torch.zeros(n * self.KP + self.KP, dtype=torch.float32, device=dev)
        if kind == "random":
            view = w[: n * self.KP].view(n, self.KP)
            step = self.INIT_CHUNK
            for c in range(lo // step, -(-hi // step)):
                f0, f1 = c * step, min(self.F, (c + 1) * step)
                g = torch.Generator().manual_seed(seed * 1_000_003 + c)
                blk = torch.randn(f1 - f0, self.K, generator=g) * scale
                a, b = max(f0, lo), min(f1, hi)
                view[a - lo:b - lo, : self.K] = blk[a - f0:b - f0].to(dev)
        elif kind != "zeros":
            raise ValueError(f"unknown init {kind!r}")
        return w
