"""Multinomial logistic regression: model spec, weight layouts, initialisation.

Reference model (LogisticRegressionTaskSpark.java:32-35, 98-140, 170-176):
``numFeatures = 1024``, ``numClasses = 5`` labels 1..5 plus a phantom class 0,
so ``K = 6`` logits and ``P = K*F + K = 6150`` parameters.  Coefficients are a
column-major ``K x F`` matrix flattened so that flat index ``k`` is class
``k % K`` / feature ``k // K``; intercepts sit at ``K*F + c``.

On the device the coefficient block is row-major ``[K][Fp]`` (``Fp`` = F padded
to a multiple of 128 for the MFMA tiles) followed by the ``K`` intercepts.  The
reference layout is used only at I/O boundaries (checkpoints, exported
weights), via :func:`to_reference_layout` / :func:`from_reference_layout`.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

SUPPORTED_FP = (128, 256, 512, 1024, 2048)


def padded_width(num_features: int) -> int:
    for fp in SUPPORTED_FP:
        if num_features <= fp:
            return fp
    raise ValueError(
        f"dense path supports up to {SUPPORTED_FP[-1]} features (got {num_features}); "
        "use the sparse or sharded model for wider inputs"
    )


@dataclass(frozen=True)
class ModelSpec:
    num_features: int  # F (real)
    num_classes: int  # K = labels + phantom class 0 (reference: 5 + 1)

    @property
    def F(self) -> int:
        return self.num_features

    @property
    def K(self) -> int:
        return self.num_classes

    @property
    def Fp(self) -> int:
        return padded_width(self.num_features)

    @property
    def P(self) -> int:  # device parameter count
        return self.K * self.Fp + self.K

    @property
    def eval_classes(self) -> int:
        return self.K

    @property
    def P_ref(self) -> int:  # reference parameter count
        return self.K * self.F + self.K

    @staticmethod
    def from_labels(num_features: int, max_label: int) -> "ModelSpec":
        """K = max label + 1 (Spark infers numClasses the same way)."""
        return ModelSpec(num_features, max(2, int(max_label) + 1))

    # ---- views -------------------------------------------------------------
    def coef(self, w: torch.Tensor) -> torch.Tensor:
        """[K, F] view of the real coefficients of a device-layout vector."""
        return w[: self.K * self.Fp].view(self.K, self.Fp)[:, : self.F]

    def intercept(self, w: torch.Tensor) -> torch.Tensor:
        return w[self.K * self.Fp :]

    def pack(self, coef: torch.Tensor, intercept: torch.Tensor, device=None) -> torch.Tensor:
        w = torch.zeros(self.P, dtype=torch.float32, device=device if device is not None else coef.device)
        w[: self.K * self.Fp].view(self.K, self.Fp)[:, : self.F] = coef.to(w.device, torch.float32)
        w[self.K * self.Fp :] = intercept.to(w.device, torch.float32)
        return w

    def init(self, kind: str = "zeros", seed: int = 0, scale: float = 0.01, device=None) -> torch.Tensor:
        """Initial weights.  The reference's ``randomlyInitializeWeights`` writes
        zeros (quirk Q6); ``random`` draws N(0, scale^2) coefficients."""
        w = torch.zeros(self.P, dtype=torch.float32)
        if kind == "random":
            g = torch.Generator().manual_seed(seed)
            coef = torch.randn(self.K, self.F, generator=g) * scale
            w = self.pack(coef, torch.zeros(self.K))
        elif kind != "zeros":
            raise ValueError(f"unknown init {kind!r}")
        return w.to(device) if device is not None else w


def to_reference_layout(spec: ModelSpec, w: torch.Tensor) -> torch.Tensor:
    """Device layout -> the reference's flat column-major layout (length K*F+K)."""
    coef = spec.coef(w.float().cpu())  # [K, F]
    flat = coef.t().contiguous().view(-1)  # index k = f*K + c  <->  class k%K, feature k//K
    return torch.cat([flat, spec.intercept(w.float().cpu())])


def from_reference_layout(spec: ModelSpec, ref: torch.Tensor) -> torch.Tensor:
    ref = ref.float().cpu()
    if ref.numel() != spec.P_ref:
        raise ValueError(f"expected {spec.P_ref} reference weights, got {ref.numel()}")
    coef = ref[: spec.K * spec.F].view(spec.F, spec.K).t()
    return spec.pack(coef, ref[spec.K * spec.F :])
