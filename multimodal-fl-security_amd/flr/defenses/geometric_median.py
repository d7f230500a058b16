"""Geometric median by Weiszfeld iterations (mirror of
src/defenses/trimmed_mean.py:177-265).

Reference loop (per iteration, two passes over the K x P matrix):
    d_i = max(||U_i - c||, 1e-10);  w = 1/d;  c' = (w U).sum(0) / w.sum()
    change = ||c' - c||;  stop when change < tolerance
starting from the coordinate-wise lower median.

method="pairwise" (default): after the first step every iterate is a convex
combination c = sum_j a_j U_j of the rows, so with the K x K squared pairwise
distances D2 (one MFMA pass, flr_pairwise_l2):
    ||c - U_i||^2 = (D2 a)_i - a^T D2 a / 2
    ||c' - c||^2  = -b^T D2 b / 2,   b = a' - a   (sum b = 0)
and for the first step (c = median, distances d0 from one flr_row_norms pass)
    ||c' - med||^2 = sum_j a_j d0_j^2 - a^T D2 a / 2.
The iterations then run on K x K numbers on the host (float64), and one
flr_weighted_rows pass forms the final (w U) / sum(w): about 4 HBM passes in
total instead of 2 per iteration.
method="direct": the reference's two passes per iteration on the HIP kernels
(flr_row_norms to c, flr_weighted_rows) — the cross-check of the identity.
"""
from __future__ import annotations

from typing import Any, Dict, List

import numpy as np
import torch

from .. import ops
from ..matrix import ClientMatrix
from .base_defense import BaseDefense


def _weights(dist64: np.ndarray):
    """fp32 clamp + reciprocal as the reference (torch.clamp(min=1e-10), 1.0 / d)."""
    d = np.maximum(dist64.astype(np.float32), np.float32(1e-10))
    w = (np.float32(1.0) / d).astype(np.float32)
    W = np.float32(w.astype(np.float64).sum())
    return w, W


# dist2_i = (D2 a)_i - a^T D2 a / 2 cancels when the iterate nears client i
# (duplicate or colluding clients): its relative error is the distances'
# relative error (Gram kernel: up to ~1e-5) times (D2 a)_i / dist2_i.  Past
# this cancellation factor the identity is not trusted and the caller runs the
# reference's direct passes instead.
CANCEL_LIMIT = 8.0


def weiszfeld_pairwise(D: np.ndarray, d0: np.ndarray, max_iters: int, tolerance: float):
    """Weiszfeld in coefficient space.  D: K x K pairwise distances, d0: the
    rows' distances to the coordinate median.  Returns (w fp32 [K], W fp32,
    num_iters) such that the estimate is (sum_j w_j U_j) / W, or None when a
    distance cancels past CANCEL_LIMIT (use the direct method)."""
    D2 = D.astype(np.float64) ** 2
    tol = np.float32(tolerance)
    w, W = _weights(d0)
    a = w.astype(np.float64) / float(W)
    change2 = float(a @ (d0 * d0)) - 0.5 * float(a @ D2 @ a)
    if np.float32(np.sqrt(max(change2, 0.0))) < tol:
        return w, W, 1
    for it in range(1, max_iters):
        D2a = D2 @ a
        dist2 = D2a - 0.5 * float(a @ D2a)
        if np.any(dist2 * CANCEL_LIMIT < D2a):
            return None
        w, W = _weights(np.sqrt(np.maximum(dist2, 0.0)))
        a_new = w.astype(np.float64) / float(W)
        b = a_new - a
        change2 = -0.5 * float(b @ D2 @ b)
        a = a_new
        if np.float32(np.sqrt(max(change2, 0.0))) < tol:
            return w, W, it + 1
    return w, W, max_iters


class GeometricMedianDefense(BaseDefense):
    def __init__(self, defense_config: Dict[str, Any] = None):
        cfg = defense_config or {}
        super().__init__(cfg)
        self.max_iters = cfg.get("max_iters", 100)
        self.tolerance = cfg.get("tolerance", 1e-5)
        self.method = cfg.get("method", "pairwise")
        self.num_iters = 0

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        X = cm.X
        self.used_direct = self.method == "direct"
        med = ops.median_lower(X)
        if self.max_iters <= 0:
            self.num_iters = 0
            return med
        if self.method == "direct":
            return self._direct(X, med)
        if self.method != "pairwise":
            raise ValueError(f"unknown geometric median method {self.method!r}")
        return self._pairwise(X, med)

    def _pairwise(self, X: torch.Tensor, med: torch.Tensor) -> torch.Tensor:
        D = ops.pairwise_l2(X).cpu().numpy()
        d0 = ops.row_norms(X, center=med).cpu().numpy()
        res = weiszfeld_pairwise(D, d0, self.max_iters, self.tolerance)
        if res is None:  # an iterate close to a client: the identity cancels
            self.used_direct = True
            return self._direct(X, med)
        w, W, self.num_iters = res
        return ops.weighted_rows(X, w, float(W))

    def _direct(self, X: torch.Tensor, med: torch.Tensor) -> torch.Tensor:
        current = med
        tol = np.float32(self.tolerance)
        self.num_iters = self.max_iters
        for it in range(self.max_iters):
            w, W = _weights(ops.row_norms(X, center=current).cpu().numpy())
            new = ops.weighted_rows(X, w, float(W))
            change = ops.row_norms(new.view(1, -1), center=current).item()
            current = new
            if np.float32(change) < tol:
                self.num_iters = it + 1
                break
        return current

    def get_metrics(self) -> Dict[str, Any]:
        return {"defense_type": "geometric_median", "max_iters": self.max_iters, "num_iters": self.num_iters}
