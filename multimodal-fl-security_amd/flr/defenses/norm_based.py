"""Norm-based defenses (mirror of src/defenses/differential_privacy.py:15-349):
GradientClippingDefense, NormBoundingDefense, DPSGDDefense.

All three are one per-client norm pass (flr_row_norms, K norms in one launch
instead of K torch.norm calls + K host syncs) and one weighted row pass
(flr_weighted_rows: per-row clip scale x example weight, Python-sum order).
Norms are exact (fp64 accumulation); the reference's fp32 torch.norm drifts
by up to ~1e-5..3e-4 relative at 1e6..1e7 coordinates, so a clip/filter
decision can differ from the reference only for a client whose norm sits
within that drift of the threshold.
"""
from __future__ import annotations

from typing import Any, Dict, List

import numpy as np
import torch

from .. import ops
from ..matrix import ClientMatrix
from .base_defense import BaseDefense


def _f32(x) -> float:
    return float(np.float32(x))


class GradientClippingDefense(BaseDefense):
    """Clip each update to clip_norm (l2 or linf), then the example-weighted
    mean (differential_privacy.py:189-293)."""

    def __init__(self, defense_config: Dict[str, Any]):
        super().__init__(defense_config)
        self.clip_norm = defense_config.get("clip_norm", 1.0)
        self.clip_type = defense_config.get("clip_type", "l2")
        self.clipped_count = 0
        self.original_norms: List[float] = []

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        kind = "linf" if self.clip_type == "linf" else "l2"
        norms = [_f32(v) for v in ops.row_norms(cm.X, kind=kind).tolist()]  # fp32 .item() values
        self.original_norms = norms
        scales = []
        self.clipped_count = 0
        for nrm in norms:
            if nrm > self.clip_norm:
                scales.append(self.clip_norm / nrm)  # Python float; torch multiplies in fp32
                self.clipped_count += 1
            else:
                scales.append(1.0)
        return ops.weighted_rows(cm.X, [float(n) for n in num_examples], float(sum(num_examples)),
                                 scales=scales)

    def get_metrics(self) -> Dict[str, Any]:
        return {
            "defense_type": "gradient_clipping",
            "clip_norm": self.clip_norm,
            "clip_type": self.clip_type,
            "clipped_count": self.clipped_count,
            "original_norms": self.original_norms,
        }


class NormBoundingDefense(BaseDefense):
    """Keep updates with min_norm <= ||u|| <= max_norm; weighted mean of the
    kept ones, all of them if none is kept (differential_privacy.py:296-349)."""

    def __init__(self, defense_config: Dict[str, Any]):
        super().__init__(defense_config)
        self.max_norm = defense_config.get("max_norm", 10.0)
        self.min_norm = defense_config.get("min_norm", 0.0)
        self.rejected_clients: List[int] = []

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        norms = [_f32(v) for v in ops.row_norms(cm.X).tolist()]
        keep = [i for i, v in enumerate(norms) if self.min_norm <= v <= self.max_norm]
        self.rejected_clients = [i for i in range(cm.K) if i not in set(keep)]
        if not keep:
            keep = list(range(cm.K))
        w = [float(num_examples[i]) for i in keep]
        return ops.weighted_rows(cm.X, w, float(sum(num_examples[i] for i in keep)), rows=keep)

    def detect_malicious(self, client_updates, num_examples) -> List[int]:
        return self.rejected_clients

    def get_metrics(self) -> Dict[str, Any]:
        return {
            "defense_type": "norm_bounding",
            "max_norm": self.max_norm,
            "min_norm": self.min_norm,
            "rejected_clients": self.rejected_clients,
        }


class DPSGDDefense(BaseDefense):
    """Clip to clip_norm, example-weighted mean, Gaussian noise of std
    clip_norm * noise_multiplier / n (differential_privacy.py:15-186).
    The noise comes from torch's device RNG (seedable via 'seed'); it is not
    RNG-identical to the reference's CPU torch.randn_like draws."""

    def __init__(self, defense_config: Dict[str, Any]):
        super().__init__(defense_config)
        self.clip_norm = defense_config.get("clip_norm", 10.0)
        self.noise_multiplier = defense_config.get("noise_multiplier", 0.005)
        self.target_epsilon = defense_config.get("target_epsilon", 8.0)
        self.target_delta = defense_config.get("target_delta", 1e-5)
        self.rounds_completed = 0
        self.privacy_spent = 0.0
        self._gen = None
        self._seed = defense_config.get("seed")

    def clipped_mean(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        norms = ops.row_norms(cm.X).to(torch.float32).cpu()  # fp32 norm tensors
        # `clip_norm / norm` on a 0-dim fp32 tensor is norm.reciprocal() * clip_norm in fp32
        scales = [float(v.reciprocal() * self.clip_norm) if v > self.clip_norm else 1.0 for v in norms]
        return ops.weighted_rows(cm.X, [float(n) for n in num_examples], float(sum(num_examples)),
                                 scales=scales)

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        n = cm.K
        agg = self.clipped_mean(cm, num_examples)
        noise_std = self.clip_norm * self.noise_multiplier / n
        if self._gen is None and self._seed is not None:
            self._gen = torch.Generator(device=agg.device)
            self._gen.manual_seed(int(self._seed))
        noise = torch.randn(agg.shape, generator=self._gen, device=agg.device, dtype=agg.dtype)
        agg = agg + noise * noise_std
        self.rounds_completed += 1
        self.privacy_spent += np.sqrt(2 * np.log(1 / self.target_delta)) / self.noise_multiplier
        return agg

    def get_privacy_spent(self) -> float:
        return self.privacy_spent

    def is_budget_exhausted(self) -> bool:
        return self.privacy_spent >= self.target_epsilon

    def get_metrics(self) -> Dict[str, Any]:
        return {
            "defense_type": "dp_sgd",
            "clip_norm": self.clip_norm,
            "noise_multiplier": self.noise_multiplier,
            "rounds_completed": self.rounds_completed,
            "privacy_spent": self.privacy_spent,
            "target_epsilon": self.target_epsilon,
        }

    def __repr__(self) -> str:
        return (f"DPSGDDefense(clip={self.clip_norm}, noise={self.noise_multiplier}, "
                f"eps={self.privacy_spent:.2f}/{self.target_epsilon})")
