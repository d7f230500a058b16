"""Coordinate-wise trimmed mean and median (mirror of src/defenses/trimmed_mean.py:14-174)."""
from __future__ import annotations

from typing import Any, Dict, List

import torch

from .. import ops
from ..matrix import ClientMatrix
from .base_defense import BaseDefense


class TrimmedMeanDefense(BaseDefense):
    """t = max(1, int(n * trim_ratio)) per end; median if n - 2t < 1 (trimmed_mean.py:63-72)."""

    def __init__(self, defense_config: Dict[str, Any]):
        super().__init__(defense_config)
        self.trim_ratio = defense_config.get("trim_ratio", 0.1)
        self.num_trimmed_per_end = 0

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        n = cm.K
        self.num_trimmed_per_end = max(1, int(n * self.trim_ratio))
        if n - 2 * self.num_trimmed_per_end < 1:
            return ops.median_lower(cm.X)
        return ops.trimmed_mean(cm.X, self.num_trimmed_per_end)

    supports_sharded = True
    order_free = True

    def aggregate_sharded(self, cs, num_examples: List[int]) -> torch.Tensor:
        return self.aggregate_flat(cs, num_examples)  # coordinate-wise: the slice is a client matrix

    def get_metrics(self) -> Dict[str, Any]:
        return {
            "defense_type": "trimmed_mean",
            "trim_ratio": self.trim_ratio,
            "num_trimmed_per_end": self.num_trimmed_per_end,
        }

    def __repr__(self) -> str:
        return f"TrimmedMeanDefense(trim_ratio={self.trim_ratio})"


class MedianDefense(BaseDefense):
    """Lower median per coordinate, torch.median(dim=0)[0] (trimmed_mean.py:141-166)."""

    def __init__(self, defense_config: Dict[str, Any] = None):
        super().__init__(defense_config or {})

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        return ops.median_lower(cm.X)

    supports_sharded = True
    order_free = True

    def aggregate_sharded(self, cs, num_examples: List[int]) -> torch.Tensor:
        return ops.median_lower(cs.X)

    def get_metrics(self) -> Dict[str, Any]:
        return {"defense_type": "median"}

    def __repr__(self) -> str:
        return "MedianDefense()"
