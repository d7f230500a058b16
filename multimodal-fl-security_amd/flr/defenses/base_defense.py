"""Defense plugin interface (mirror of src/defenses/base_defense.py:13-97).

``aggregate(client_updates, num_examples) -> List[Tensor]`` keeps the
reference signature.  ``client_updates`` may be the reference's
``List[List[Tensor]]`` (any device; converted to a device client matrix) or a
:class:`flr.matrix.ClientMatrix` (zero-copy, the engine's own round path).
Results are returned on the device the updates came from.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, List, Sequence, Union

import torch

from .. import ops
from ..matrix import ClientMatrix

Updates = Union[ClientMatrix, Sequence[Sequence[torch.Tensor]]]


def as_matrix(client_updates: Updates) -> ClientMatrix:
    if isinstance(client_updates, ClientMatrix):
        return client_updates
    return ClientMatrix.from_updates(client_updates)


def source_device(client_updates: Updates) -> torch.device:
    if isinstance(client_updates, ClientMatrix):
        return client_updates.device
    return client_updates[0][0].device


class BaseDefense(ABC):
    """Abstract defense (base_defense.py:13-71).

    Subclasses implement ``aggregate_flat(cm, num_examples) -> [P] tensor``
    on a device client matrix; ``aggregate`` adapts the reference signature.
    """

    def __init__(self, defense_config: Dict[str, Any]):
        self.config = defense_config
        self.name = self.__class__.__name__

    @abstractmethod
    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        ...

    def aggregate(self, client_updates: Updates, num_examples: List[int]) -> List[torch.Tensor]:
        cm = as_matrix(client_updates)
        flat = self.aggregate_flat(cm, num_examples)
        return cm.unflatten(flat, source_device(client_updates))

    # Coordinate-sharded form (flr.shard): aggregate one GPU's coordinate
    # range of all K clients; returns the [cs.n] slice of the aggregate.
    # Defenses that need whole rows (norms, dots) do not implement it and run
    # on the all-gathered matrix instead.
    supports_sharded = False
    # The aggregate's coordinate i depends only on column i and on row-level
    # quantities invariant under one common permutation of the coordinates
    # (pairwise distances, row selections): the round engine may then hand
    # over the client matrix in the trainer's own coordinate order (tap-major
    # conv weights) and permute only the aggregated vector back.
    order_free = False

    def aggregate_sharded(self, cs, num_examples: List[int]) -> torch.Tensor:
        raise NotImplementedError(f"{self.name} has no coordinate-sharded form")

    def detect_malicious(self, client_updates: Updates, num_examples: List[int]) -> List[int]:
        return []

    def get_metrics(self) -> Dict[str, Any]:
        return {}

    def __repr__(self) -> str:
        return f"{self.name}(config={self.config})"


class NoDefense(BaseDefense):
    """FedAvg: sum(n_i * u_i) / sum(n_i) (base_defense.py:80-97) on the flr_fedavg kernel."""

    def __init__(self, defense_config: Dict[str, Any] = None):
        super().__init__(defense_config or {})

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int]) -> torch.Tensor:
        return ops.fedavg(cm.X, list(num_examples))

    supports_sharded = True
    order_free = True

    def aggregate_sharded(self, cs, num_examples: List[int]) -> torch.Tensor:
        return ops.fedavg(cs.X, list(num_examples))
