"""Krum / Multi-Krum (mirror of src/defenses/krum.py:14-237).

Pipeline on the device, no host round trip until the selected indices are
published: flr_pairwise_l2 (K×K fp64 distances, krum.py:73-99) ->
flr_krum_select (scores + argsort, krum.py:101-131, 149-176) ->
flr_rows_mean over the first multi_k rows of the order (krum.py:182-192).
Single Krum (multi_k == 1) returns the caller's own list for the selected
client, as the reference does (krum.py:178-181).
"""
from __future__ import annotations

from typing import Any, Dict, List

import torch

from .. import ops
from ..matrix import ClientMatrix
from .base_defense import BaseDefense, Updates, as_matrix, source_device


class KrumDefense(BaseDefense):
    def __init__(self, defense_config: Dict[str, Any]):
        super().__init__(defense_config)
        self.num_malicious = defense_config.get("num_malicious", 1)
        self.multi_k = defense_config.get("multi_k", 1)
        # "reference" (default): D bit-identical to the reference's torch.norm,
        # so the selection is the reference's by construction; "gram": the
        # centred Gram on MFMA (HBM-bound, coordinate-sharded: the scaling path)
        self.pairwise_method = defense_config.get("pairwise_method", "reference")
        # flr.shard.Comm of a multi-GPU round (set by RoundEngine): the
        # reference-exact distances then split their pair tiles over the ranks
        self.comm = None
        # reference mode over a training-order client matrix: its tap-major
        # convolution blocks [(off, Cout, Cin, KK), ...] (set by RoundEngine)
        self.tap_blocks = None
        # ... and its dead-tap slabs not yet in X (masks per block, training-order
        # global vector, negated rows; RoundEngine: FLR_TC_DEFER_DEAD), with the
        # call that makes X whole before rows are read (the side-stream fill joined)
        self.tap_dead = None
        self.before_rows = None
        # FLR_DEFER_DEAD=2: X's dead-tap ranges never written — (ranges, gtrain,
        # nneg) for the Multi-Krum mean and the selected row
        self.rows_dead = None
        self.selected_clients: List[int] = []
        self.rejected_clients: List[int] = []
        self.client_scores: List[float] = []
        # device-side results of the last call (engine consumers use these)
        self.distances = None
        self.scores_device = None
        self.order_device = None

    def select(self, cm: ClientMatrix) -> torch.Tensor:
        """Distances, scores and order on the device; returns the int32 order."""
        n, f = cm.K, self.num_malicious
        if n < 2 * f + 3:  # krum.py:153-157
            raise ValueError(
                f"Krum requires n >= 2f + 3. Got n={n}, f={f}. Need at least {2 * f + 3} clients.")
        ref = self.pairwise_method == "reference"
        self.distances = ops.pairwise_l2(cm.X, self.pairwise_method, comm=self.comm,
                                         tap_blocks=self.tap_blocks if ref else None,
                                         dead=self.tap_dead if ref and self.tap_blocks else None)
        self._check_refine_capacity(n)
        self.scores_device, self.order_device = ops.krum_select(self.distances, f)
        return self.order_device

    def _check_refine_capacity(self, K: int) -> None:
        """The Gram path's refine list holds 128 rows: every row at K <= 128.
        Past that, more far-cluster rows than it holds turn the whole D NaN,
        diagonal included (include/flr.h) — raised here, on the device path of
        every round, before any row is selected (one 8-byte read, K > 128 and
        the Gram path only)."""
        if self.pairwise_method == "gram" and K > ops.REFINE_ROWS and bool(torch.isnan(self.distances[0, 0])):
            from .._capi import FlrError
            raise FlrError("KrumDefense", -3, "more far-cluster rows than the Gram path refines (128): use "
                                              "pairwise_method='direct' or 'reference'")

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int], publish: bool = True) -> torch.Tensor:
        """Device pipeline; with publish=False the host copies of the scores
        and indices are skipped (no device sync) — call publish() later."""
        order = self.select(cm)
        if publish:
            self.publish()
        if self.before_rows is not None:
            self.before_rows()
        if self.multi_k == 1:
            i = int(order[0].item())
            if self.rows_dead is not None:
                ranges, g, nneg = self.rows_dead
                return ops.fill_dead_ranges(cm.data[i, : cm.P].clone(), ranges, g, i < nneg)
            return cm.data[i, : cm.P]
        return ops.rows_mean(cm.X, order[: min(self.multi_k, cm.K)], divisor=self.multi_k, dead=self.rows_dead)

    # pairwise_method="reference" reproduces the reference's torch.norm
    # accumulation, which runs over the whole vector in parameters() order:
    # whole rows (all-gather exchange) in torch order or with tap_blocks naming
    # the tap-major convolution weights (training-order rounds), or coordinate
    # slices in torch order (the chains run through the ranks in order)
    @property
    def supports_sharded(self) -> bool:
        return True

    @property
    def order_free(self) -> bool:
        return True

    # the round engine may leave X's dead-tap ranges unwritten (FLR_DEFER_DEAD):
    # this defense reads them through tap_dead / rows_dead / before_rows
    supports_dead_rows = True

    @property
    def needs_tap_blocks(self) -> bool:
        """A training-order client matrix needs tap_blocks set (reference mode)."""
        return self.pairwise_method == "reference"

    def aggregate_sharded(self, cs, num_examples: List[int], publish: bool = True, events=None) -> torch.Tensor:
        """Coordinate-sharded Krum (flr.shard): distances from the per-slice
        Gram sums of every GPU (bit-identical to the one-GPU D), scores and
        order replicated, then the Multi-Krum mean of this GPU's range."""
        n, f = cs.K, self.num_malicious
        if n < 2 * f + 3:  # krum.py:153-157
            raise ValueError(
                f"Krum requires n >= 2f + 3. Got n={n}, f={f}. Need at least {2 * f + 3} clients.")
        self.distances = self._sharded_distances(cs, events)
        self._check_refine_capacity(n)
        self.scores_device, self.order_device = ops.krum_select(self.distances, f)
        if publish:
            self.publish()
        if self.before_rows is not None:
            self.before_rows()
        if self.multi_k == 1:
            if self.rows_dead is not None:  # one GPU: the slice is the whole matrix
                i = int(self.order_device[0].item())
                ranges, g, nneg = self.rows_dead
                return ops.fill_dead_ranges(cs.data[i, : cs.n].clone(), ranges, g, i < nneg)
            return cs.data[self.order_device[0].long(), : cs.n]
        return ops.rows_mean(cs.X, self.order_device[: min(self.multi_k, n)], divisor=self.multi_k,
                             dead=self.rows_dead)

    def _sharded_distances(self, cs, events=None):
        if self.pairwise_method == "reference":
            if cs.comm.world == 1:  # the one slice is the whole matrix
                return ops.pairwise_l2(cs.X, "reference", tap_blocks=self.tap_blocks,
                                       dead=self.tap_dead if self.tap_blocks else None)
            if self.tap_dead is not None:
                raise ValueError("deferred dead taps are a one-GPU mode")
            # training order: the rank boundaries are tap-block aligned (shard.aligned_bounds)
            return ops.pairwise_l2_reference_sharded(cs, self.tap_blocks)
        if self.pairwise_method != "gram":
            raise ValueError(f"pairwise_method {self.pairwise_method!r} has no coordinate-sharded form")
        return ops.pairwise_l2_sharded(cs, events=events)

    def publish(self) -> None:
        """Host copies of scores / selected / rejected (krum.py:171-176).  A
        client that sent NaN has a NaN score and is ranked last, as numpy's
        sort / argsort order NaN (the reference rejects it)."""
        order_host = self.order_device.cpu().tolist()
        self.client_scores = self.scores_device.cpu().tolist()
        self.selected_clients = order_host[: self.multi_k]
        self.rejected_clients = order_host[self.multi_k:]

    def aggregate(self, client_updates: Updates, num_examples: List[int]) -> List[torch.Tensor]:
        cm = as_matrix(client_updates)
        if self.multi_k == 1:  # single Krum returns the caller's own list (krum.py:178-181)
            self.select(cm)
            self.publish()
            sel = self.selected_clients[0]
            return cm.row(sel) if isinstance(client_updates, ClientMatrix) else client_updates[sel]
        flat = self.aggregate_flat(cm, num_examples)
        return cm.unflatten(flat, source_device(client_updates))

    def detect_malicious(self, client_updates: Updates, num_examples: List[int]) -> List[int]:
        if not self.client_scores:
            self.aggregate(client_updates, num_examples)
        return self.rejected_clients

    def get_metrics(self) -> Dict[str, Any]:
        return {
            "defense_type": "krum",
            "num_malicious_assumed": self.num_malicious,
            "multi_k": self.multi_k,
            "selected_clients": self.selected_clients,
            "rejected_clients": self.rejected_clients,
            "client_scores": self.client_scores,
        }

    def __repr__(self) -> str:
        return f"KrumDefense(f={self.num_malicious}, k={self.multi_k})"


class MultiKrumDefense(KrumDefense):
    """multi_k defaults to cfg['default_k'] or 3, written back into the config
    dict as the reference does (krum.py:232-237)."""

    def __init__(self, defense_config: Dict[str, Any]):
        if "multi_k" not in defense_config:
            defense_config["multi_k"] = defense_config.get("default_k", 3)
        super().__init__(defense_config)


class KrumTrimmedMeanDefense(KrumDefense):
    """"Krum + trimmed-mean" (BASELINE.json configs[4]): the Multi-Krum
    selection (krum.py:149-176, multi_k rows by score) followed by the
    coordinate-wise trimmed mean of the selected rows (trimmed_mean.py:63-90:
    t = max(1, int(m * trim_ratio)), the median if m - 2t < 1) — the Bulyan
    composition of the reference's two defenses.  The reference has no such
    class; its two halves are the reference's own rules, each restated by the
    oracle.  One extra pass over the selected rows (flr_trimmed_mean_rows),
    no gather copy of the selection."""

    def __init__(self, defense_config: Dict[str, Any]):
        super().__init__(defense_config)
        self.trim_ratio = defense_config.get("trim_ratio", 0.1)
        self.num_trimmed_per_end = 0

    # the trimmed mean reads the selected rows whole: no dead-tap deferral
    supports_dead_rows = False

    def _combine(self, X: torch.Tensor, order: torch.Tensor) -> torch.Tensor:
        m = min(self.multi_k, X.shape[0])
        t = max(1, int(m * self.trim_ratio))
        self.num_trimmed_per_end = t
        sel = order[:m]
        if m - 2 * t < 1:
            return ops.median_lower(X, rows=sel)
        return ops.trimmed_mean(X, t, rows=sel)

    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int], publish: bool = True) -> torch.Tensor:
        order = self.select(cm)
        if publish:
            self.publish()
        return self._combine(cm.X, order)

    def aggregate_sharded(self, cs, num_examples: List[int], publish: bool = True, events=None) -> torch.Tensor:
        n, f = cs.K, self.num_malicious
        if n < 2 * f + 3:  # krum.py:153-157
            raise ValueError(
                f"Krum requires n >= 2f + 3. Got n={n}, f={f}. Need at least {2 * f + 3} clients.")
        self.distances = self._sharded_distances(cs, events)
        self._check_refine_capacity(n)
        self.scores_device, self.order_device = ops.krum_select(self.distances, f)
        if publish:
            self.publish()
        return self._combine(cs.X, self.order_device)

    def aggregate(self, client_updates: Updates, num_examples: List[int]) -> List[torch.Tensor]:
        cm = as_matrix(client_updates)
        return cm.unflatten(self.aggregate_flat(cm, num_examples), source_device(client_updates))

    def get_metrics(self) -> Dict[str, Any]:
        m = super().get_metrics()
        m.update({"defense_type": "krum_trimmed_mean", "trim_ratio": self.trim_ratio,
                  "num_trimmed_per_end": self.num_trimmed_per_end})
        return m
