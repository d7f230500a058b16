"""FLTrust (mirror of src/defenses/fltrust.py:17-307).

  g = server update: global -> SGD(lr, momentum 0.9) over the root dataset
      for local_epochs (fltrust.py:99-152), g = params_after - params_before
  trust_i = max(0, (u_i . g) / (||u_i|| ||g||))   (0 if a norm < 1e-10)
  u_i' = u_i * (||g|| / ||u_i||)                  (unchanged if ||u_i|| < 1e-10)
  aggregate = sum_i trust_i * u_i' / sum_i trust_i   (g itself if the sum < 1e-10)

Engine: the server update runs on the client-batched trainer with one client
(no gradient clipping — the reference's FLTrust loop has none; max_norm = 0
skips the clip pass of the fused step); the K dots, K norms and the
trust-weighted combination are one flr_row_dots, one flr_row_norms and one
flr_weighted_rows pass over the client matrix.  Scalars follow the
reference's fp32 tensor ops (dot / (norm * norm), ratio of fp32 norms).

The root dataset is given as tensors (images [N, C, H, W], tokens [N, T],
labels [N]) for the multimodal model; the reference's DataLoader(shuffle=True)
order becomes a seeded permutation per epoch ('seed', default 0) or the
given order with shuffle=False.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..matrix import ClientMatrix
from .base_defense import BaseDefense, as_matrix, source_device


class FLTrustDefense(BaseDefense):
    def __init__(self, defense_config: Dict[str, Any]):
        super().__init__(defense_config)
        self.root_dataset_size = defense_config.get("root_dataset_size", 100)
        self.learning_rate = defense_config.get("learning_rate", 0.01)
        self.local_epochs = defense_config.get("local_epochs", 1)
        self.batch_size = defense_config.get("batch_size", 32)
        self.shuffle = defense_config.get("shuffle", True)
        self.seed = defense_config.get("seed", 0)
        self.device = defense_config.get("device", "cuda")
        self.root_dataset = None
        self.spec = None
        self.trust_scores: List[float] = []
        self.server_gradient: Optional[torch.Tensor] = None
        self._epoch = 0

    # ---- setup (fltrust.py:68-91) ----
    def set_root_dataset(self, images: torch.Tensor, tokens: torch.Tensor, labels: torch.Tensor) -> None:
        n = images.shape[0]
        if n > self.root_dataset_size:  # np.random.choice subsample, as the reference
            idx = torch.as_tensor(np.random.choice(n, size=self.root_dataset_size, replace=False))
            images, tokens, labels = images[idx], tokens[idx], labels[idx]
        self.root_dataset = (images, tokens, labels)

    def set_model(self, model_or_spec) -> None:
        self.spec = getattr(model_or_spec, "spec", model_or_spec)

    # ---- server update (fltrust.py:93-152) ----
    def _batches(self, dev):
        images, tokens, labels = self.root_dataset
        n = images.shape[0]
        if self.shuffle:
            g = torch.Generator().manual_seed(int(self.seed) + self._epoch)
            order = torch.randperm(n, generator=g)
        else:
            order = torch.arange(n)
        self._epoch += 1
        out = []
        for s in range(0, n, self.batch_size):
            idx = order[s:s + self.batch_size]
            out.append((images[idx].unsqueeze(0).to(dev), tokens[idx].unsqueeze(0).to(dev),
                        labels[idx].unsqueeze(0).to(dev)))
        return out

    def compute_server_gradient(self, global_flat: torch.Tensor) -> torch.Tensor:
        if self.root_dataset is None:
            raise ValueError("Root dataset not set. Call set_root_dataset() first.")
        if self.spec is None:
            raise ValueError("Model not set. Call set_model() first.")
        from ..train import ClientBatchTrainer, TrainConfig
        dev = global_flat.device
        cfg = TrainConfig(lr=self.learning_rate, momentum=0.9, weight_decay=0.0, clip=0.0)  # 0: no clip pass
        tr = ClientBatchTrainer(self.spec, 1, dev, cfg)
        tr.load_global(global_flat)
        batches = [b for _ in range(self.local_epochs) for b in self._batches(dev)]
        tr.local_update(batches, None)  # one fresh optimizer over all epochs, as the reference
        g = tr.X.X[0] - global_flat
        self.server_gradient = g
        return g

    # ---- aggregation (fltrust.py:215-270) ----
    def aggregate_flat(self, cm: ClientMatrix, num_examples: List[int],
                       global_flat: Optional[torch.Tensor] = None) -> torch.Tensor:
        if global_flat is None:
            raise ValueError("global_params must be provided for FLTrust")
        g = self.compute_server_gradient(global_flat.to(cm.device).float().contiguous())
        gn = np.float32(torch.linalg.vector_norm(g.double()).item())
        dots = ops.row_dots(cm.X, g).cpu().numpy().astype(np.float32)
        norms = ops.row_norms(cm.X).cpu().numpy().astype(np.float32)
        trust, scales = [], []
        for d, un in zip(dots, norms):
            if un < 1e-10 or gn < 1e-10:
                trust.append(0.0)
            else:
                trust.append(max(0.0, float(np.float32(d / np.float32(un * gn)))))
            scales.append(1.0 if un < 1e-10 else float(np.float32(gn / un)))
        self.trust_scores = trust
        total = sum(trust)
        if total < 1e-10:
            return g.clone()
        return ops.weighted_rows(cm.X, trust, total, scales=scales)

    def aggregate(self, client_updates, num_examples: List[int],
                  global_params: Optional[List[torch.Tensor]] = None) -> List[torch.Tensor]:
        if global_params is None:
            raise ValueError("global_params must be provided for FLTrust")
        cm = as_matrix(client_updates)
        gflat = torch.cat([p.reshape(-1).float() for p in global_params]).to(cm.device)
        flat = self.aggregate_flat(cm, num_examples, gflat)
        return cm.unflatten(flat, source_device(client_updates))

    def detect_malicious(self, client_updates, num_examples, threshold: float = 0.1) -> List[int]:
        return [i for i, s in enumerate(self.trust_scores) if s < threshold]

    def get_metrics(self) -> Dict[str, Any]:
        return {
            "defense_type": "fltrust",
            "root_dataset_size": self.root_dataset_size,
            "trust_scores": self.trust_scores,
            "avg_trust": np.mean(self.trust_scores) if self.trust_scores else 0.0,
        }

    def __repr__(self) -> str:
        return f"FLTrustDefense(root_size={self.root_dataset_size})"
