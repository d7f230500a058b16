"""Client plugin (mirror of FLClient.fit / _train, src/client/fl_client.py:76-149,
and of MaliciousFLClient.fit's post-training poison hook, malicious_client.py:87-126).

``Client.local_update(global_params, config) -> (params, num_examples,
{"loss", "client_id"})`` keeps the reference contract; ``fit`` returns
NumPy arrays like the Flower NumPyClient.  It runs on the engine's
client-batched trainer with K = 1 (the round engine trains all of a GPU's
clients in one batch instead).  Differences from the reference, by design:
parameters() only (the simulation path, run_experiments.py:238), fixed
batches instead of a shuffling DataLoader, explicit dropout masks.

No gradient clipping by default (clip = 0.0), as FLClient._train
(fl_client.py:130-141: zero_grad, forward, loss, backward, step); pass
clip = 1.0 for the simulation loop's clip_grad_norm_ (run_experiments.py:234).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .models.multimodal import ModelSpec
from .train import ClientBatchTrainer, TrainConfig


class Client:
    def __init__(self, client_id: int, batches: Sequence, spec: ModelSpec = ModelSpec(), device="cuda",
                 local_epochs: int = 1, learning_rate: float = 0.01, clip: float = 0.0, momentum: float = 0.9,
                 weight_decay: float = 0.0, dropout_masks: Optional[Sequence] = None, malicious: bool = False):
        self.client_id = client_id
        self.batches = list(batches)  # [(images [B,...], tokens [B,T], labels [B])]
        self.spec = spec
        self.local_epochs = local_epochs
        self.learning_rate = learning_rate
        self.masks = dropout_masks
        self.malicious = malicious
        self.trainer = ClientBatchTrainer(spec, 1, device, TrainConfig(lr=learning_rate, momentum=momentum,
                                                                       weight_decay=weight_decay, clip=clip))

    @property
    def num_examples(self) -> int:
        return sum(int(b[2].shape[0]) for b in self.batches)

    def local_update(self, global_params: List[torch.Tensor], config: Dict) -> Tuple[List[torch.Tensor], int, Dict]:
        epochs = int(config.get("local_epochs", self.local_epochs))       # fl_client.py:95
        lr = float(config.get("learning_rate", self.learning_rate))      # fl_client.py:96
        self.trainer.cfg.lr = lr
        flat = torch.cat([torch.as_tensor(p).reshape(-1).float() for p in global_params])
        self.trainer.load_global(flat)
        batches = [(i.unsqueeze(0), t.unsqueeze(0), y.unsqueeze(0)) for (i, t, y) in self.batches] * epochs
        steps = config.get("local_steps")
        if steps is not None:
            batches = batches[: int(steps)]
        masks = None if self.masks is None else [m.unsqueeze(0) for m in self.masks] * epochs
        if masks is not None:
            masks = masks[: len(batches)]
        # a malicious client's row is written negated by the export: the sign
        # flip (model_poisoning.py:274-276) after training (malicious_client.py:103-115)
        loss = self.trainer.local_update(batches, masks, negate_rows=1 if self.malicious else 0)
        params = [t.clone() for t in self.trainer.X.row(0)]
        return params, self.num_examples, {"loss": float(loss[0].item()), "client_id": self.client_id}

    def fit(self, parameters, config):
        params, n, metrics = self.local_update([torch.as_tensor(p) for p in parameters], config)
        return [p.cpu().numpy() for p in params], n, metrics

    def get_parameters(self, config=None) -> List[np.ndarray]:
        return [p.detach().cpu().numpy() for p in self.trainer.X.row(0)]
