"""Workload generators for the attacked configurations.

* sign flip — InnerProductManipulationAttack.poison_update with no benign
  mean negates the submitted update (src/attacks/model_poisoning.py:274-276),
  applied after local training (malicious_client.py:103-115).  The engine
  negates the malicious rows of the client matrix in place.
* backdoor — BackdoorAttack.poison_data (src/attacks/backdoor.py:115-290):
  a trigger_size x trigger_size square of trigger_value at the bottom-right
  position (h - size - 1, w - size - 1) on every channel of the (normalised)
  image, on poison_ratio of the client's samples chosen with
  np.random.seed(seed) + np.random.choice(range(n), n*ratio, replace=False),
  and the label replaced by target_class (BackdoorDataset, :13-60).
  Applied here to a malicious client's resident synthetic batches before the
  round (data generation, not timed).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch


def sign_flip_(X: torch.Tensor, rows: Sequence[int]) -> None:
    """In place: X[r] = -X[r] for the malicious rows."""
    for r in rows:
        X[r].neg_()


class Backdoor:
    def __init__(self, trigger_size: int = 3, target_class: int = 0, poison_ratio: float = 0.1,
                 trigger_value: float = 1.0, seed: int = 42, image_size: Tuple[int, int] = (32, 32)):
        self.trigger_size = trigger_size
        self.target_class = target_class
        self.poison_ratio = poison_ratio
        self.trigger_value = trigger_value
        self.seed = seed
        h, w = image_size
        self.position = (h - trigger_size - 1, w - trigger_size - 1)  # 'bottom_right'
        self.num_poisoned = 0
        self.poisoned_indices: List[int] = []

    def choose(self, num_samples: int) -> List[int]:
        np.random.seed(self.seed)
        idx = np.random.choice(list(range(num_samples)), size=int(num_samples * self.poison_ratio),
                               replace=False).tolist()
        self.num_poisoned = len(idx)
        self.poisoned_indices = idx
        return idx

    def apply_trigger_(self, images: torch.Tensor) -> torch.Tensor:
        """images [..., C, H, W] in place."""
        r, c = self.position
        s = self.trigger_size
        images[..., r:r + s, c:c + s] = self.trigger_value
        return images

    def poison_client_(self, images: torch.Tensor, labels: torch.Tensor) -> List[int]:
        """One client's samples flattened in dataset order: images [N, C, H, W],
        labels [N]; poisons them in place and returns the indices."""
        idx = self.choose(images.shape[0])
        if idx:
            sel = torch.tensor(idx, device=images.device)
            sub = images[sel]
            self.apply_trigger_(sub)
            images[sel] = sub
            labels[sel] = self.target_class
        return idx


def poison_batches_(batches, client_cols: Sequence[int], attack: Backdoor) -> None:
    """Poison the resident per-step batches [(images [K,B,...], tokens, labels [K,B])]
    of the client columns `client_cols`: the client's dataset is its samples
    across steps in order (step-major), as a DataLoader over them would see."""
    steps = len(batches)
    for j in client_cols:
        imgs = torch.cat([b[0][j] for b in batches])   # [steps*B, C, H, W]
        labs = torch.cat([b[2][j] for b in batches])
        attack.poison_client_(imgs, labs)
        B = batches[0][0].shape[1]
        for s in range(steps):
            batches[s][0][j].copy_(imgs[s * B:(s + 1) * B])
            batches[s][2][j].copy_(labs[s * B:(s + 1) * B])
