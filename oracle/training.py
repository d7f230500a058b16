"""ORACLE (test infrastructure only) — the reference's local-training loop on CPU.

Restates experiments/run_experiments.py:195-240 (the fp32 CPU branch
:230-235) and the loss averaging of src/client/fl_client.py:129-149, for one
client at a time, on flr's MultimodalNet (the reference has no ResNet-18+GRU
model; its fusion-head structure is cub200_cnn.py:88-93).  Two deviations are
required for a deterministic comparison and are made explicit: fixed batches
instead of a shuffling DataLoader, and dropout applied through an explicit mask
(or p = 0) instead of torch's RNG stream.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn


class _MaskDropout(nn.Module):
    def __init__(self):
        super().__init__()
        self.mask = None

    def forward(self, x):
        return x if self.mask is None else x * self.mask


def _mask_dropouts(model: nn.Module) -> List[_MaskDropout]:
    """Replace every nn.Dropout of the model (an attribute or a Sequential
    entry) by a module that applies an explicit mask."""
    out = []
    for mod in list(model.modules()):
        for cname, child in list(mod.named_children()):
            if isinstance(child, nn.Dropout):
                md = _MaskDropout()
                setattr(mod, cname, md)
                out.append(md)
    return out


def local_update(model_cls, spec, global_flat: torch.Tensor, batches: Sequence, lr: float = 0.01,
                 momentum: float = 0.9, weight_decay: float = 0.0, max_norm: float = 1.0,
                 masks: Optional[Sequence[torch.Tensor]] = None, threads: Optional[int] = None
                 ) -> Tuple[List[torch.Tensor], float]:
    """One client's local update.  Returns (params after training, mean loss)."""
    if threads:
        torch.set_num_threads(threads)
    model = model_cls(spec)
    off = 0
    with torch.no_grad():
        for p in model.parameters():  # load_state_dict(global) for parameters() (:203)
            n = p.numel()
            p.copy_(global_flat[off:off + n].view(p.shape))
            off += n
    drops = _mask_dropouts(model)
    optimizer = torch.optim.SGD(model.parameters(), lr=lr, momentum=momentum, weight_decay=weight_decay)  # :206-211
    criterion = nn.CrossEntropyLoss()
    model.train()
    losses = []
    for s, (images, tokens, labels) in enumerate(batches):
        for d in drops:
            d.mask = None if masks is None else masks[s]
        optimizer.zero_grad()
        outputs = model(images, tokens)
        loss = criterion(outputs, labels)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)  # :234
        optimizer.step()
        losses.append(loss.item())
    update = [p.data.clone() for p in model.parameters()]  # :238
    return update, sum(losses) / len(losses)


def fl_client_train(model_cls, spec, global_flat: torch.Tensor, batches: Sequence, learning_rate: float = 0.01,
                    masks: Optional[Sequence[torch.Tensor]] = None) -> Tuple[List[torch.Tensor], float]:
    """FLClient._train (src/client/fl_client.py:109-149): SGD(lr, momentum=0.9),
    no weight decay and NO gradient clipping (only the simulation loop clips,
    run_experiments.py:234); loss = sum of batch losses / number of batches.
    clip_grad_norm_ with max_norm = inf scales by exactly 1, i.e. no clip."""
    return local_update(model_cls, spec, global_flat, batches, lr=learning_rate, momentum=0.9, weight_decay=0.0,
                        max_norm=float("inf"), masks=masks)
