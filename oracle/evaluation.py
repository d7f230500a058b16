"""ORACLE (test infrastructure only) — the reference's evaluation metrics on CPU.

Restates evaluate_model (src/utils/metrics.py:14-59), compute_attack_success_rate
(:62-98) and compute_label_flip_asr (:101-157) over in-memory test tensors
batched like the reference's DataLoader(test, batch_size) (no shuffle), and the
backdoor's triggered test set (TriggeredTestDataset, src/attacks/backdoor.py:62-112,
exclude_target=True).  The model is flr's per-client module loaded from a flat
parameters() vector; its BatchNorm buffers are torch's initial ones, as the
reference's global model's (run_experiments.py:257-259 copies parameters() only).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn


def _model(model_cls, spec, global_flat: torch.Tensor) -> nn.Module:
    model = model_cls(spec)
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.copy_(global_flat[off:off + n].view(p.shape))
            off += n
    return model


def _batches(images, text, labels, bs):
    for a in range(0, images.shape[0], bs):
        yield images[a:a + bs], None if text is None else text[a:a + bs], labels[a:a + bs]


def evaluate_model(model_cls, spec, global_flat, images, text, labels, batch_size: int = 32) -> Dict[str, float]:
    model = _model(model_cls, spec, global_flat)
    model.eval()  # metrics.py:30
    criterion = nn.CrossEntropyLoss()
    total_loss, correct, total = 0.0, 0, 0
    with torch.no_grad():
        for im, tx, lb in _batches(images, text, labels, batch_size):
            outputs = model(im, tx)
            loss = criterion(outputs, lb)
            total_loss += loss.item() * im.size(0)
            _, predicted = torch.max(outputs.data, 1)
            total += lb.size(0)
            correct += (predicted == lb).sum().item()
    return {"accuracy": correct / total, "loss": total_loss / total, "correct": correct, "total": total}


def triggered_testset(images, text, labels, backdoor):
    """TriggeredTestDataset (backdoor.py:62-112) with exclude_target=True."""
    keep = [i for i in range(labels.shape[0]) if int(labels[i]) != backdoor.target_class]
    idx = torch.tensor(keep, dtype=torch.long)
    trig = images[idx].clone()
    r, c = backdoor.position
    s = backdoor.trigger_size
    trig[:, :, r:r + s, c:c + s] = backdoor.trigger_value  # backdoor.py:102-112
    return trig, None if text is None else text[idx], labels[idx]


def attack_success_rate(model_cls, spec, global_flat, images, text, target_class: int,
                        batch_size: int = 32) -> float:
    model = _model(model_cls, spec, global_flat)
    model.eval()
    total, success = 0, 0
    with torch.no_grad():
        for im, tx, _ in _batches(images, text, torch.zeros(images.shape[0]), batch_size):
            outputs = model(im, tx)
            _, predicted = torch.max(outputs.data, 1)
            total += im.size(0)
            success += (predicted == target_class).sum().item()
    return success / total if total > 0 else 0.0


def label_flip_asr(model_cls, spec, global_flat, images, text, labels, source_class: int, target_class: int,
                   batch_size: int = 32) -> Dict[str, float]:
    model = _model(model_cls, spec, global_flat)
    model.eval()
    st = sc = s2t = 0
    with torch.no_grad():
        for im, tx, lb in _batches(images, text, labels, batch_size):
            _, predicted = torch.max(model(im, tx).data, 1)
            mask = lb == source_class
            sp, sl = predicted[mask], lb[mask]
            st += mask.sum().item()
            sc += (sp == sl).sum().item()
            s2t += (sp == target_class).sum().item()
    return {"source_accuracy": sc / st if st else 0.0, "flip_rate": s2t / st if st else 0.0,
            "source_total": st, "source_correct": sc, "misclassified_as_target": s2t}
