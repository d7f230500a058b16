"""Per-round evaluation of the global model on the HIP kernels (SURVEY §8(f)
rank 3).

Mirrors, for the engine's global model:
* evaluate_model (src/utils/metrics.py:14-59): model.eval(); per test batch
  the mean cross-entropy, total_loss += loss.item() * batch_size,
  predicted = torch.max(outputs, 1); returns accuracy, loss, correct, total;
* compute_attack_success_rate (:62-98): share of samples predicted as the
  target class, over the backdoor's triggered test set — every non-target
  sample with the trigger stamped in (TriggeredTestDataset,
  src/attacks/backdoor.py:62-112, created by create_poisoned_testset
  :301-319 with exclude_target=True);
* compute_label_flip_asr (:101-157).
Called by the reference after every round (run_experiments.py:262) and for
the ASR at the end of the run (:281-291).

Engine: the global vector is loaded once into a one-client trainer's layout
(tap-major conv weights included); the forward runs the training kernels with
BatchNorm in eval mode (flr_batchnorm_infer, running statistics) over chunks
of the test set, and flr_classify_rows produces every row's prediction, loss
and the integer tallies in one launch.  BatchNorm statistics in eval mode are
the reference global model's buffers: torch's initial (0, 1), because the
simulation copies parameters() only (run_experiments.py:257-259); pass
bn_stats to use others.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _capi
from .attacks import Backdoor
from .models.multimodal import ModelSpec, batched_forward
from .train import ClientBatchTrainer


class GlobalEvaluator:
    def __init__(self, spec: ModelSpec, device="cuda", batch_size: int = 32, chunk: int = 1024,
                 bn_stats: Optional[Dict[str, Tuple[torch.Tensor, torch.Tensor]]] = None):
        self.spec = spec
        self.device = torch.device(device)
        self.batch_size = batch_size  # the reference's test DataLoader batch (run_experiments.py:180)
        self.chunk = max(batch_size, chunk // batch_size * batch_size)
        self.bn_stats = bn_stats if bn_stats is not None else {}
        self.tr = ClientBatchTrainer(spec, 1, self.device)

    def load(self, global_flat: torch.Tensor) -> None:
        """The global model to evaluate (a [P] vector in parameters() order)."""
        self.tr.load_global(global_flat)

    @torch.no_grad()
    def _scan(self, images: torch.Tensor, text: Optional[torch.Tensor], labels: Optional[torch.Tensor],
              target: int = -1, source: int = -1):
        """One pass over the set: per-row predictions, losses and the tallies."""
        n = images.shape[0]
        dev = self.device
        pred = torch.empty(n, dtype=torch.int32, device=dev)
        loss_rows = torch.empty(n, dtype=torch.float32, device=dev)
        counts = torch.zeros(5, dtype=torch.int64, device=dev)
        params = dict(zip(self.tr.names, self.tr.W))
        st = torch.cuda.current_stream(dev).cuda_stream
        for a in range(0, n, self.chunk):
            b = min(n, a + self.chunk)
            im = images[a:b].to(dev, torch.float32).unsqueeze(0)
            tx = None if text is None else text[a:b].to(dev).unsqueeze(0)
            logits = batched_forward(params, im, tx, self.spec, None, self.tr.tap_major,
                                     bn_stats=self.bn_stats)[0].contiguous()
            lab = None if labels is None else labels[a:b].to(dev, torch.int64).contiguous()
            _capi.call("flr_classify_rows", logits.data_ptr(), None if lab is None else lab.data_ptr(), b - a,
                       logits.shape[1], int(target), int(source), pred[a:].data_ptr(), loss_rows[a:].data_ptr(),
                       counts.data_ptr(), st)
        return pred, loss_rows, counts.cpu().tolist()

    def evaluate_model(self, images: torch.Tensor, text: Optional[torch.Tensor],
                       labels: torch.Tensor) -> Dict[str, float]:
        """metrics.py:14-59 (batches of batch_size in order, the last one partial)."""
        n = int(labels.shape[0])
        _, loss_rows, counts = self._scan(images, text, labels)
        rows = loss_rows.cpu().numpy()
        total_loss = 0.0
        for a in range(0, n, self.batch_size):  # loss.item() * images.size(0) per batch
            blk = rows[a:a + self.batch_size]
            total_loss += float(np.float32(blk.sum(dtype=np.float32) / np.float32(len(blk)))) * len(blk)
        correct = int(counts[0])
        return {"accuracy": correct / n if n else 0.0, "loss": total_loss / n if n else 0.0,
                "correct": correct, "total": n}

    def attack_success_rate(self, images: torch.Tensor, text: Optional[torch.Tensor], labels: torch.Tensor,
                            backdoor: Backdoor) -> float:
        """metrics.py:62-98 over the triggered test set (backdoor.py:62-112,
        301-319): samples of the target class are left out, the trigger is
        stamped on the rest, ASR = share predicted as the target class."""
        keep = (labels != backdoor.target_class).nonzero().flatten()
        if keep.numel() == 0:
            return 0.0
        trig = backdoor.apply_trigger_(images[keep].clone())
        _, _, counts = self._scan(trig, None if text is None else text[keep], None, target=backdoor.target_class)
        return counts[1] / int(keep.numel())

    def label_flip_asr(self, images: torch.Tensor, text: Optional[torch.Tensor], labels: torch.Tensor,
                       source_class: int, target_class: int) -> Dict[str, float]:
        """metrics.py:101-157."""
        _, _, c = self._scan(images, text, labels, target=target_class, source=source_class)
        st, sc, s2t = int(c[2]), int(c[3]), int(c[4])
        return {"source_accuracy": sc / st if st else 0.0, "flip_rate": s2t / st if st else 0.0,
                "source_total": st, "source_correct": sc, "misclassified_as_target": s2t}
