"""Find native ops that leave output elements unwritten: every float tensor from
torch.empty / empty_like is pre-filled with NaN, and the outputs of each flr
autograd Function (forward and backward) are checked for NaN.
Writes gpurun_out/diag_uninit.log."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch  # noqa: E402

import flr.nn as fnn  # noqa: E402
import flr.train as ftrain  # noqa: E402
from flr.models.multimodal import TINY, ModelSpec  # noqa: E402
from flr.round import initial_global  # noqa: E402
from flr.train import ClientBatchTrainer, TrainConfig, make_dropout_masks, synthetic_batches  # noqa: E402

out = None
_empty, _empty_like = torch.empty, torch.empty_like


def nan_empty(*a, **k):
    t = _empty(*a, **k)
    if t.is_floating_point():
        t.fill_(float("nan"))
    return t


def nan_empty_like(*a, **k):
    t = _empty_like(*a, **k)
    if t.is_floating_point():
        t.fill_(float("nan"))
    return t


def wrap(cls):
    fwd, bwd = cls.forward, cls.backward

    def check(tag, res):
        torch.cuda.synchronize()
        items = res if isinstance(res, tuple) else (res,)
        for i, t in enumerate(items):
            if isinstance(t, torch.Tensor) and t.is_floating_point() and torch.isnan(t).any():
                print(f"NaN in {cls.__name__}.{tag} output {i} shape {tuple(t.shape)} "
                      f"count {int(torch.isnan(t).sum())}", file=out, flush=True)
        return res

    cls.forward = staticmethod(lambda ctx, *a: check("forward", fwd(ctx, *a)))
    cls.backward = staticmethod(lambda ctx, *a: check("backward", bwd(ctx, *a)))


def main():
    global out
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = open(os.path.join(ROOT, "gpurun_out", "diag_uninit.log"), "w")
    torch.empty, torch.empty_like = nan_empty, nan_empty_like
    for c in (fnn.ClientConv2d, fnn.ClientConv2dT, fnn.ClientLinear, fnn.ClientGRU, fnn.ClientBatchNorm,
              fnn.ClientMaxPool2d, ftrain.CrossEntropy):
        wrap(c)
    for spec, name in ((TINY, "tiny"), (ModelSpec(), "resnet18")):
        print("==", name, file=out, flush=True)
        ids = list(range(4))
        tr = ClientBatchTrainer(spec, len(ids), "cuda", TrainConfig(local_steps=2))
        b = synthetic_batches(spec, 2, ids, 4, "cuda")
        m = make_dropout_masks(spec, 2, ids, 4, "cuda", seed=5)
        tr.load_global(initial_global(spec, 42, "cuda"))
        loss = tr.local_update(b, m)
        torch.cuda.synchronize()
        print("loss", loss.tolist(), "X has NaN:", bool(torch.isnan(tr.X.X).any()), file=out, flush=True)
    print("done", file=out, flush=True)


if __name__ == "__main__":
    main()
