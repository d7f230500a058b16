"""Diagnostic: where the native ResNet+GRU trainer's fc1.weight update differs
from the oracle loop's (tests/test_gpu_native_trainer.py
::test_native_trainer_matches_reference_loop, client 1: per-tensor report
0.28 of max|dW|)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import training as otrain  # noqa: E402
from flr import native_trainer as nt  # noqa: E402
from flr.models.multimodal import ModelSpec, MultimodalNet, param_layout  # noqa: E402
from flr.round import initial_global  # noqa: E402
from flr.train import TrainConfig, make_dropout_masks, synthetic_batches  # noqa: E402

cuda = torch.device("cuda:0")
spec = ModelSpec()
K, B, steps = 2, 8, 2
glob = initial_global(spec, 42, cuda)
batches = synthetic_batches(spec, steps, range(K), B, cuda)
masks = make_dropout_masks(spec, steps, K, B, cuda, seed=3)
X, loss, _ = nt.train_clients(spec, glob, batches, TrainConfig(local_steps=steps), masks)
lay = param_layout(spec)
offs, o = {}, 0
for n, s in lay:
    offs[n] = (o, s)
    o += int(torch.Size(s).numel())
gl = glob.cpu()
for k in range(K):
    cb = [(im[k].cpu(), tk[k].cpu(), lb[k].cpu()) for im, tk, lb in batches]
    pre = []
    orig = MultimodalNet.forward

    class Hooked(MultimodalNet):
        def __init__(self, s):
            super().__init__(s)
            self.fc1.register_forward_hook(lambda m, i, out: pre.append(out.detach().clone()))
    upd, ref_loss = otrain.local_update(Hooked, spec, gl, cb, masks=[m[k].cpu() for m in masks])
    ref = torch.cat([u.reshape(-1) for u in upd])
    got = X[k].cpu()
    for name in ("fc1.weight", "fc1.bias", "fc2.weight", "gru.weight_hh_l0", "layers.3.1.conv2.weight"):
        a, shp = offs[name]
        n = int(torch.Size(shp).numel())
        g, r, w0 = got[a:a + n].double(), ref[a:a + n].double(), gl[a:a + n].double()
        dg, dr = g - w0, r - w0
        err = (dg - dr).abs()
        i = int(err.argmax())
        print(f"client {k} {name}: max|dref| {dr.abs().max().item():.3e} max|diff| {err.max().item():.3e} at {i} "
              f"(dgpu {dg[i].item():.6e} dref {dr[i].item():.6e}); n>1e-2 max: {(err > 1e-2 * dr.abs().max()).sum().item()}")
        if name == "fc1.weight":
            E = err.view(shp)
            rows = torch.nonzero(E.max(dim=1).values > 1e-2 * dr.abs().max()).flatten().tolist()
            print("   rows with large diffs:", rows[:20])
            for s_, p in enumerate(pre):
                for j in rows[:5]:
                    v = p[:, j]
                    print(f"   step {s_} unit {j}: fc1 pre-activations min|.| {v.abs().min().item():.3e} values "
                          f"{[round(x, 6) for x in v.tolist()]}")
    print(f"client {k} loss gpu {loss[k].item():.8f} ref {ref_loss:.8f}")
