"""Diagnostic, part 2: client 1 of the native-trainer parity test, step by step.
(1) after ONE local step: GPU vs oracle fc1 rows; (2) the step-1 forward on the
CPU from the GPU's own step-0 weights, in fp32 and fp64: the fc1
pre-activations of unit 150 (the row whose update differs)."""
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
X1, loss1, n1 = nt.train_clients(spec, glob, batches[:1], TrainConfig(local_steps=1), masks[:1])
X2, loss2, n2 = nt.train_clients(spec, glob, batches, TrainConfig(local_steps=2), masks)
lay = param_layout(spec)
offs, o = {}, 0
for n, s in lay:
    offs[n] = (o, s)
    o += int(torch.Size(s).numel())
gl = glob.cpu()
k = 1
cb = [(im[k].cpu(), tk[k].cpu(), lb[k].cpu()) for im, tk, lb in batches]
mk = [m[k].cpu() for m in masks]
upd1, l1 = otrain.local_update(MultimodalNet, spec, gl, cb[:1], masks=mk[:1])
ref1 = torch.cat([u.reshape(-1) for u in upd1])
print("step-0 loss gpu", loss1[k].item(), "ref", l1, "| clip norms gpu", n1.tolist())
for name in ("fc1.weight", "fc1.bias", "fc2.weight"):
    a, shp = offs[name]
    n = int(torch.Size(shp).numel())
    d = (X1[k].cpu()[a:a + n] - ref1[a:a + n]).abs()
    print(f"after 1 step {name}: max|gpu-ref| {d.max().item():.3e} (max|dW| {(ref1[a:a+n]-gl[a:a+n]).abs().max().item():.3e})")


def fwd_pre(wflat, dtype):
    m = MultimodalNet(spec)
    off = 0
    with torch.no_grad():
        for p in m.parameters():
            nn_ = p.numel()
            p.copy_(wflat[off:off + nn_].view(p.shape))
            off += nn_
    m = m.to(dtype).train()
    pre = []
    m.fc1.register_forward_hook(lambda mod, i, out: pre.append(out.detach()))
    im, tk, lb = cb[1]
    m(im.to(dtype), tk)
    return pre[0][:, 150]


w_gpu0 = X1[k].cpu()
print("step-1 fc1 pre unit 150 from GPU step-0 weights fp32:", fwd_pre(w_gpu0, torch.float32).tolist())
print("                                               fp64:", fwd_pre(w_gpu0.double(), torch.float64).tolist())
print("                 from oracle step-0 weights  fp32:", fwd_pre(ref1, torch.float32).tolist())
print("dropout mask step1 unit150:", mk[1][:, 150].tolist())
