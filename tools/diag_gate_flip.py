"""Diagnostic: is a per-tensor update difference of the native trainer against
the oracle an isolated ReLU-gate / max-pool flip (the reference's own fp32
conditioning) or a kernel error?  Client `k` of the native-trainer parity test:
(1) after ONE local step, per-tensor GPU vs oracle weights; (2) the step-1
forward on the CPU, in fp32 from the GPU's step-0 weights and from the oracle's,
and in fp64 from the GPU's: every ReLU input and max-pool window whose decision
differs between the two fp32 forwards, with its value and the fp64 value.
Usage: python tools/diag_gate_flip.py [B] [k] [mask_seed]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import training as otrain  # noqa: E402
from flr import native_trainer as nt  # noqa: E402
from flr.models.multimodal import ModelSpec, MultimodalNet, param_layout  # noqa: E402
from flr.round import initial_global  # noqa: E402
from flr.train import TrainConfig, make_dropout_masks, synthetic_batches  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
k = int(sys.argv[2]) if len(sys.argv) > 2 else 0
mseed = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cuda = torch.device("cuda:0")
spec = ModelSpec()
K, steps = 2, 2
glob = initial_global(spec, 42, cuda)
batches = synthetic_batches(spec, steps, range(K), B, cuda)
masks = make_dropout_masks(spec, steps, K, B, cuda, seed=mseed)
X1, loss1, _ = nt.train_clients(spec, glob, batches[:1], TrainConfig(local_steps=1), masks[:1])
torch.cuda.synchronize()
gl = glob.cpu()
cb = [(im[k].cpu(), tk[k].cpu(), lb[k].cpu()) for im, tk, lb in batches]
mk = [m[k].cpu() for m in masks]
upd1, l1 = otrain.local_update(MultimodalNet, spec, gl, cb[:1], masks=mk[:1])
ref1 = torch.cat([u.reshape(-1) for u in upd1])
w1 = X1[k].cpu()
print(f"B={B} client {k}: step-0 loss gpu {loss1[k].item():.9g} ref {l1:.9g}")
off, worst = 0, []
for name, shp in param_layout(spec):
    n = int(torch.Size(shp).numel())
    d = (w1[off:off + n] - ref1[off:off + n]).abs().max().item()
    dr = (ref1[off:off + n] - gl[off:off + n]).abs().max().item()
    worst.append((d / dr if dr else 0.0, name, d))
    off += n
worst.sort(reverse=True)
print("after 1 step, worst per-tensor max|gpu - ref| / max|dW|:", [(f"{r:.2e}", nm) for r, nm, _ in worst[:4]])

records = []
orig_relu, orig_pool = F.relu, F.max_pool2d


def relu_hook(x, *a, **kw):
    records.append(("relu", x.detach().clone()))
    return orig_relu(x, *a, **kw)


def pool_hook(x, *a, **kw):
    y, idx = orig_pool(x, *a, return_indices=True, **{kk: v for kk, v in kw.items() if kk != "return_indices"})
    records.append(("pool", idx.detach().clone()))
    records.append(("pool_in", x.detach().clone()))
    return y


def forward_records(wflat, dtype):
    m = MultimodalNet(spec)
    o = 0
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(wflat[o:o + p.numel()].view(p.shape))
            o += p.numel()
    m = m.to(dtype).train()
    records.clear()
    F.relu, F.max_pool2d = relu_hook, pool_hook
    try:
        im, tk, _ = cb[1]
        m(im.to(dtype), tk)
    finally:
        F.relu, F.max_pool2d = orig_relu, orig_pool
    return list(records)


ra = forward_records(w1, torch.float32)
rb = forward_records(ref1, torch.float32)
rc = forward_records(w1.double(), torch.float64)
flips = 0
for i, ((kind, a), (_, b), (_, c)) in enumerate(zip(ra, rb, rc)):
    if kind == "relu":
        diff = (a > 0) != (b > 0)
        n = int(diff.sum())
        if n:
            flips += n
            idx = diff.nonzero()[:5]
            for j in idx:
                t = tuple(j.tolist())
                print(f"ReLU #{i} {tuple(a.shape)} at {t}: fp32(gpu w) {a[t].item():.3e} fp32(ref w) {b[t].item():.3e} "
                      f"fp64(gpu w) {c[t].item():.3e}")
    elif kind == "pool":
        n = int((a != b).sum())
        if n:
            flips += n
            print(f"max-pool #{i}: {n} windows pick a different argmax")
print(f"decision flips in the step-1 forward: {flips} (ReLU inputs compared: {sum(r[1].numel() for r in ra if r[0] == 'relu')})")
