"""Diagnostic: whose arithmetic flips the layers.1.0 gate of
client 0's second local step?  From the GPU's own step-1 state w1 (native
trainer, one step), the step-2 forward's ReLU inputs are computed five ways:
  gpu_default  the shipped kernels (bf16x6 conv products),
  gpu_f32      the same with FLR_GEMM=f32 (exact fp32 MFMA products),
  cpu_f32      the reference's fp32 forward (MultimodalNet on the CPU),
  cpu_f64      the same in fp64 (the yardstick),
and per ReLU layer the error of each against fp64 (max and RMS, in units of the
layer's std) and every element whose gate decision differs from fp64.
Writes gpurun_out/diag_gate_prec.json.
Usage: python tools/diag_gate_prec.py [B] [k] [mask_seed]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from flr import _capi  # noqa: E402
from flr import native_trainer as nt  # noqa: E402
from flr.models import multimodal as mm  # noqa: E402
from flr.models.multimodal import ModelSpec, MultimodalNet  # noqa: E402
from flr.nn import client_batchnorm  # noqa: E402
from flr.round import initial_global  # noqa: E402
from flr.train import ClientBatchTrainer, TrainConfig, make_dropout_masks, synthetic_batches  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
k = int(sys.argv[2]) if len(sys.argv) > 2 else 0
mseed = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cuda = torch.device("cuda:0")
spec = ModelSpec()
K, steps = 2, 2
glob = initial_global(spec, 42, cuda)
batches = synthetic_batches(spec, steps, range(K), B, cuda)
masks = make_dropout_masks(spec, steps, K, B, cuda, seed=mseed)
X1, _, _ = nt.train_clients(spec, glob, batches[:1], TrainConfig(local_steps=1), masks[:1])
torch.cuda.synchronize()
w1 = X1[k].clone()
im, tk, _ = batches[1]

# ---- GPU: the trainer's own forward (tap-major conv weights), pre-activations
gpu_rec = []
orig_bn_act = mm._bn_act


def rec_bn_act(x, g, b, residual=None, relu=True, stats=None):
    if relu and stats is None:
        z = client_batchnorm(x, g, b, residual, relu=False)
        C = g.numel()
        gpu_rec.append(z.detach().view(C, *z.shape[1:]).transpose(0, 1).double().cpu())
    return orig_bn_act(x, g, b, residual, relu, stats)


def gpu_forward(gemm):
    _capi.set_knob("FLR_GEMM", gemm)
    tr = ClientBatchTrainer(spec, 1, cuda, TrainConfig(local_steps=1))
    tr.load_global(w1)
    params = dict(zip(tr.names, [w.detach() for w in tr.W]))
    gpu_rec.clear()
    mm._bn_act = rec_bn_act
    try:
        with torch.no_grad():
            mm.batched_forward(params, im[k:k + 1], tk[k:k + 1], spec, masks[1][k:k + 1], tr.tap_major, tr.skip_dead)
    finally:
        mm._bn_act = orig_bn_act
        _capi.set_knob("FLR_GEMM", None)
    torch.cuda.synchronize()
    return list(gpu_rec)


# ---- CPU: the reference model, fp32 and fp64, ReLU inputs in call order
cpu_rec = []
orig_relu = F.relu


def relu_hook(x, *a, **kw):
    cpu_rec.append(x.detach().double().clone())
    return orig_relu(x, *a, **kw)


def cpu_forward(dtype):
    m = MultimodalNet(spec)
    o = 0
    wc = w1.cpu()
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(wc[o:o + p.numel()].view(p.shape))
            o += p.numel()
    m = m.to(dtype).train()
    cpu_rec.clear()
    F.relu = relu_hook
    try:
        with torch.no_grad():
            m(im[k].cpu().to(dtype), tk[k].cpu())
    finally:
        F.relu = orig_relu
    return list(cpu_rec)


forms = {"gpu_default": gpu_forward(None), "gpu_f32": gpu_forward("f32"),
         "cpu_f32": cpu_forward(torch.float32)}
ref = cpu_forward(torch.float64)
n = len(forms["gpu_default"])
out = {"config": f"B={B} client {k} mask_seed {mseed}: step-2 forward from the GPU's step-1 state", "layers": []}
for i in range(n):
    z64 = ref[i]
    sd = z64.std().item()
    row = {"relu": i, "shape": list(z64.shape), "std": sd}
    for name, recs in forms.items():
        z = recs[i]
        assert z.shape == z64.shape, (name, i, z.shape, z64.shape)
        e = (z - z64).abs()
        flip = (z > 0) != (z64 > 0)
        row[name] = {"max_err_std": e.max().item() / sd, "rms_err_std": e.pow(2).mean().sqrt().item() / sd,
                     "flips": int(flip.sum())}
        if flip.any():
            idx = flip.nonzero()[:8]
            row[name]["flipped"] = [{"at": tuple(j.tolist()), "z": z[tuple(j.tolist())].item(),
                                     "z64": z64[tuple(j.tolist())].item(),
                                     **{f"z_{o}": forms[o][i][tuple(j.tolist())].item() for o in forms}}
                                    for j in idx]
    out["layers"].append(row)
    print(json.dumps(row))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", f"diag_gate_prec_B{B}_k{k}.json"), "w") as f:
    json.dump(out, f, indent=1)
