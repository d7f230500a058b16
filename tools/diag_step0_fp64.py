"""Diagnostic: one local step of client `k` (native trainer, batch B) against
the oracle in fp32 AND in fp64 (the same loop, model and data in double): per
tensor, the GPU's and the fp32 reference's update error against the fp64 update
(max over elements / max |update_64|), and where the GPU and fp32 reference
differ most.  Tells a kernel error (GPU far from fp64, reference close) from the
reference's own fp32 error (both off, or the reference further off).
Usage: python tools/diag_step0_fp64.py [B] [k] [mask_seed] [steps]
(steps: how many of the parity test's 2 generated steps to run, default 1)"""
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
k = int(sys.argv[2]) if len(sys.argv) > 2 else 0
mseed = int(sys.argv[3]) if len(sys.argv) > 3 else 3
nst = int(sys.argv[4]) if len(sys.argv) > 4 else 1
cuda = torch.device("cuda:0")
spec = ModelSpec()
K = 2
glob = initial_global(spec, 42, cuda)
# the native-trainer parity test's data (2 steps generated), its first step only
batches = synthetic_batches(spec, 2, range(K), B, cuda)[:nst]
masks = make_dropout_masks(spec, 2, K, B, cuda, seed=mseed)[:nst]
X1, loss1, norms1 = nt.train_clients(spec, glob, batches, TrainConfig(local_steps=nst), masks)
torch.cuda.synchronize()
gl = glob.cpu()
cb = [(im[k].cpu(), tk[k].cpu(), lb[k].cpu()) for im, tk, lb in batches]
mk = [m[k].cpu() for m in masks]
upd32, l32 = otrain.local_update(MultimodalNet, spec, gl, cb, masks=mk)


class Net64(MultimodalNet):
    def __init__(self, s):
        super().__init__(s)
        self.double()


torch.set_default_dtype(torch.float64)
try:
    cb64 = [(im.double(), tk, lb) for im, tk, lb in cb]
    upd64, l64 = otrain.local_update(Net64, spec, gl.double(), cb64, masks=[m.double() for m in mk])
finally:
    torch.set_default_dtype(torch.float32)
w32 = torch.cat([u.reshape(-1) for u in upd32]).double()
w64 = torch.cat([u.reshape(-1) for u in upd64]).double()
wg = X1[k].cpu().double()
g0 = gl.double()
print(f"B={B} client {k}, {nst} step(s): loss gpu {loss1[k].item():.9g} ref32 {l32:.9g} ref64 {l64:.12g}; gpu clip norm {norms1[k].item():.9g}")
rows = []
off = 0
for name, shp in param_layout(spec):
    n = int(torch.Size(shp).numel())
    sl = slice(off, off + n)
    off += n
    u64 = w64[sl] - g0[sl]
    sc = u64.abs().max().item()
    if sc == 0:
        continue
    # parity.py's figure: forgive 2 ulp of the stored fp32 weight (the fp64 weight rounded to fp32)
    w64r = w64[sl].float()
    ulp = (torch.nextafter(w64r.abs(), torch.tensor(float("inf"))) - w64r.abs()).double()
    eg = ((wg[sl] - w64[sl]).abs() - 2 * ulp).clamp(min=0).max().item() / sc
    er = ((w32[sl] - w64[sl]).abs() - 2 * ulp).clamp(min=0).max().item() / sc
    d = (wg[sl] - w32[sl]).abs()
    i = int(d.argmax())
    rows.append((max(eg, er), name, eg, er, i, d[i].item(), (wg[sl] - g0[sl])[i].item(), (w32[sl] - g0[sl])[i].item(),
                 u64[i].item()))
rows.sort(reverse=True)
print("tensor: gpu-vs-fp64, ref32-vs-fp64 (max err / max |u64|); at the largest gpu-ref32 difference: index, |diff|, u_gpu, u_ref32, u_64")
for r in rows[:10]:
    print(f"  {r[1]:34s} gpu {r[2]:.2e}  ref32 {r[3]:.2e}  @{r[4]} diff {r[5]:.2e} u_gpu {r[6]:.6e} u_ref {r[7]:.6e} u64 {r[8]:.6e}")
