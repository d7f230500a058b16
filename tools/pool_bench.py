"""Time the max-pool kernels at the C3 stem shape (K=128 clients x 64 channels x
B=32 planes of 16x16, 3x3/2 pad 1)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-fl-security_amd"))
import torch
from flr import _capi
from flr.nn import _stream

n = 128 * 64 * 32
x = torch.randn(n, 16, 16, device="cuda")
y = torch.empty(n, 8, 8, device="cuda")
a = torch.empty(n, 8, 8, dtype=torch.uint8, device="cuda")
dx = torch.empty_like(x)
st = _stream(x)
fwd = lambda: _capi.call("flr_maxpool2d_fwd", x.data_ptr(), y.data_ptr(), a.data_ptr(), n, 16, 16, 3, 3, 2, 1, st)
bwd = lambda: _capi.call("flr_maxpool2d_bwd", y.data_ptr(), a.data_ptr(), dx.data_ptr(), n, 16, 16, 3, 3, 2, 1, st)
for name, fn, nbytes in [("fwd", fwd, 4 * n * 256 + 5 * n * 64), ("bwd", bwd, 4 * n * 256 + 5 * n * 64)]:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f"pool {name}: {us:.1f} us  {nbytes / us / 1e6:.2f} TB/s", flush=True)
