"""One batched-GEMM shape (vit.fc1 at K = 32: M 2080, N 1536, R 384) launched
20 times, for PMC passes of the 4-wave and the 8-wave ping-pong forms
(FLR_GEMM_PP8 read from the environment at library load)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch
from flr.nn import bgemm

g = torch.Generator().manual_seed(1)
A = torch.randn(32, 2080, 384, generator=g).cuda()
B = torch.randn(32, 1536, 384, generator=g).transpose(1, 2).contiguous().transpose(1, 2).cuda()
for _ in range(20):
    C = bgemm(A, B)
torch.cuda.synchronize()
print("ok", float(C.float().abs().sum()))
