"""a3: the HIP GRU gate kernels (flr_gru_fwd_step / flr_gru_bwd_step) inside
ClientGRU vs the same recurrence in fp64 torch ops (nn.GRU's cell,
h' = (h - n) * z + n).  Tolerance 2e-6 x scale (fp32 pointwise + GEMM order)."""
import pytest
import torch

from flr.models.multimodal import _gru_torch
from flr.nn import client_gru

pytestmark = pytest.mark.gpu

SHAPES = [  # (K, B, T, H)
    (3, 4, 5, 8),
    (2, 3, 1, 5),
    (4, 32, 16, 256),  # the model's text branch, 4 clients
    (2, 32, 4, 300),   # H not a multiple of the fused kernels' 32-unit blocks
    (2, 33, 3, 40),    # B > 32: the batched-GEMM + gate-kernel path
]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_gru_fwd_bwd_vs_fp64(cuda, shape):
    K, B, T, H = shape
    g = torch.Generator().manual_seed(K * 1000 + T * 10 + H)
    gi = torch.randn(K, B, T, 3 * H, generator=g)
    whh = torch.randn(K, 3 * H, H, generator=g) / H ** 0.5
    bhh = torch.randn(K, 3 * H, generator=g) * 0.1
    dy = torch.randn(K, B, H, generator=g)
    args = [t.to(cuda).requires_grad_(True) for t in (gi, whh, bhh)]
    h = client_gru(*args)
    h.backward(dy.to(cuda))
    ref = [t.double().requires_grad_(True) for t in (gi, whh, bhh)]
    hr = _gru_torch(*ref)
    hr.backward(dy.double())
    for got, want in [(h, hr)] + [(a.grad, r.grad) for a, r in zip(args, ref)]:
        err = (got.detach().cpu().double() - want.detach()).abs().max().item()
        scale = want.detach().abs().max().item()
        assert err <= 2e-6 * max(scale, 1.0), (err, scale)
