"""a2: HIP BatchNorm(train) + residual + ReLU (flr_batchnorm_fwd/_bwd inside
ClientBatchNorm, on the engine's [K*C, B, H, W] layout) vs fp64 torch
F.batch_norm on the grouped layout [B, K*C, H, W].
Covers every plane size of the model (HW = 256, 64, 16, 4, 1), a non power of
two plane (7x9) and channel counts that leave a wave partially filled."""
import pytest
import torch
import torch.nn.functional as F

from flr.nn import client_batchnorm

pytestmark = pytest.mark.gpu

SHAPES = [  # (B, KC, H, W)
    (4, 6, 16, 16),
    (3, 10, 8, 8),
    (5, 7, 4, 4),
    (32, 20, 2, 2),
    (32, 130, 1, 1),
    (2, 3, 7, 9),
    (32, 256, 8, 8),
    (32, 3, 16, 16),   # the stem's planes (8192 values: a whole workgroup per plane)
    (16, 5, 16, 16),   # 4096 values per plane
    (2, 9, 1, 2),      # 4 values per plane, 9 planes
]
MODES = [(True, False), (True, True), (False, False), (False, True)]  # (relu, residual)


@pytest.mark.parametrize("mode", MODES, ids=[f"relu{int(a)}_res{int(b)}" for a, b in MODES])
@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_batchnorm_fwd_bwd_vs_fp64(cuda, shape, mode):
    relu, with_res = mode
    B, KC, H, W = shape
    g = torch.Generator().manual_seed(B * 7 + KC * 3 + H)
    x = torch.randn(B, KC, H, W, generator=g) * 2 + 0.5
    gam = torch.rand(KC, generator=g) + 0.5
    bet = torch.randn(KC, generator=g) * 0.1
    res = torch.randn(B, KC, H, W, generator=g) if with_res else None
    dy = torch.randn(B, KC, H, W, generator=g)
    # the engine's client-channel-major layout [KC, B, H, W]
    cb = lambda t: t.transpose(0, 1).contiguous()  # noqa: E731
    ins = [t.to(cuda).requires_grad_(True) for t in (cb(x), gam, bet)]
    rg = cb(res).to(cuda).requires_grad_(True) if with_res else None
    y = client_batchnorm(ins[0], ins[1], ins[2], rg, relu)
    y.backward(cb(dy).to(cuda))
    ref = [t.double().requires_grad_(True) for t in (x, gam, bet)]
    rr = res.double().requires_grad_(True) if with_res else None
    yr = F.batch_norm(ref[0], None, None, ref[1], ref[2], training=True, momentum=0.0, eps=1e-5)
    if with_res:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    yr.backward(dy.double())
    pairs = [(y.transpose(0, 1), yr), (ins[0].grad.transpose(0, 1), ref[0].grad)]
    pairs += [(a.grad, r.grad) for a, r in zip(ins[1:], ref[1:])]
    if with_res:
        pairs.append((rg.grad.transpose(0, 1), rr.grad))
    for got, want in pairs:
        err = (got.detach().cpu().double() - want.detach()).abs().max().item()
        scale = want.detach().abs().max().item()
        assert err <= 5e-6 * max(scale, 1.0), (err, scale)
