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


@pytest.mark.parametrize("NI", [32, 16])
def test_stem_bn_relu_pool_fused_bit_identical(cuda, NI):
    """flr_batchnorm_relu_maxpool_fwd / flr_maxpool_relu_batchnorm_bwd (the
    ResNet stem's bn1 -> relu -> maxpool in one kernel each way) equal the
    three-kernel composition bit for bit: pooled values, argmax, statistics,
    dx, dgamma, dbeta — with window ties (a constant image), a NaN and
    negative-only planes (ReLU zeros everywhere) among the planes."""
    from flr import _capi
    KC, H, W = 37, 16, 16
    g = torch.Generator(device="cpu").manual_seed(NI)
    x = torch.randn(KC, NI, H, W, generator=g)
    x[3] = 2.0                      # constant plane: every window ties
    x[5, 1, 4, 7] = float("nan")    # NaN wins its windows
    x[7] = -x[7].abs() - 1.0        # all negative before BN (not after: BN recentres)
    x[9, :, ::2, ::2] = 5.0         # ties inside windows
    x = x.to(cuda)
    gamma = torch.randn(KC, generator=g).to(cuda)
    gamma[11] = -1.0                # negative scale flips the ReLU region
    beta = torch.randn(KC, generator=g).to(cuda)
    dyp = torch.randn(KC, NI, H // 2, W // 2, generator=g).to(cuda)
    st = torch.cuda.current_stream().cuda_stream
    # three-kernel reference
    a = torch.empty_like(x)
    m0, s0 = torch.empty(KC, device=cuda), torch.empty(KC, device=cuda)
    _capi.call("flr_batchnorm_fwd", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), None, a.data_ptr(),
               m0.data_ptr(), s0.data_ptr(), 1, KC, NI * H * W, 1e-5, 1, st)
    p0 = torch.empty(KC, NI, H // 2, W // 2, device=cuda)
    g0 = torch.empty(KC, NI, H // 2, W // 2, dtype=torch.uint8, device=cuda)
    _capi.call("flr_maxpool2d_fwd", a.data_ptr(), p0.data_ptr(), g0.data_ptr(), KC * NI, H, W, 3, 3, 2, 1, st)
    da = torch.empty_like(x)
    _capi.call("flr_maxpool2d_bwd", dyp.data_ptr(), g0.data_ptr(), da.data_ptr(), KC * NI, H, W, 3, 3, 2, 1, st)
    dx0, dg0, db0 = torch.empty_like(x), torch.empty(KC, device=cuda), torch.empty(KC, device=cuda)
    _capi.call("flr_batchnorm_bwd", da.data_ptr(), x.data_ptr(), a.data_ptr(), gamma.data_ptr(), m0.data_ptr(),
               s0.data_ptr(), dx0.data_ptr(), dg0.data_ptr(), db0.data_ptr(), None, 1, KC, NI * H * W, 1, st)
    # fused
    p1, g1 = torch.full_like(p0, float("nan")), torch.full_like(g0, 255)
    m1, s1 = torch.empty(KC, device=cuda), torch.empty(KC, device=cuda)
    _capi.call("flr_batchnorm_relu_maxpool_fwd", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), p1.data_ptr(),
               g1.data_ptr(), m1.data_ptr(), s1.data_ptr(), KC, NI, H, W, 1e-5, st)
    dx1, dg1, db1 = torch.full_like(x, float("nan")), torch.empty(KC, device=cuda), torch.empty(KC, device=cuda)
    _capi.call("flr_maxpool_relu_batchnorm_bwd", dyp.data_ptr(), g0.data_ptr(), x.data_ptr(), gamma.data_ptr(),
               beta.data_ptr(), m0.data_ptr(), s0.data_ptr(), dx1.data_ptr(), dg1.data_ptr(), db1.data_ptr(), KC, NI,
               H, W, st)
    torch.cuda.synchronize()
    eq = lambda u, v: torch.equal(u.nan_to_num(7.0), v.nan_to_num(7.0))  # noqa: E731  (NaN positions must agree)
    assert eq(m1, m0) and eq(s1, s0)
    assert eq(p1, p0) and torch.equal(g1, g0)
    assert eq(dx1, dx0) and eq(dg1, dg0) and eq(db1, db0)
    assert not torch.isnan(dx1[0]).any()


def test_stem_fused_rejects_other_shapes(cuda):
    from flr import _capi
    x = torch.zeros(2, 8, 8, 8, device=cuda)
    v = torch.zeros(2, device=cuda)
    rc = _capi.lib().flr_batchnorm_relu_maxpool_fwd(x.data_ptr(), v.data_ptr(), v.data_ptr(), x.data_ptr(),
                                                    x.data_ptr(), v.data_ptr(), v.data_ptr(), 2, 8, 8, 8,
                                                    ctypes_float(1e-5), None)
    assert rc == -3  # FLR_ERR_UNSUPPORTED


def ctypes_float(v):
    import ctypes
    return ctypes.c_float(v)
