"""GPU: the client-batched conv kernels (activations [K*C, B, H, W]) vs fp64
grouped convolution (torch CPU, [B, K*C, H, W])."""
import pytest
import torch
import torch.nn.functional as F

from flr.nn import client_conv2d

pytestmark = pytest.mark.gpu


def cb(t):
    """torch's grouped layout [B, K*C, H, W] -> the engine's [K*C, B, H, W]."""
    return t.transpose(0, 1).contiguous()

SHAPES = [  # (K, B, Cin, H, W, Cout, KH, stride, pad)
    (3, 4, 3, 32, 32, 8, 7, 2, 3),     # stem 7x7/2 (direct stem kernels, Cout < 64)
    (2, 8, 3, 32, 32, 64, 7, 2, 3),    # the C3 stem: two image groups per client
    (2, 4, 3, 32, 32, 72, 7, 2, 3),    # stem, Cout past one 64-channel block
    (2, 5, 3, 32, 32, 16, 7, 2, 3),    # stem, B not a multiple of 4: the gathered GEMM
    (3, 4, 8, 8, 8, 8, 3, 1, 1),       # layer1 3x3
    (2, 4, 8, 8, 8, 16, 3, 2, 1),      # layer2 first conv, stride 2
    (2, 4, 8, 8, 8, 16, 1, 2, 0),      # downsample 1x1/2
    (2, 3, 16, 2, 2, 24, 3, 1, 1),     # tiny spatial
    (2, 5, 16, 1, 1, 70, 3, 1, 1),     # 1x1 spatial, ragged Cout
    (1, 2, 5, 7, 9, 3, 3, 2, 1),       # odd everything
    (4, 32, 64, 8, 8, 64, 3, 1, 1),    # real layer1 shape, 4 clients
    (8, 32, 256, 4, 4, 256, 3, 1, 1),  # layer3 conv2: split-K path
    (4, 32, 512, 1, 1, 512, 3, 1, 1),  # layer4 at 1x1: 8 of 9 taps dead, split-K
    (4, 32, 256, 2, 2, 512, 3, 2, 1),  # layer4 first conv: 2x2 -> 1x1, 4 taps live
    (3, 3, 64, 5, 5, 96, 3, 1, 1),     # fast loaders with ragged M and N tiles
    (2, 5, 32, 7, 7, 64, 3, 2, 1),     # fast fwd/dgrad (stride 2, odd size), generic wgrad (Cin % 64)
    (2, 4, 64, 8, 8, 128, 1, 2, 0),    # fast 1x1 stride-2 downsample
]


def _tol(shape, which):
    """Relative tolerance (of the output's max |value|) for an fp32 reduction:
    2e-6 up to 256 terms, then growing as sqrt(n) — the random-walk growth of
    sequential fp32 rounding (reduction lengths: fwd Cin*KS^2, dgrad
    Cout*KS^2, wgrad B*Ho*Wo)."""
    K, B, Cin, H, W, Cout, KS, stride, pad = shape
    Ho, Wo = (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1
    n = {"y": Cin * KS * KS, "dx": Cout * KS * KS, "dw": B * Ho * Wo}[which]
    return 2e-6 * max(1.0, (n / 256) ** 0.5)


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_conv_fwd_bwd_vs_fp64(cuda, shape):
    K, B, Cin, H, W, Cout, KS, stride, pad = shape
    g = torch.Generator(device="cpu").manual_seed(sum(shape))
    x = torch.randn(B, K * Cin, H, W, generator=g)
    w = torch.randn(K, Cout, Cin, KS, KS, generator=g) * 0.1
    xg = cb(x).to(cuda).requires_grad_(True)
    wg = w.to(cuda).requires_grad_(True)
    y = client_conv2d(xg, wg, stride, pad).transpose(0, 1)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy.to(cuda))
    xd = x.double().requires_grad_(True)
    wd = w.double().requires_grad_(True)
    yr = F.conv2d(xd, wd.reshape(K * Cout, Cin, KS, KS), stride=stride, padding=pad, groups=K)
    yr.backward(dy.double())
    for which, got, ref in (("y", y, yr), ("dx", xg.grad.transpose(0, 1), xd.grad), ("dw", wg.grad, wd.grad)):
        err = (got.detach().cpu().double() - ref.detach()).abs().max().item()
        scale = ref.detach().abs().max().item()
        assert err <= _tol(shape, which) * max(scale, 1.0), (which, err, scale)


TAP_SHAPES = [s for s in SHAPES if s[2] % 64 == 0 and s[5] % 64 == 0] + [
    (2, 3, 64, 3, 5, 128, 3, 1, 1),    # ragged N tile, odd spatial
    (3, 2, 128, 2, 2, 64, 1, 1, 0),    # 1x1 stride 1, HoWo % 4 == 0
    (2, 5, 64, 3, 3, 64, 3, 2, 1),     # wgrad B gather (HoWo = 4 -> vec), dgrad stride 2
    (2, 3, 64, 3, 3, 64, 3, 1, 1),     # HoWo = 9: wgrad B gather path
    (2, 4, 64, 7, 6, 64, 3, 2, 1),     # dgrad parity classes of unequal size (odd H, even W)
    (1, 2, 64, 7, 7, 64, 3, 3, 1),     # stride 3: nine classes
    (2, 3, 64, 5, 4, 128, 1, 2, 0),    # 1x1/2: three of four classes have no tap (zero dx)
    (32, 32, 512, 1, 1, 512, 3, 1, 1),  # flattened multi-tile wgrad (R = 32, 2 tiles per workgroup)
    (16, 32, 256, 2, 2, 256, 3, 1, 1),  # flattened wgrad, R = 128 (4 K-tiles per tile)
]


@pytest.mark.parametrize("shape", TAP_SHAPES, ids=[str(s) for s in TAP_SHAPES])
def test_tap_major_conv_vs_fp64(cuda, shape):
    from flr.models.multimodal import from_tap_major, to_tap_major
    from flr.nn import client_conv2d_t, tap_major_ok
    K, B, Cin, H, W, Cout, KS, stride, pad = shape
    assert tap_major_ok(Cin, Cout)
    g = torch.Generator(device="cpu").manual_seed(sum(shape) + 1)
    x = torch.randn(B, K * Cin, H, W, generator=g)
    w = torch.randn(K, Cout, Cin, KS, KS, generator=g) * 0.1
    xg = cb(x).to(cuda).requires_grad_(True)
    wt = to_tap_major(w).contiguous().to(cuda).requires_grad_(True)
    y = client_conv2d_t(xg, wt, stride, pad).transpose(0, 1)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy.to(cuda))
    xd = x.double().requires_grad_(True)
    wd = w.double().requires_grad_(True)
    yr = F.conv2d(xd, wd.reshape(K * Cout, Cin, KS, KS), stride=stride, padding=pad, groups=K)
    yr.backward(dy.double())
    dw = from_tap_major(wt.grad.detach().cpu())
    for which, got, ref in (("y", y, yr), ("dx", xg.grad.transpose(0, 1), xd.grad), ("dw", dw, wd.grad)):
        err = (got.detach().cpu().double() - ref.detach()).abs().max().item()
        scale = ref.detach().abs().max().item()
        assert err <= _tol(shape, which) * max(scale, 1.0), (which, err, scale)


def _run_tap_major(cuda, shape, seed):
    from flr.models.multimodal import to_tap_major
    from flr.nn import client_conv2d_t
    K, B, Cin, H, W, Cout, KS, stride, pad = shape
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B, K * Cin, H, W, generator=g)
    w = torch.randn(K, Cout, Cin, KS, KS, generator=g) * 0.1
    xg = cb(x).to(cuda).requires_grad_(True)
    wt = to_tap_major(w).contiguous().to(cuda).requires_grad_(True)
    y = client_conv2d_t(xg, wt, stride, pad)
    dy = torch.randn(y.shape, generator=g).to(cuda)
    y.backward(dy)
    torch.cuda.synchronize()
    return y.detach().clone(), xg.grad.clone(), wt.grad.clone()


@pytest.mark.parametrize("form", ["pipe", "old"])
@pytest.mark.parametrize("shape", TAP_SHAPES, ids=[str(s) for s in TAP_SHAPES])
def test_gemm_forms_bit_identical(cuda, shape, form, knob):
    """Every bf16x6 form (FLR_GEMM: the default split at stash time (bf16 LDS
    images; the weight gradient's transposed images) where the plan supports
    it, "pipe", "old"; the split-at-stash kernels' prefetch depth) feeds each
    accumulator the same products in the same order: bit-identical results."""
    from flr import _capi
    if form == "old" and "ablation" not in _capi.build_info():
        pytest.skip("the unpipelined loop is a tools-build form (make ABLATION=1)")
    ref = _run_tap_major(cuda, shape, 7)
    knob("FLR_GEMM", form)
    got = _run_tap_major(cuda, shape, 7)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dims", [(3, 32, 768, 256), (2, 200, 130, 96), (4, 64, 64, 48)])
def test_bgemm_forms_bit_identical(cuda, dims, knob):
    from flr.nn import bgemm
    K, M, N, R = dims
    g = torch.Generator(device="cpu").manual_seed(M + N)
    A = torch.randn(K, M, R, generator=g).to(cuda)
    Bm = torch.randn(K, N, R, generator=g).to(cuda)
    from flr import _capi
    outs = []
    # default (row-major images), the per-wave split; the tools build adds
    # k-contiguous operands on transposed images (measured slower)
    forms = [None, "pipe"] + (["FLR_BGEMM_TIMG=1"] if "ablation" in _capi.build_info() else [])
    for form in forms:
        if form and "=" in form:
            knob("FLR_GEMM", None)
            knob(*form.split("="))
        elif form:
            knob("FLR_GEMM", form)
        outs.append([bgemm(A, Bm).clone(), bgemm(A.transpose(1, 2).contiguous().transpose(1, 2), Bm).clone(),
                     bgemm(A, Bm.transpose(1, 2).contiguous().transpose(1, 2)).clone()])
    torch.cuda.synchronize()
    for f in range(1, len(outs)):
        for i in range(3):
            assert torch.equal(outs[0][i], outs[f][i]), (forms[f], i)


NORM_SHAPES = [  # ResNet-18 layers at the C3 shapes (B = 32): split-K wgrad (l1), one tile pass, dead taps (l4)
    (4, 32, 64, 8, 8, 64, 3, 1, 1),
    (4, 32, 128, 4, 4, 128, 3, 1, 1),
    (4, 32, 256, 2, 2, 256, 3, 1, 1),
    (4, 32, 512, 1, 1, 512, 3, 1, 1),
    (4, 32, 256, 2, 2, 512, 3, 2, 1),
    (4, 32, 64, 8, 8, 128, 1, 2, 0),
]


@pytest.mark.parametrize("shape", NORM_SHAPES, ids=[str(s) for s in NORM_SHAPES])
def test_wgrad_norm_partials(cuda, shape):
    """flr_conv2d_bwd_weight_t_sq: the same dw_t as flr_conv2d_bwd_weight_t
    (bit-identical), and per-client partials that sum to sum(dw^2) (fp64, the
    clip norm of run_experiments.py:234) within 1e-12; the partials of a client
    do not depend on how many clients share the launch (K = 4 vs K = 1)."""
    from flr import _capi
    from flr.nn import _stream, _workspace_t
    K, B, Cin, H, W, Cout, KS, stride, pad = shape
    g = torch.Generator(device="cpu").manual_seed(sum(shape))
    x = torch.randn(K * Cin, B, H, W, generator=g).to(cuda)
    Ho = (H + 2 * pad - KS) // stride + 1
    dy = torch.randn(K * Cout, B, Ho, Ho, generator=g).to(cuda)
    outs = []
    for k_lo, k_n in ((0, K), (2, 1)):
        geom = (k_n, B, Cin, H, W, Cout, KS, KS, stride, pad)
        n = int(_capi.lib().flr_conv2d_bwd_weight_t_sq_slots(*geom))
        assert n > 0
        ws, nb = _workspace_t(geom, cuda)
        wsp = None if ws is None else ws.data_ptr()
        xs, dys = x[k_lo * Cin:(k_lo + k_n) * Cin], dy[k_lo * Cout:(k_lo + k_n) * Cout]
        dw_ref = torch.zeros(k_n, KS, KS, Cin, Cout, device=cuda)
        dw = torch.zeros_like(dw_ref)
        sq = torch.full((k_n, n + 3), float("nan"), dtype=torch.float64, device=cuda)
        _capi.call("flr_conv2d_bwd_weight_t", xs.data_ptr(), dys.data_ptr(), dw_ref.data_ptr(), *geom, 1, wsp, nb,
                   _stream(x))
        _capi.call("flr_conv2d_bwd_weight_t_sq", xs.data_ptr(), dys.data_ptr(), dw.data_ptr(), *geom, 1,
                   sq.data_ptr(), n + 3, wsp, nb, _stream(x))
        torch.cuda.synchronize()
        assert torch.equal(dw, dw_ref)
        assert torch.isnan(sq[:, n:]).all()  # nothing past the slot count
        want = dw.double().pow(2).reshape(k_n, -1).sum(1)
        got = sq[:, :n].sum(1)
        assert torch.allclose(got, want, rtol=1e-12, atol=0), (got, want)
        outs.append(sq[:, :n].cpu())
    assert torch.equal(outs[0][2], outs[1][0])


@pytest.mark.parametrize("form", [None, "pipe"])
@pytest.mark.parametrize("shape", TAP_SHAPES, ids=[str(s) for s in TAP_SHAPES])
def test_dgrad_addend_bit_identical(cuda, shape, form, knob):
    """flr_conv2d_bwd_data_t_add: dx = dgrad + add in the epilogue (linear
    stride-1 stores, the parity-class stores, the split-K reduce, classes with
    no tap) equals flr_conv2d_bwd_data_t followed by one fp32 add — the sum
    autograd forms of a residual block's two input-gradient paths."""
    from flr import _capi
    from flr.nn import _stream, _workspace_t
    if form:
        knob("FLR_GEMM", form)
    K, B, Cin, H, W, Cout, KS, stride, pad = shape
    g = torch.Generator(device="cpu").manual_seed(sum(shape) + 3)
    Ho, Wo = (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1
    dy = torch.randn(K * Cout, B, Ho, Wo, generator=g).to(cuda)
    wt = (torch.randn(K, KS, KS, Cin, Cout, generator=g) * 0.1).to(cuda)
    add = torch.randn(K * Cin, B, H, W, generator=g).to(cuda)
    geom = (K, B, Cin, H, W, Cout, KS, KS, stride, pad)
    ws, nb = _workspace_t(geom, cuda)
    wsp = None if ws is None else ws.data_ptr()
    dx = torch.full_like(add, float("nan"))
    _capi.call("flr_conv2d_bwd_data_t", dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), *geom, wsp, nb, _stream(dy))
    want = dx + add
    got = torch.full_like(add, float("nan"))
    _capi.call("flr_conv2d_bwd_data_t_add", dy.data_ptr(), wt.data_ptr(), add.data_ptr(), got.data_ptr(), *geom,
               wsp, nb, _stream(dy))
    torch.cuda.synchronize()
    assert torch.equal(got, want)

    # in place (add == dx): dx += dgrad, the classes no tap reaches left untouched
    inplace = add.clone()
    _capi.call("flr_conv2d_bwd_data_t_add", dy.data_ptr(), wt.data_ptr(), inplace.data_ptr(), inplace.data_ptr(),
               *geom, wsp, nb, _stream(dy))
    torch.cuda.synchronize()
    assert torch.equal(inplace, want)


@pytest.mark.parametrize("shape", [(32, 32, 512, 1, 1, 512, 3, 1, 1), (8, 8, 256, 2, 2, 512, 3, 2, 1),
                                   (5, 24, 256, 1, 1, 256, 1, 1, 0), (3, 32, 256, 2, 2, 512, 1, 2, 0)],
                         ids=["l4b", "l4a", "1x1-n24", "l4ds"])
def test_narrow_tiles_bit_identical(cuda, shape, knob):
    """The l4 convolutions' narrow-N tiles (N = B*Ho*Wo <= 32: four waves stacked
    along M) give the 64 x 64-tile kernels' bits: forward, data gradient (incl.
    the strided classes and the in-place addend) and split-K."""
    from flr import _capi
    from flr.nn import _stream, _workspace_t
    K, B, Cin, H, W, Cout, KS, stride, pad = shape
    g = torch.Generator(device="cpu").manual_seed(sum(shape))
    Ho, Wo = (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1
    x = torch.randn(K * Cin, B, H, W, generator=g).to(cuda)
    dy = torch.randn(K * Cout, B, Ho, Wo, generator=g).to(cuda)
    wt = (torch.randn(K, KS, KS, Cin, Cout, generator=g) * 0.1).to(cuda)
    add = torch.randn(K * Cin, B, H, W, generator=g).to(cuda)
    geom = (K, B, Cin, H, W, Cout, KS, KS, stride, pad)
    ws, nb = _workspace_t(geom, cuda)
    wsp = None if ws is None else ws.data_ptr()
    outs = []
    for narrow in ("1", "0"):
        knob("FLR_CONV_NARROW", narrow)
        y = torch.full((K * Cout, B, Ho, Wo), float("nan"), device=cuda)
        _capi.call("flr_conv2d_fwd_t", x.data_ptr(), wt.data_ptr(), y.data_ptr(), *geom, wsp, nb, _stream(x))
        dx = torch.full_like(x, float("nan"))
        _capi.call("flr_conv2d_bwd_data_t", dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), *geom, wsp, nb, _stream(x))
        acc = add.clone()
        _capi.call("flr_conv2d_bwd_data_t_add", dy.data_ptr(), wt.data_ptr(), acc.data_ptr(), acc.data_ptr(), *geom,
                   wsp, nb, _stream(x))
        torch.cuda.synchronize()
        outs.append((y.cpu(), dx.cpu(), acc.cpu()))
    for a, b in zip(*outs):
        assert not torch.isnan(a).any()
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(16, 32, 128, 4, 4, 128, 3, 1, 1), (16, 32, 256, 2, 2, 256, 3, 1, 1),
                                   (16, 32, 128, 4, 4, 256, 3, 2, 1), (16, 32, 64, 8, 8, 128, 3, 2, 1),
                                   (4, 32, 64, 8, 8, 64, 3, 1, 1), (16, 32, 128, 4, 4, 256, 1, 2, 0),
                                   (16, 32, 512, 1, 1, 512, 3, 1, 1), (16, 32, 256, 2, 2, 512, 3, 2, 1)],
                         ids=["l2b", "l3b", "l3a", "l2a", "l1-k4", "l3ds", "l4b-narrow", "l4a-narrow"])
def test_fill_tiles_bit_identical(cuda, shape, knob):
    """Small client counts (K/G per GPU) run the forward and data-gradient
    launches whose default grid is under one wave of the chip on 64 x 64 tiles
    with the default tile's split-K count (FLR_CONV_FILL): the same bits as
    the default tiles — forward, data gradient (strided classes, split-K) and
    the in-place addend; the l4 layers' narrow tiles (N = 32) likewise."""
    from flr import _capi
    from flr.nn import _stream, _workspace_t
    K, B, Cin, H, W, Cout, KS, stride, pad = shape
    g = torch.Generator(device="cpu").manual_seed(sum(shape) + 11)
    Ho, Wo = (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1
    x = torch.randn(K * Cin, B, H, W, generator=g).to(cuda)
    dy = torch.randn(K * Cout, B, Ho, Wo, generator=g).to(cuda)
    wt = (torch.randn(K, KS, KS, Cin, Cout, generator=g) * 0.1).to(cuda)
    add = torch.randn(K * Cin, B, H, W, generator=g).to(cuda)
    geom = (K, B, Cin, H, W, Cout, KS, KS, stride, pad)
    ws, nb = _workspace_t(geom, cuda)
    wsp = None if ws is None else ws.data_ptr()
    outs = []
    for fill in ("1", "0"):
        knob("FLR_CONV_FILL", fill)
        y = torch.full((K * Cout, B, Ho, Wo), float("nan"), device=cuda)
        _capi.call("flr_conv2d_fwd_t", x.data_ptr(), wt.data_ptr(), y.data_ptr(), *geom, wsp, nb, _stream(x))
        dx = torch.full_like(x, float("nan"))
        _capi.call("flr_conv2d_bwd_data_t", dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), *geom, wsp, nb, _stream(x))
        acc = add.clone()
        _capi.call("flr_conv2d_bwd_data_t_add", dy.data_ptr(), wt.data_ptr(), acc.data_ptr(), acc.data_ptr(), *geom,
                   wsp, nb, _stream(x))
        torch.cuda.synchronize()
        outs.append((y.cpu(), dx.cpu(), acc.cpu()))
    for a, b in zip(*outs):
        assert not torch.isnan(a).any()
        assert torch.equal(a, b)
