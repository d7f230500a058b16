"""Autograd wrappers over the client-batched HIP layer kernels."""
from __future__ import annotations

import os

import torch

from . import _capi


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _workspace(geom, device):
    n = int(_capi.lib().flr_conv2d_workspace(*geom))
    if n == 0:
        return None, 0
    return torch.empty(n, dtype=torch.uint8, device=device), n


class ClientConv2d(torch.autograd.Function):
    """y[K*Cout, B, Ho, Wo] = conv(x[K*Cin, B, H, W], w[K, Cout, Cin, KH, KW]) per client
    (flr_conv2d_fwd / _bwd_data / _bwd_weight).  Activations are in the
    engine's client-channel-major layout [K][C][B][H][W]."""

    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int, need_dx: bool = True):
        x = x.contiguous()
        w = w.contiguous()
        K, Cout, Cin, KH, KW = w.shape
        KC, B, H, W = x.shape
        assert KC == K * Cin, (x.shape, w.shape)
        Ho = (H + 2 * pad - KH) // stride + 1
        Wo = (W + 2 * pad - KW) // stride + 1
        y = torch.empty(K * Cout, B, Ho, Wo, dtype=x.dtype, device=x.device)
        geom = (K, B, Cin, H, W, Cout, KH, KW, stride, pad)
        ws, n = _workspace(geom, x.device)
        _capi.call("flr_conv2d_fwd", x.data_ptr(), w.data_ptr(), y.data_ptr(), *geom,
                   None if ws is None else ws.data_ptr(), n, _stream(x))
        ctx.save_for_backward(x, w)
        ctx.geom = geom
        ctx.need_dx = need_dx
        ctx.fwd_ws = (ws, n)  # holds the forward's im2col column matrix for the weight gradient
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        g = ctx.geom
        fws, fn = ctx.fwd_ws
        ctx.fwd_ws = None
        ws, n = _workspace(g, dy.device)
        wsp = None if ws is None else ws.data_ptr()
        dx = None
        if ctx.need_dx and ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _capi.call("flr_conv2d_bwd_data", dy.data_ptr(), w.data_ptr(), dx.data_ptr(), *g, wsp, n, _stream(dy))
        dw = None
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w)
            if fws is not None:  # the forward's workspace: its column matrix is reused
                _capi.call("flr_conv2d_bwd_weight_reuse", x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *g,
                           fws.data_ptr(), fn, _stream(dy))
            else:
                _capi.call("flr_conv2d_bwd_weight", x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *g, wsp, n,
                           _stream(dy))
        return dx, dw, None, None, None


class ClientConv2dT(torch.autograd.Function):
    """ClientConv2d with tap-major weights w_t [K, KH, KW, Cin, Cout]
    (flr_conv2d_fwd_t / _bwd_data_t / _bwd_weight_t; Cin, Cout multiples of 64)."""

    @staticmethod
    def forward(ctx, x, w_t, stride: int, pad: int, need_dx: bool = True, zero_dead: bool = True, norm_slot=None):
        x = x.contiguous()
        w_t = w_t.contiguous()
        ctx.zero_dead = zero_dead
        ctx.norm_slot = norm_slot  # a NormSlot or None
        K, KH, KW, Cin, Cout = w_t.shape
        KC, B, H, W = x.shape
        assert KC == K * Cin, (x.shape, w_t.shape)
        Ho = (H + 2 * pad - KH) // stride + 1
        Wo = (W + 2 * pad - KW) // stride + 1
        y = torch.empty(K * Cout, B, Ho, Wo, dtype=x.dtype, device=x.device)
        geom = (K, B, Cin, H, W, Cout, KH, KW, stride, pad)
        ws, n = _workspace_t(geom, x.device)
        _capi.call("flr_conv2d_fwd_t", x.data_ptr(), w_t.data_ptr(), y.data_ptr(), *geom,
                   None if ws is None else ws.data_ptr(), n, _stream(x))
        ctx.save_for_backward(x, w_t)
        ctx.geom = geom
        ctx.need_dx = need_dx
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_t = ctx.saved_tensors
        dy = dy.contiguous()
        g = ctx.geom
        ws, n = _workspace_t(g, dy.device)
        wsp = None if ws is None else ws.data_ptr()
        dx = None
        if ctx.need_dx and ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _capi.call("flr_conv2d_bwd_data_t", dy.data_ptr(), w_t.data_ptr(), dx.data_ptr(), *g, wsp, n,
                       _stream(dy))
        dw = None
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w_t)
            if ctx.norm_slot is None:
                _capi.call("flr_conv2d_bwd_weight_t", x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *g,
                           int(ctx.zero_dead), wsp, n, _stream(dy))
            else:  # + the clip norm's partial sums of squares (flr_clip_sgd_step_blocked_x extra_sq)
                s = ctx.norm_slot
                _capi.call("flr_conv2d_bwd_weight_t_sq", x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *g,
                           int(ctx.zero_dead), s.ptr, s.ld, wsp, n, _stream(dy))
                s.used = True
        return dx, dw, None, None, None, None, None


class NormSlot:
    """Where a conv weight gradient's clip-norm partials go (sq pointer, row
    stride); `used` is set by the backward that wrote them, so the optimizer
    can refuse a step whose norm would miss a block."""

    def __init__(self, ptr: int, ld: int):
        self.ptr, self.ld, self.used = ptr, ld, False


def _workspace_t(geom, device):
    n = int(_capi.lib().flr_conv2d_t_workspace(*geom))
    if n == 0:
        return None, 0
    return torch.empty(n, dtype=torch.uint8, device=device), n


def tap_major_ok(cin: int, cout: int) -> bool:
    return bool(_capi.lib().flr_conv2d_tap_major_ok(int(cin), int(cout)))


def client_conv2d_t(x: torch.Tensor, w_t: torch.Tensor, stride: int, pad: int, need_dx: bool = True,
                    zero_dead: bool = True, norm_slot=None) -> torch.Tensor:
    return ClientConv2dT.apply(x, w_t, stride, pad, need_dx, zero_dead, norm_slot)


def client_conv2d(x, w, stride: int, pad: int, need_dx: bool = True):
    return ClientConv2d.apply(x, w, stride, pad, need_dx)


def bgemm(A: torch.Tensor, B: torch.Tensor, bias=None, add=None, out=None) -> torch.Tensor:
    """out[k] = (bias[k] | add[k] | 0) + A[k] @ B[k]^T on flr_bgemm: A [K, M, R] and
    B [K, N, R] are any strided views (transposes are free), bias [K, N]
    (row stride 1), add shaped and strided like out (default: contiguous)."""
    K, M, R = A.shape
    N = B.shape[1]
    if B.shape[0] != K or B.shape[2] != R:
        raise ValueError(f"bgemm operand shapes {tuple(A.shape)} / {tuple(B.shape)}")
    if out is None:
        out = torch.empty(K, M, N, dtype=A.dtype, device=A.device)
    if add is not None and add.stride() != out.stride():
        raise ValueError("bgemm addend must share the output strides")
    if bias is not None and (bias.shape != (K, N) or bias.stride(1) != 1):
        raise ValueError("bgemm bias must be [K, N] with unit row stride")
    n = int(_capi.lib().flr_bgemm_workspace(K, M, N, R))
    ws = torch.empty(n, dtype=torch.uint8, device=A.device) if n else None
    _capi.call("flr_bgemm", A.data_ptr(), *A.stride(), B.data_ptr(), *B.stride(), out.data_ptr(), *out.stride(),
               _ptr(bias), 0 if bias is None else bias.stride(0), _ptr(add), K, M, N, R,
               None if ws is None else ws.data_ptr(), n, _stream(A))
    return out


def sum_rows(X: torch.Tensor) -> torch.Tensor:
    """[K, M, N] -> [K, N]: sum over m in order (flr_sum_rows); X row stride 1."""
    K, M, N = X.shape
    if X.stride(2) != 1:
        X = X.contiguous()
    out = torch.empty(K, N, dtype=X.dtype, device=X.device)
    n = int(_capi.lib().flr_sum_rows_workspace(K, M, N))
    ws = torch.empty(n, dtype=torch.uint8, device=X.device) if n else None
    _capi.call("flr_sum_rows_ex", X.data_ptr(), X.stride(0), X.stride(1), K, M, N, out.data_ptr(), N,
               None if ws is None else ws.data_ptr(), n, _stream(X))
    return out


class ClientLinear(torch.autograd.Function):
    """y[K, M, out] = x[K, M, in] W[K, out, in]^T + b[K, out] — nn.Linear of
    every client at once (fusion head and GRU input projection,
    cub200_cnn.py:88-93, 109-117 template) on the flr_bgemm MFMA kernel."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return bgemm(x, W, bias=b)

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dy = dy.contiguous()
        dx = bgemm(dy, W.transpose(1, 2)) if ctx.needs_input_grad[0] else None
        dW = bgemm(dy.transpose(1, 2), x.transpose(1, 2)) if ctx.needs_input_grad[1] else None
        db = sum_rows(dy) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dx, dW, db


def client_linear(x, W, b=None):
    return ClientLinear.apply(x, W, b)


def _gru_packed(ng: int, h: int, c: int) -> int:
    """Floats per client of a weight packed by flr_gru_pack: ng groups of
    ceil(h/32) row blocks x ceil(c/16) k-steps x 512."""
    return ng * ((h + 31) // 32) * ((c + 15) // 16) * 512


class ClientGRU(torch.autograd.Function):
    """Final hidden state of a 1-layer GRU (h_0 = 0) for K clients at once.

    gi [K, B, T, 3H] = x W_ih^T + b_ih (computed by the caller, so autograd
    handles W_ih, b_ih and the embedding), whh [K, 3H, H], bhh [K, 3H] ->
    h_T [K, B, H].  B <= 32: W_hh is packed once into MFMA-fragment order
    (flr_gru_pack) and each step is one flr_gru_fwd_fused launch (recurrence
    GEMM + gate math); backward packs W_hh^T and runs one flr_gru_bwd_fused
    per step.  Otherwise per step one flr_bgemm (h W_hh^T + b_hh) and one
    flr_gru_fwd_step / flr_gru_bwd_step.  dW_hh / db_hh over all steps at once
    (flr_bgemm, flr_sum_rows).
    """

    @staticmethod
    def forward(ctx, gi, whh, bhh):
        gi = gi.contiguous()
        K, B, T, H3 = gi.shape
        H = H3 // 3
        dev = gi.device
        hseq = torch.empty(K, T + 1, B, H, dtype=gi.dtype, device=dev)
        gates = torch.empty(K, T, B, 4, H, dtype=gi.dtype, device=dev)
        bias = bhh.contiguous()
        whh = whh.contiguous()
        st = _stream(gi)
        # FLR_GRU_FUSED=0: the batched GEMM + gate kernel per step (A/B timing)
        fused = B <= 32 and os.environ.get("FLR_GRU_FUSED", "1") != "0"
        if fused:  # one launch per step: the recurrence GEMM with the gate math in its epilogue
            fill_(hseq)  # h_0 = 0
            whhP = torch.empty(K, _gru_packed(3, H, H), dtype=whh.dtype, device=dev)
            _capi.call("flr_gru_pack", whh.data_ptr(), K, 3, H, H, 0, whhP.data_ptr(), st)
            for t in range(T):
                _capi.call("flr_gru_fwd_fused", gi.data_ptr(), whhP.data_ptr(), bias.data_ptr(), hseq.data_ptr(),
                           gates.data_ptr(), K, B, T, H, t, st)
        else:
            hseq[:, 0].zero_()
            gh = torch.empty(K, B, H3, dtype=gi.dtype, device=dev)
            for t in range(T):
                bgemm(hseq[:, t], whh, bias=bias, out=gh)
                _capi.call("flr_gru_fwd_step", gi.data_ptr(), gh.data_ptr(), hseq.data_ptr(), gates.data_ptr(),
                           K, B, T, H, t, st)
        ctx.save_for_backward(whh, hseq, gates)
        ctx.fused = fused
        return hseq[:, T].contiguous()

    @staticmethod
    def backward(ctx, dhT):
        whh, hseq, gates = ctx.saved_tensors
        K, T, B, _, H = gates.shape
        dev = dhT.device
        dgh = torch.empty(K, T, B, 3 * H, dtype=dhT.dtype, device=dev)
        dgi = torch.empty(K, B, T, 3 * H, dtype=dhT.dtype, device=dev)
        dh = dhT.contiguous()
        dh_direct = torch.empty(K, B, H, dtype=dhT.dtype, device=dev)
        st = _stream(dh)
        if ctx.fused:  # step T-1's gate backward, then one launch per earlier step (GEMM + gate backward)
            whhT = torch.empty(K, _gru_packed(1, H, 3 * H), dtype=whh.dtype, device=dev)  # W_hh^T, packed
            _capi.call("flr_gru_pack", whh.data_ptr(), K, 1, H, 3 * H, 1, whhT.data_ptr(), st)
            _capi.call("flr_gru_bwd_step", dh.data_ptr(), gates.data_ptr(), hseq.data_ptr(), dgh.data_ptr(),
                       dgi.data_ptr(), dh_direct.data_ptr(), K, B, T, H, T - 1, st)
            for t in range(T - 1, 0, -1):
                _capi.call("flr_gru_bwd_fused", whhT.data_ptr(), gates.data_ptr(), hseq.data_ptr(), dgh.data_ptr(),
                           dgi.data_ptr(), dh_direct.data_ptr(), None, K, B, T, H, t, st)
        else:
            for t in range(T - 1, -1, -1):
                _capi.call("flr_gru_bwd_step", dh.data_ptr(), gates.data_ptr(), hseq.data_ptr(), dgh.data_ptr(),
                           dgi.data_ptr(), dh_direct.data_ptr(), K, B, T, H, t, st)
                if t > 0:  # dL/dh_t = z-path + dgh_t W_hh   (dL/dh_0 is not needed)
                    dh = bgemm(dgh[:, t], whh.transpose(1, 2), add=dh_direct)
        dgh2 = dgh.view(K, T * B, 3 * H)
        dwhh = bgemm(dgh2.transpose(1, 2), hseq[:, :T].reshape(K, T * B, H).transpose(1, 2))
        dbhh = sum_rows(dgh2)
        return dgi, dwhh, dbhh


def client_gru(gi: torch.Tensor, whh: torch.Tensor, bhh: torch.Tensor) -> torch.Tensor:
    return ClientGRU.apply(gi, whh, bhh)


def _ptr(t):
    return None if t is None else t.data_ptr()


class ClientBatchNorm(torch.autograd.Function):
    """out = act(BN_train(x) [+ residual]) per (client, channel) plane of the
    client-channel-major layout x[K*C, B, H, W] — each plane is one contiguous
    run of B*H*W values, passed to flr_batchnorm_fwd/_bwd as B = 1;
    gamma/beta [K, C]."""

    @staticmethod
    def forward(ctx, x, gamma, beta, residual, relu: bool, eps: float):
        x = x.contiguous()
        B, KC = 1, x.shape[0]
        HW = x[0].numel()
        g = gamma.contiguous()
        b = beta.contiguous()
        assert g.numel() == KC and b.numel() == KC, (x.shape, gamma.shape)
        res = None if residual is None else residual.contiguous()
        y = torch.empty_like(x)
        mean = torch.empty(KC, dtype=x.dtype, device=x.device)
        invstd = torch.empty_like(mean)
        _capi.call("flr_batchnorm_fwd", x.data_ptr(), g.data_ptr(), b.data_ptr(), _ptr(res), y.data_ptr(),
                   mean.data_ptr(), invstd.data_ptr(), B, KC, HW, eps, int(relu), _stream(x))
        ctx.save_for_backward(x, y if relu else None, g, mean, invstd)
        ctx.relu = relu
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, g, mean, invstd = ctx.saved_tensors
        dy = dy.contiguous()
        B, KC = 1, x.shape[0]
        HW = x[0].numel()
        dx = torch.empty_like(x)
        dg = torch.empty_like(g)
        db = torch.empty_like(g)
        dres = torch.empty_like(x) if ctx.has_res and ctx.needs_input_grad[3] else None
        _capi.call("flr_batchnorm_bwd", dy.data_ptr(), x.data_ptr(), _ptr(y), g.data_ptr(), mean.data_ptr(),
                   invstd.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), _ptr(dres), B, KC, HW,
                   int(ctx.relu), _stream(dy))
        return dx, dg, db, dres, None, None


def client_batchnorm(x, gamma, beta, residual=None, relu: bool = True, eps: float = 1e-5):
    return ClientBatchNorm.apply(x, gamma, beta, residual, relu, eps)


def client_batchnorm_infer(x, gamma, beta, running_mean, running_var, residual=None, relu: bool = True,
                           eps: float = 1e-5):
    """model.eval() BatchNorm (+ residual, ReLU) on flr_batchnorm_infer; forward
    only.  x [K*C, ...] (one contiguous plane per row), stats / affine [K*C]."""
    x = x.contiguous()
    KC = x.shape[0]
    res = None if residual is None else residual.contiguous()
    y = torch.empty_like(x)
    args = [t.contiguous().reshape(-1) for t in (gamma, beta, running_mean, running_var)]
    assert all(a.numel() == KC for a in args), (x.shape, [a.numel() for a in args])
    _capi.call("flr_batchnorm_infer", x.data_ptr(), *[a.data_ptr() for a in args], _ptr(res), y.data_ptr(), KC,
               x[0].numel(), eps, int(relu), _stream(x))
    return y


class ClientMaxPool2d(torch.autograd.Function):
    """F.max_pool2d over every H x W plane of x[..., H, W] (flr_maxpool2d_fwd/_bwd)."""

    @staticmethod
    def forward(ctx, x, k: int, stride: int, pad: int):
        x = x.contiguous()
        H, W = x.shape[-2:]
        planes = x.numel() // (H * W)
        Ho = (H + 2 * pad - k) // stride + 1
        Wo = (W + 2 * pad - k) // stride + 1
        y = torch.empty(*x.shape[:-2], Ho, Wo, dtype=x.dtype, device=x.device)
        arg = torch.empty(*x.shape[:-2], Ho, Wo, dtype=torch.uint8, device=x.device)
        _capi.call("flr_maxpool2d_fwd", x.data_ptr(), y.data_ptr(), arg.data_ptr(), planes, H, W, k, k, stride, pad,
                   _stream(x))
        ctx.save_for_backward(arg)
        ctx.geom = (planes, H, W, k, k, stride, pad)
        ctx.xshape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty(ctx.xshape, dtype=dy.dtype, device=dy.device)
        _capi.call("flr_maxpool2d_bwd", dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), *ctx.geom, _stream(dy))
        return dx, None, None, None


def client_maxpool2d(x, k: int, stride: int, pad: int):
    return ClientMaxPool2d.apply(x, k, stride, pad)


# ---------------------------------------------------------------------------
# a3 / a4 / C4-C5 encoders: embedding, fused-epilogue GEMM, LayerNorm, attention
# ---------------------------------------------------------------------------

ACT = {"none": 0, "relu": 1, "gelu": 2, "tanh": 3, "drelu": 4, "dgelu": 5, "dtanh": 6}


def fill_(t: torch.Tensor, value: float = 0.0) -> torch.Tensor:
    """t[...] = value on the flr_fill kernel (contiguous t)."""
    assert t.is_contiguous()
    _capi.call("flr_fill", t.data_ptr(), t.numel(), float(value), _stream(t))
    return t


def bgemm_ex(A: torch.Tensor, B: torch.Tensor, bias=None, add=None, act: str = "none", mul=None, aux=None,
             pre=None, out=None) -> torch.Tensor:
    """bgemm with the fused epilogue of flr_bgemm_ex: pre <- v; v <- act(v, aux);
    v <- v * mul.  add / mul / aux / pre share out's strides."""
    K, M, R = A.shape
    N = B.shape[1]
    if B.shape[0] != K or B.shape[2] != R:
        raise ValueError(f"bgemm operand shapes {tuple(A.shape)} / {tuple(B.shape)}")
    if out is None:
        out = torch.empty(K, M, N, dtype=A.dtype, device=A.device)
    for name, t in (("add", add), ("mul", mul), ("aux", aux), ("pre", pre)):
        if t is not None and (t.shape != out.shape or t.stride() != out.stride()):
            raise ValueError(f"bgemm_ex {name} must share the output's shape and strides")
    if bias is not None and (bias.shape != (K, N) or bias.stride(1) != 1):
        raise ValueError("bgemm bias must be [K, N] with unit row stride")
    n = int(_capi.lib().flr_bgemm_workspace(K, M, N, R))
    ws = torch.empty(n, dtype=torch.uint8, device=A.device) if n else None
    _capi.call("flr_bgemm_ex", A.data_ptr(), *A.stride(), B.data_ptr(), *B.stride(), out.data_ptr(), *out.stride(),
               _ptr(bias), 0 if bias is None else bias.stride(0), _ptr(add), ACT[act], _ptr(mul), _ptr(aux),
               _ptr(pre), K, M, N, R, None if ws is None else ws.data_ptr(), n, _stream(A))
    return out


class ClientEmbedding(torch.autograd.Function):
    """out[K, N, E] = table[K, V, E][ids[K, N]] (nn.Embedding per client) on
    flr_embedding_fwd; backward: flr_embedding_bwd, torch's index_add order."""

    @staticmethod
    def forward(ctx, table, ids):
        K, V, E = table.shape
        table = table.contiguous()
        ids = ids.reshape(K, -1).contiguous()
        N = ids.shape[1]
        out = torch.empty(K, N, E, dtype=table.dtype, device=table.device)
        _capi.call("flr_embedding_fwd", table.data_ptr(), V * E, V, ids.data_ptr(), N, None, 0, 0, None, 0, None, 0, 0,
                   None, 0, K, N, E, out.data_ptr(), _stream(table))
        ctx.save_for_backward(ids)
        ctx.shape = (K, V, E, N)
        return out

    @staticmethod
    def backward(ctx, dout):
        (ids,) = ctx.saved_tensors
        K, V, E, N = ctx.shape
        dout = dout.contiguous()
        dtab = torch.empty(K, V, E, dtype=dout.dtype, device=dout.device)
        n = int(_capi.lib().flr_embedding_bwd_workspace(K, N))
        ws = torch.empty(n, dtype=torch.uint8, device=dout.device)
        _capi.call("flr_embedding_bwd", dout.data_ptr(), ids.data_ptr(), N, K, N, V, E, dtab.data_ptr(), V * E, 1,
                   ws.data_ptr(), n, _stream(dout))
        return dtab, None


def client_embedding(table: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    return ClientEmbedding.apply(table, ids)


class ClientEmbeddingSum(torch.autograd.Function):
    """BERT embeddings before the LayerNorm: (word[ids] + type[type_ids]) +
    pos[pos_ids] per client (one flr_embedding_fwd); each table's gradient is
    its own flr_embedding_bwd.  ids [K, N]; type_ids / pos_ids [N] shared by
    every client (client stride 0)."""

    @staticmethod
    def forward(ctx, word, typ, pos, ids, type_ids, pos_ids):
        K, V, E = word.shape
        word, typ, pos = word.contiguous(), typ.contiguous(), pos.contiguous()
        ids = ids.reshape(K, -1).contiguous()
        N = ids.shape[1]
        Vt, Vp = typ.shape[1], pos.shape[1]
        out = torch.empty(K, N, E, dtype=word.dtype, device=word.device)
        _capi.call("flr_embedding_fwd", word.data_ptr(), V * E, V, ids.data_ptr(), N,
                   typ.data_ptr(), Vt * E, Vt, type_ids.data_ptr(), 0,
                   pos.data_ptr(), Vp * E, Vp, pos_ids.data_ptr(), 0, K, N, E, out.data_ptr(), _stream(word))
        ctx.save_for_backward(ids, type_ids, pos_ids)
        ctx.shape = (K, E, N, V, Vt, Vp)
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, type_ids, pos_ids = ctx.saved_tensors
        K, E, N, V, Vt, Vp = ctx.shape
        dout = dout.contiguous()
        n = int(_capi.lib().flr_embedding_bwd_workspace(K, N))
        ws = torch.empty(n, dtype=torch.uint8, device=dout.device)
        grads = []
        for idv, ik, rows in ((ids, N, V), (type_ids, 0, Vt), (pos_ids, 0, Vp)):
            d = torch.empty(K, rows, E, dtype=dout.dtype, device=dout.device)
            _capi.call("flr_embedding_bwd", dout.data_ptr(), idv.data_ptr(), ik, K, N, rows, E, d.data_ptr(),
                       rows * E, 1, ws.data_ptr(), n, _stream(dout))
            grads.append(d)
        return grads[0], grads[1], grads[2], None, None, None


def client_embedding_sum(word, typ, pos, ids, type_ids, pos_ids):
    return ClientEmbeddingSum.apply(word, typ, pos, ids, type_ids, pos_ids)


class ClientLayerNorm(torch.autograd.Function):
    """y = LayerNorm(x [+ residual]) per client over rows of width D; with a
    residual it also returns s = x + residual (the encoder's residual stream)
    so the skip path's gradient can be handed back as the backward's addend.
    x / residual [K, R, D] contiguous, gamma / beta [K, D]."""

    @staticmethod
    def forward(ctx, x, residual, gamma, beta, eps: float):
        x = x.contiguous()
        K, R, D = x.shape
        y = torch.empty_like(x)
        mean = torch.empty(K * R, dtype=x.dtype, device=x.device)
        rstd = torch.empty_like(mean)
        s = None
        if residual is not None:
            residual = residual.contiguous()
            s = torch.empty_like(x)
        g, b = gamma.contiguous(), beta.contiguous()
        _capi.call("flr_layernorm_fwd", x.data_ptr(), D, _ptr(residual), D, g.data_ptr(), b.data_ptr(), y.data_ptr(),
                   D, _ptr(s), D, mean.data_ptr(), rstd.data_ptr(), K * R, D, R, eps, _stream(x))
        ctx.save_for_backward(x if s is None else s, g, mean, rstd)
        ctx.has_res = residual is not None
        return y, s

    @staticmethod
    def backward(ctx, dy, ds):
        s, g, mean, rstd = ctx.saved_tensors
        K, R, D = s.shape
        dy = dy.contiguous()
        dx = torch.empty_like(s)
        dg = torch.empty_like(g)
        db = torch.empty_like(g)
        dskip = None if ds is None else ds.contiguous()
        n = int(_capi.lib().flr_layernorm_bwd_workspace(K, R, D))
        ws = torch.empty(n, dtype=torch.uint8, device=dy.device)
        _capi.call("flr_layernorm_bwd", dy.data_ptr(), D, s.data_ptr(), D, g.data_ptr(), mean.data_ptr(),
                   rstd.data_ptr(), _ptr(dskip), D, dx.data_ptr(), D, dg.data_ptr(), db.data_ptr(), K, R, D,
                   ws.data_ptr(), n, _stream(dy))
        return dx, (dx if ctx.has_res else None), dg, db, None


def client_layernorm(x, gamma, beta, residual=None, eps: float = 1e-5):
    """Returns y (residual None) or (y, s = x + residual)."""
    y, s = ClientLayerNorm.apply(x, residual, gamma, beta, eps)
    return y if residual is None else (y, s)


class ClientAttention(torch.autograd.Function):
    """ctx [K, B, T, D] = softmax(q k^T / sqrt(64)) v per (client, batch row,
    head) from the fused projection qkv [K, B, T, 3D] (flr_attention_fwd/_bwd)."""

    @staticmethod
    def forward(ctx, qkv, heads: int):
        qkv = qkv.contiguous()
        K, B, T, D3 = qkv.shape
        D = D3 // 3
        out = torch.empty(K, B, T, D, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(K * B * heads * T, dtype=qkv.dtype, device=qkv.device)
        _capi.call("flr_attention_fwd", qkv.data_ptr(), K * B, T, heads, D // heads, out.data_ptr(), lse.data_ptr(),
                   _stream(qkv))
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads = heads
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        K, B, T, D3 = qkv.shape
        dout = dout.contiguous()
        dqkv = torch.empty_like(qkv)
        _capi.call("flr_attention_bwd", qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), K * B, T,
                   ctx.heads, D3 // 3 // ctx.heads, dqkv.data_ptr(), _stream(dout))
        return dqkv, None


def client_attention(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    return ClientAttention.apply(qkv, heads)


def _act_bwd(dy: torch.Tensor, aux: torch.Tensor, mask, act: str) -> torch.Tensor:
    """d(pre) = dy * act'(aux) [* mask] on flr_act_bwd (contiguous operands)."""
    out = torch.empty_like(dy)
    _capi.call("flr_act_bwd", dy.data_ptr(), aux.data_ptr(), _ptr(mask), ACT["d" + act], out.data_ptr(), dy.numel(),
               _stream(dy))
    return out


class ClientLinearAct(torch.autograd.Function):
    """y = act(x W^T + b) per client on flr_bgemm_ex (act in relu / gelu / tanh,
    fused in the GEMM epilogue); the backward's activation derivative is one
    flr_act_bwd pass.  BERT's pooler (tanh) and the CUB attribute MLP use it.
    x [K, M, in] (any strides), W [K, out, in], b [K, out]."""

    @staticmethod
    def forward(ctx, x, W, b, act: str):
        pre = torch.empty(x.shape[0], x.shape[1], W.shape[1], dtype=x.dtype, device=x.device) \
            if act == "gelu" else None
        y = bgemm_ex(x, W, bias=b, act=act, pre=pre)
        ctx.save_for_backward(x, W, pre if act == "gelu" else y)  # relu: y > 0 <=> pre > 0; tanh': 1 - y^2
        ctx.act = act
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W, aux = ctx.saved_tensors
        dpre = _act_bwd(dy.contiguous(), aux, None, ctx.act)
        dx = bgemm(dpre, W.transpose(1, 2)) if ctx.needs_input_grad[0] else None
        dW = bgemm(dpre.transpose(1, 2), x.transpose(1, 2)) if ctx.needs_input_grad[1] else None
        db = sum_rows(dpre) if (ctx.has_b and ctx.needs_input_grad[2]) else None
        return dx, dW, db, None


def client_linear_act(x, W, b, act: str):
    return ClientLinearAct.apply(x, W, b, act)


class ClientMLP(torch.autograd.Function):
    """y = act(x W1^T + b1) [* mask] W2^T + b2 [+ residual] — the encoder MLP
    (GELU) and the late-fusion head (ReLU + dropout mask, cub200_cnn.py:88-93).
    x is one operand [K, M, in] or a tuple of column blocks (the head's
    [img | text] concat, never materialised: fc1 runs as one GEMM per block
    accumulating through the addend).  Fused epilogues: act (+ mask, + the
    saved GELU input) in fc1's, act' (and the mask) in the dy W2 GEMM's."""

    @staticmethod
    def forward(ctx, W1, b1, W2, b2, mask, residual, act: str, *xs):
        K, M = xs[0].shape[:2]
        F = W1.shape[1]
        pre = torch.empty(K, M, F, dtype=W1.dtype, device=W1.device) if act == "gelu" else None
        mask = None if mask is None else mask.contiguous()
        h = None
        c0 = 0
        for i, x in enumerate(xs):
            w = W1[:, :, c0:c0 + x.shape[2]]
            c0 += x.shape[2]
            last = i == len(xs) - 1
            h = bgemm_ex(x, w, bias=b1 if i == 0 else None, add=h, act=act if last else "none",
                         mul=mask if last else None, pre=pre if last else None, out=h)
        y = bgemm(h, W2, bias=b2, add=None if residual is None else residual.contiguous())
        ctx.save_for_backward(W1, W2, h, pre, mask, *xs)
        ctx.act = act
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        W1, W2, h, pre, mask, *xs = ctx.saved_tensors
        dy = dy.contiguous()
        aux = pre if ctx.act == "gelu" else h  # relu: h > 0 <=> kept and pre > 0
        dpre = bgemm_ex(dy, W2.transpose(1, 2), act="d" + ctx.act, aux=aux, mul=mask)
        dW2 = bgemm(dy.transpose(1, 2), h.transpose(1, 2))
        db2 = sum_rows(dy)
        K, F, Din = W1.shape
        dW1 = torch.empty(K, F, Din, dtype=W1.dtype, device=W1.device)
        dxs = []
        c0 = 0
        for i, x in enumerate(xs):
            w = x.shape[2]
            if ctx.needs_input_grad[7 + i]:
                dxs.append(bgemm(dpre, W1[:, :, c0:c0 + w].transpose(1, 2)))
            else:
                dxs.append(None)
            bgemm(dpre.transpose(1, 2), x.transpose(1, 2), out=dW1[:, :, c0:c0 + w])
            c0 += w
        db1 = sum_rows(dpre)
        return (dW1, db1, dW2, db2, None, dy if ctx.has_res else None, None, *dxs)


def client_mlp(x, W1, b1, W2, b2, act: str, mask=None, residual=None):
    """x: a [K, M, in] tensor or a tuple of column blocks (see ClientMLP)."""
    xs = tuple(x) if isinstance(x, (tuple, list)) else (x,)
    return ClientMLP.apply(W1, b1, W2, b2, mask, residual, act, *xs)


class ClientViTTokens(torch.autograd.Function):
    """x0 [K, B, P+1, D]: the class token and the patch projections tok
    [K, B*P, D], plus the position embedding pos [K, P+1, D] (flr_vit_tokens).
    Backward: dpos / dcls = per-client sums over the batch rows (flr_sum_rows),
    dtok = rows 1..P of every sequence (flr_copy_rows)."""

    @staticmethod
    def forward(ctx, tok, cls, pos, B: int):
        K, BP, D = tok.shape
        P = BP // B
        tok, cls, pos = tok.contiguous(), cls.contiguous(), pos.contiguous()
        x0 = torch.empty(K, B, P + 1, D, dtype=tok.dtype, device=tok.device)
        _capi.call("flr_vit_tokens", tok.data_ptr(), cls.data_ptr(), pos.data_ptr(), K, B, P, D, x0.data_ptr(),
                   _stream(tok))
        ctx.dims = (K, B, P, D)
        ctx.cls_shape = cls.shape
        return x0

    @staticmethod
    def backward(ctx, dx0):
        K, B, P, D = ctx.dims
        dx0 = dx0.contiguous()
        T = P + 1
        st = _stream(dx0)
        dpos = torch.empty(K, T, D, dtype=dx0.dtype, device=dx0.device)
        _capi.call("flr_sum_rows", dx0.data_ptr(), B * T * D, T * D, K, B, T * D, dpos.data_ptr(), T * D, st)
        dcls = torch.empty(K, D, dtype=dx0.dtype, device=dx0.device)
        _capi.call("flr_sum_rows", dx0.data_ptr(), B * T * D, T * D, K, B, D, dcls.data_ptr(), D, st)
        dtok = torch.empty(K, B * P, D, dtype=dx0.dtype, device=dx0.device)
        _capi.call("flr_copy_rows", dx0.data_ptr() + 4 * D, T * D, P * D, dtok.data_ptr(), P * D, K * B, st)
        return dtok, dcls.view(ctx.cls_shape), dpos, None


def client_vit_tokens(tok, cls, pos, B: int):
    return ClientViTTokens.apply(tok, cls, pos, B)
