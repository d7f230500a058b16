"""Autograd wrappers over the client-batched HIP layer kernels."""
from __future__ import annotations

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
    """y[B, K*Cout, Ho, Wo] = conv(x[B, K*Cin, H, W], w[K, Cout, Cin, KH, KW]) per client
    (flr_conv2d_fwd / _bwd_data / _bwd_weight)."""

    @staticmethod
    def forward(ctx, x, w, stride: int, pad: int, need_dx: bool = True):
        x = x.contiguous()
        w = w.contiguous()
        K, Cout, Cin, KH, KW = w.shape
        B, KC, H, W = x.shape
        assert KC == K * Cin, (x.shape, w.shape)
        Ho = (H + 2 * pad - KH) // stride + 1
        Wo = (W + 2 * pad - KW) // stride + 1
        y = torch.empty(B, K * Cout, Ho, Wo, dtype=x.dtype, device=x.device)
        geom = (K, B, Cin, H, W, Cout, KH, KW, stride, pad)
        ws, n = _workspace(geom, x.device)
        _capi.call("flr_conv2d_fwd", x.data_ptr(), w.data_ptr(), y.data_ptr(), *geom,
                   None if ws is None else ws.data_ptr(), n, _stream(x))
        ctx.save_for_backward(x, w)
        ctx.geom = geom
        ctx.need_dx = need_dx
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        g = ctx.geom
        ws, n = _workspace(g, dy.device)
        wsp = None if ws is None else ws.data_ptr()
        dx = None
        if ctx.need_dx and ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _capi.call("flr_conv2d_bwd_data", dy.data_ptr(), w.data_ptr(), dx.data_ptr(), *g, wsp, n, _stream(dy))
        dw = None
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w)
            _capi.call("flr_conv2d_bwd_weight", x.data_ptr(), dy.data_ptr(), dw.data_ptr(), *g, wsp, n,
                       _stream(dy))
        return dx, dw, None, None, None


def client_conv2d(x, w, stride: int, pad: int, need_dx: bool = True):
    return ClientConv2d.apply(x, w, stride, pad, need_dx)
