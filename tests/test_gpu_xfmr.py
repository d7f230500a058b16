"""GPU numerics of the encoder kernels (csrc/train_xfmr.hip, flr_bgemm_ex)
against torch on the CPU: embedding forward / backward bit-exact (torch's
index_add order), LayerNorm / attention / the fused GEMM epilogues within
fp32 tolerances of an fp64 reference."""
import math

import pytest
import torch
import torch.nn.functional as F

from flr import nn as fnn

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("K,V,E,N", [(3, 50, 8, 64), (2, 1000, 128, 512), (2, 30522, 256, 512), (1, 7, 12, 5)])
def test_embedding_fwd_bwd_bitexact(cuda, K, V, E, N):
    g = torch.Generator().manual_seed(V)
    table = torch.randn(K, V, E, generator=g)
    ids = torch.randint(0, V, (K, N), generator=g)
    ids[:, : N // 4] = ids[:, :1]  # repeated ids: multi-row runs in the scatter
    dout = torch.randn(K, N, E, generator=g)
    t = table.to(cuda).requires_grad_(True)
    out = fnn.client_embedding(t, ids.to(cuda))
    (dt,) = torch.autograd.grad(out, t, dout.to(cuda))
    for k in range(K):
        tk = table[k].clone().requires_grad_(True)
        ref = F.embedding(ids[k], tk)
        assert torch.equal(out[k].cpu(), ref)
        (dref,) = torch.autograd.grad(ref, tk, dout[k])
        assert torch.equal(dt[k].cpu(), dref)


def test_embedding_sum_bert_order(cuda):
    K, V, E, B, T = 2, 300, 64, 4, 16
    g = torch.Generator().manual_seed(3)
    word, typ, pos = (torch.randn(K, n, E, generator=g) for n in (V, 2, 32))
    ids = torch.randint(0, V, (K, B * T), generator=g)
    type_ids = torch.zeros(B * T, dtype=torch.int64)
    pos_ids = torch.arange(T).repeat(B)
    dout = torch.randn(K, B * T, E, generator=g)
    leaves = [x.to(cuda).requires_grad_(True) for x in (word, typ, pos)]
    out = fnn.client_embedding_sum(*leaves, ids.to(cuda), type_ids.to(cuda), pos_ids.to(cuda))
    grads = torch.autograd.grad(out, leaves, dout.to(cuda))
    for k in range(K):
        lk = [x[k].clone().requires_grad_(True) for x in (word, typ, pos)]
        ref = (F.embedding(ids[k], lk[0]) + F.embedding(type_ids, lk[1])) + F.embedding(pos_ids, lk[2])
        assert torch.equal(out[k].cpu(), ref)
        rg = torch.autograd.grad(ref, lk, dout[k])
        for a, b in zip(grads, rg):
            assert torch.equal(a[k].cpu(), b)


@pytest.mark.parametrize("R,D,res", [(65 * 4, 384, True), (16 * 3, 256, False), (130, 64, True), (7, 1024, True)])
def test_layernorm_fwd_bwd(cuda, R, D, res):
    K = 3
    g = torch.Generator().manual_seed(R + D)
    x = torch.randn(K, R, D, generator=g) * 2 + 0.5
    r = torch.randn(K, R, D, generator=g) if res else None
    gam = 1 + 0.1 * torch.randn(K, D, generator=g)
    bet = 0.1 * torch.randn(K, D, generator=g)
    dy = torch.randn(K, R, D, generator=g)
    ds = torch.randn(K, R, D, generator=g) if res else None
    eps = 1e-6
    dev = [t.to(cuda).requires_grad_(True) if t is not None else None for t in (x, r, gam, bet)]
    out = fnn.client_layernorm(dev[0], dev[2], dev[3], residual=dev[1], eps=eps)
    leaves = [t for t in dev if t is not None]
    if res:
        y, s = out
        grads = torch.autograd.grad([y, s], leaves, [dy.to(cuda), ds.to(cuda)])
    else:
        y = out
        grads = torch.autograd.grad(y, leaves, dy.to(cuda))
    ref_leaves = [t.double().requires_grad_(True) for t in (x, r, gam, bet) if t is not None]
    xs = ref_leaves[0] + ref_leaves[1] if res else ref_leaves[0]
    gg, bb = ref_leaves[-2], ref_leaves[-1]
    yr = torch.stack([F.layer_norm(xs[k], (D,), gg[k], bb[k], eps) for k in range(K)])
    outs, gos = ([yr, xs], [dy.double(), ds.double()]) if res else ([yr], [dy.double()])
    rgrads = torch.autograd.grad(outs, ref_leaves, gos)
    assert _rel(y, yr) < 2e-6
    for a, b in zip(grads, rgrads):
        assert _rel(a, b) < 1e-5, _rel(a, b)


@pytest.mark.parametrize("T,H", [(65, 6), (16, 4), (17, 1), (96, 2), (5, 3)])
def test_attention_fwd_bwd(cuda, T, H):
    K, B, dh = 2, 3, 64
    D = H * dh
    g = torch.Generator().manual_seed(T * H)
    qkv = torch.randn(K, B, T, 3 * D, generator=g)
    dctx = torch.randn(K, B, T, D, generator=g)
    q_ = qkv.to(cuda).requires_grad_(True)
    ctx = fnn.client_attention(q_, H)
    (dq,) = torch.autograd.grad(ctx, q_, dctx.to(cuda))
    qd = qkv.double().requires_grad_(True)
    q, k, v = qd.view(K, B, T, 3, H, dh).permute(3, 0, 1, 4, 2, 5)
    a = torch.softmax(q @ k.transpose(-2, -1) / math.sqrt(dh), dim=-1)
    ref = (a @ v).transpose(2, 3).reshape(K, B, T, D)
    (dref,) = torch.autograd.grad(ref, qd, dctx.double())
    assert _rel(ctx, ref) < 2e-6, _rel(ctx, ref)
    assert _rel(dq, dref) < 1e-5, _rel(dq, dref)


@pytest.mark.parametrize("T", [65, 96])
def test_attention_thread_forms_bit_identical(cuda, T, knob):
    """The 256- and 512-thread attention forms (FLR_ATT_THREADS) compute every
    score and output in the same order: bit-identical outputs and gradients."""
    K, B, H, dh = 2, 3, 2, 64
    g = torch.Generator().manual_seed(T)
    qkv = torch.randn(K, B, T, 3 * H * dh, generator=g).to(cuda)
    dctx = torch.randn(K, B, T, H * dh, generator=g).to(cuda)
    outs = []
    for thr in ("256", "512"):
        knob("FLR_ATT_THREADS", thr)
        q_ = qkv.clone().requires_grad_(True)
        ctx = fnn.client_attention(q_, H)
        (dq,) = torch.autograd.grad(ctx, q_, dctx)
        outs.append((ctx.detach(), dq))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("act", ["relu", "gelu", "tanh"])
def test_bgemm_ex_epilogues(cuda, act):
    K, M, N, R = 3, 70, 96, 130
    g = torch.Generator().manual_seed(11)
    A, W = torch.randn(K, M, R, generator=g), torch.randn(K, N, R, generator=g) * 0.1
    b, add = torch.randn(K, N, generator=g), torch.randn(K, M, N, generator=g)
    mask = (torch.rand(K, M, N, generator=g) > 0.5).float() * 2.0
    pre = torch.empty(K, M, N, device=cuda)
    y = fnn.bgemm_ex(A.to(cuda), W.to(cuda), bias=b.to(cuda), add=add.to(cuda), act=act, mul=mask.to(cuda), pre=pre)
    pref = (A.double() @ W.double().transpose(1, 2) + b.double().unsqueeze(1)) + add.double()
    fn = {"relu": F.relu, "gelu": F.gelu, "tanh": torch.tanh}[act]
    assert _rel(pre, pref) < 2e-6
    assert _rel(y, fn(pref) * mask.double()) < 2e-6
    # backward modes: dpre = (dY W2) * act'(aux) * mask
    dY, W2 = torch.randn(K, M, 40, generator=g), torch.randn(K, 40, N, generator=g) * 0.1
    aux = pref.float() if act == "gelu" else fn(pref).float()
    d = fnn.bgemm_ex(dY.to(cuda), W2.to(cuda).transpose(1, 2), act="d" + act, aux=aux.to(cuda), mul=mask.to(cuda))
    pr = pref.clone().requires_grad_(True)
    (dref,) = torch.autograd.grad(fn(pr), pr, dY.double() @ W2.double())
    assert _rel(d, dref * mask.double()) < 2e-6
    # the same derivative as a standalone pass (flr_act_bwd)
    e = fnn._act_bwd((dY @ W2).to(cuda), aux.to(cuda), mask.to(cuda), act)
    assert _rel(e, dref * mask.double()) < 2e-6


def test_client_mlp_split_input_and_mask(cuda):
    """The late-fusion head: [a | b] -> fc1 -> ReLU -> mask -> fc2, concat never built."""
    K, M, Da, Db, Fh, C = 2, 32, 96, 64, 48, 10
    g = torch.Generator().manual_seed(5)
    a, b = torch.randn(K, M, Da, generator=g), torch.randn(K, M, Db, generator=g)
    W1, b1 = torch.randn(K, Fh, Da + Db, generator=g) * 0.1, torch.randn(K, Fh, generator=g)
    W2, b2 = torch.randn(K, C, Fh, generator=g) * 0.1, torch.randn(K, C, generator=g)
    mask = (torch.rand(K, M, Fh, generator=g) > 0.5).float() * 2.0
    dy = torch.randn(K, M, C, generator=g)
    leaves = [t.to(cuda).requires_grad_(True) for t in (a, b, W1, b1, W2, b2)]
    y = fnn.client_mlp((leaves[0], leaves[1]), *leaves[2:], "relu", mask=mask.to(cuda))
    grads = torch.autograd.grad(y, leaves, dy.to(cuda))
    rl = [t.double().requires_grad_(True) for t in (a, b, W1, b1, W2, b2)]
    h = F.relu(torch.cat(rl[:2], 2) @ rl[2].transpose(1, 2) + rl[3].unsqueeze(1)) * mask.double()
    yr = h @ rl[4].transpose(1, 2) + rl[5].unsqueeze(1)
    rg = torch.autograd.grad(yr, rl, dy.double())
    assert _rel(y, yr) < 2e-6
    for x, r in zip(grads, rg):
        assert _rel(x, r) < 1e-5


def test_vit_tokens_fwd_bwd(cuda):
    K, B, P, D = 2, 3, 16, 64
    g = torch.Generator().manual_seed(2)
    tok, cls, pos = torch.randn(K, B * P, D, generator=g), torch.randn(K, 1, 1, D, generator=g), \
        torch.randn(K, P + 1, D, generator=g)
    dx = torch.randn(K, B, P + 1, D, generator=g)
    leaves = [t.to(cuda).requires_grad_(True) for t in (tok, cls, pos)]
    x0 = fnn.client_vit_tokens(*leaves, B)
    grads = torch.autograd.grad(x0, leaves, dx.to(cuda))
    rl = [t.clone().requires_grad_(True) for t in (tok, cls, pos)]
    ref = torch.cat([rl[1].view(K, 1, 1, D).expand(K, B, 1, D), rl[0].view(K, B, P, D)], 2) + rl[2].view(K, 1, P + 1, D)
    assert torch.equal(x0.cpu(), ref)
    rg = torch.autograd.grad(ref, rl, dx)
    for x, r in zip(grads, rg):
        assert _rel(x, r) < 1e-6
