"""The C4/C5 model family: ViT-S image encoder + BERT-mini text encoder, late fusion.

BASELINE.json configs[3-4] name "ViT-S(img)+BERT-mini(text)".  The reference
has no such model; its only multimodal model,
CUB200MultimodalCNN (src/models/cub200_cnn.py:57-118), fixes the structure this
family keeps: one encoder per modality, concat late fusion, then
Linear -> ReLU -> Dropout -> Linear (cub200_cnn.py:88-93, 109-117).  The
encoders follow the published definitions at the 32x32 / 16-token input sizes
of SURVEY §8:

* ViT-S/4 (timm's vit_small layout): 4x4 patches of the 3x32x32 image -> 64
  patch tokens + a class token, width 384, 12 pre-LN blocks (6 heads of 64,
  MLP 1536, exact-erf GELU), final LayerNorm, the class token's features.
  The patch embedding is a Linear over the flattened (c, kh, kw) patch — the
  same map as Conv2d(3, 384, 4, stride 4) with its weight viewed [384, 48].
* BERT-mini (L=4, H=256, A=4, intermediate 1024): word (30522) + token-type
  (2) + position (512) embeddings, LayerNorm, 4 post-LN blocks, the pooler
  tanh(W h_[CLS] + b) over the first token.

Both use a fused q|k|v in-projection (nn.MultiheadAttention's layout), no
attention mask (the synthetic texts have no padding) and no dropout inside the
encoders; the fusion head's dropout uses explicit masks, as the other
families.  ~32.7M parameters (P is pinned by tests/test_model_geometry.py).

Two forms, as flr.models.multimodal:
* ``ViTBertNet`` — one client's nn.Module; parameters() order is the client
  matrix row layout; the oracle trains it with the reference's loop.
* ``vit_bert_forward`` — every client at once on the flr HIP kernels
  (flr_bgemm[_ex], flr_attention_*, flr_layernorm_*, flr_embedding_*,
  flr_vit_tokens), or on torch ops off the GPU (the CPU check of the layout).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


def patchify(images: torch.Tensor, p: int) -> torch.Tensor:
    """[..., C, H, W] -> [..., (H/p)(W/p), C p p] patch rows in (c, kh, kw) order
    (Conv2d(C, D, p, stride p)'s receptive fields, flattened as its weight)."""
    *lead, C, H, W = images.shape
    x = images.reshape(*lead, C, H // p, p, W // p, p)
    n = len(lead)
    x = x.permute(*range(n), n + 1, n + 3, n, n + 2, n + 4)
    return x.reshape(*lead, (H // p) * (W // p), C * p * p)


class EncoderLayer(nn.Module):
    def __init__(self, dim: int, heads: int, mlp: int, eps: float, pre_ln: bool):
        super().__init__()
        self.heads, self.pre_ln = heads, pre_ln
        self.ln1 = nn.LayerNorm(dim, eps=eps)
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)
        self.ln2 = nn.LayerNorm(dim, eps=eps)
        self.fc1 = nn.Linear(dim, mlp)
        self.fc2 = nn.Linear(mlp, dim)

    def attn(self, x):
        B, T, D = x.shape
        H = self.heads
        q, k, v = self.qkv(x).view(B, T, 3, H, D // H).permute(2, 0, 3, 1, 4)
        a = torch.softmax(torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(D // H), dim=-1)
        return self.proj(torch.matmul(a, v).transpose(1, 2).reshape(B, T, D))

    def mlp(self, x):
        return self.fc2(F.gelu(self.fc1(x)))

    def forward(self, x):
        if self.pre_ln:  # ViT
            x = x + self.attn(self.ln1(x))
            return x + self.mlp(self.ln2(x))
        x = self.ln1(x + self.attn(x))  # BERT (post-LN)
        return self.ln2(x + self.mlp(x))


class ViTEncoder(nn.Module):
    def __init__(self, spec):
        super().__init__()
        D, p = spec.vit_dim, spec.patch
        n = (spec.image_size // p) ** 2
        self.patch = p
        self.cls_token = nn.Parameter(torch.randn(1, 1, D) * 0.02)
        self.pos_embed = nn.Parameter(torch.randn(1, n + 1, D) * 0.02)
        self.patch_embed = nn.Linear(spec.in_channels * p * p, D)
        self.blocks = nn.ModuleList(EncoderLayer(D, spec.vit_heads, spec.vit_mlp, 1e-6, True)
                                    for _ in range(spec.vit_depth))
        self.norm = nn.LayerNorm(D, eps=1e-6)

    def forward(self, images):
        t = self.patch_embed(patchify(images, self.patch))
        x = torch.cat([self.cls_token.expand(t.shape[0], -1, -1), t], dim=1) + self.pos_embed
        for blk in self.blocks:
            x = blk(x)
        return self.norm(x)[:, 0]


class BertEncoder(nn.Module):
    def __init__(self, spec):
        super().__init__()
        D = spec.bert_dim
        self.word_embeddings = nn.Embedding(spec.vocab, D)
        self.position_embeddings = nn.Embedding(spec.bert_max_pos, D)
        self.token_type_embeddings = nn.Embedding(2, D)
        self.emb_ln = nn.LayerNorm(D, eps=1e-12)
        self.layers = nn.ModuleList(EncoderLayer(D, spec.bert_heads, spec.bert_ffn, 1e-12, False)
                                    for _ in range(spec.bert_depth))
        self.pooler = nn.Linear(D, D)

    def forward(self, tokens):
        B, T = tokens.shape
        pos = torch.arange(T, device=tokens.device).unsqueeze(0).expand(B, T)
        e = self.word_embeddings(tokens) + self.token_type_embeddings(torch.zeros_like(tokens))
        e = e + self.position_embeddings(pos)  # HF BertEmbeddings order
        x = self.emb_ln(e)
        for layer in self.layers:
            x = layer(x)
        return torch.tanh(self.pooler(x[:, 0]))


class ViTBertNet(nn.Module):
    """One client: ViT-S image features (384) || BERT-mini pooled text (256) ->
    fusion head (cub200_cnn.py:88-93 structure)."""

    def __init__(self, spec):
        super().__init__()
        self.spec = spec
        self.vit = ViTEncoder(spec)
        self.bert = BertEncoder(spec)
        self.fc1 = nn.Linear(spec.vit_dim + spec.bert_dim, spec.fusion)
        self.dropout = nn.Dropout(spec.dropout)
        self.fc2 = nn.Linear(spec.fusion, spec.num_classes)

    def forward(self, images, tokens):
        z = torch.cat([self.vit(images), self.bert(tokens)], dim=1)
        return self.fc2(self.dropout(F.relu(self.fc1(z))))


# ---------------------------------------------------------------------------
# client-batched form
# ---------------------------------------------------------------------------

class _TorchOps:
    """The same ops on torch (any device): the CPU check of the batched layout."""

    @staticmethod
    def linear(x, W, b):
        return torch.baddbmm(b.unsqueeze(1), x, W.transpose(1, 2))

    @staticmethod
    def linear_act(x, W, b, act):
        y = _TorchOps.linear(x, W, b)
        return {"relu": F.relu, "gelu": F.gelu, "tanh": torch.tanh}[act](y)

    @staticmethod
    def layernorm(x, g, b, eps, residual=None):
        s = x if residual is None else x + residual
        mu = s.mean(dim=-1, keepdim=True)
        var = ((s - mu) ** 2).mean(dim=-1, keepdim=True)
        y = (s - mu) / torch.sqrt(var + eps) * g.unsqueeze(1) + b.unsqueeze(1)
        return y if residual is None else (y, s)

    @staticmethod
    def attention(qkv, heads):
        K, B, T, D3 = qkv.shape
        D = D3 // 3
        q, k, v = qkv.view(K, B, T, 3, heads, D // heads).permute(3, 0, 1, 4, 2, 5)
        a = torch.softmax(torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(D // heads), dim=-1)
        return torch.matmul(a, v).transpose(2, 3).reshape(K, B, T, D)

    @staticmethod
    def mlp(x, W1, b1, W2, b2, act, mask=None, residual=None):
        xs = x if isinstance(x, (tuple, list)) else (x,)
        h = _TorchOps.linear_act(torch.cat(xs, dim=2), W1, b1, act)
        if mask is not None:
            h = h * mask
        y = _TorchOps.linear(h, W2, b2)
        return y if residual is None else y + residual

    @staticmethod
    def vit_tokens(tok, cls, pos, B):
        K, BP, D = tok.shape
        t = tok.view(K, B, BP // B, D)
        return torch.cat([cls.view(K, 1, 1, D).expand(K, B, 1, D), t], dim=2) + pos.view(K, 1, -1, D)

    @staticmethod
    def embed_sum(word, typ, pos, ids, type_ids, pos_ids):
        K, V, E = word.shape
        kk = torch.arange(K, device=ids.device).view(K, 1)
        e = word[kk, ids] + typ[:, type_ids]
        return e + pos[:, pos_ids]


class _NativeOps:
    """The flr HIP kernels (flr.nn autograd wrappers)."""

    def __init__(self):
        from .. import nn as fnn
        self.f = fnn

    def linear(self, x, W, b):
        return self.f.client_linear(x, W, b)

    def linear_act(self, x, W, b, act):
        return self.f.client_linear_act(x, W, b, act)

    def layernorm(self, x, g, b, eps, residual=None):
        return self.f.client_layernorm(x, g, b, residual=residual, eps=eps)

    def attention(self, qkv, heads):
        return self.f.client_attention(qkv, heads)

    def mlp(self, x, W1, b1, W2, b2, act, mask=None, residual=None):
        return self.f.client_mlp(x, W1, b1, W2, b2, act, mask=mask, residual=residual)

    def vit_tokens(self, tok, cls, pos, B):
        return self.f.client_vit_tokens(tok, cls, pos, B)

    def embed_sum(self, word, typ, pos, ids, type_ids, pos_ids):
        return self.f.client_embedding_sum(word, typ, pos, ids, type_ids, pos_ids)


def _encoder_pre_ln(ops, p, pre, x, L, heads, eps, K, B, T, D):
    """ViT blocks; x [K, B*T, D] -> the final LayerNorm's output rows."""
    s = x
    r = None  # pending residual branch (added inside the next LayerNorm)
    for i in range(L):
        q = f"{pre}blocks.{i}."
        if r is None:
            h = ops.layernorm(s, p[q + "ln1.weight"], p[q + "ln1.bias"], eps)
        else:
            h, s = ops.layernorm(s, p[q + "ln1.weight"], p[q + "ln1.bias"], eps, residual=r)
        qkv = ops.linear(h, p[q + "qkv.weight"], p[q + "qkv.bias"])
        ctx = ops.attention(qkv.view(K, B, T, 3 * D), heads).view(K, B * T, D)
        a = ops.linear(ctx, p[q + "proj.weight"], p[q + "proj.bias"])
        h2, s = ops.layernorm(s, p[q + "ln2.weight"], p[q + "ln2.bias"], eps, residual=a)
        r = ops.mlp(h2, p[q + "fc1.weight"], p[q + "fc1.bias"], p[q + "fc2.weight"], p[q + "fc2.bias"], "gelu")
    y, _ = ops.layernorm(s, p[pre + "norm.weight"], p[pre + "norm.bias"], eps, residual=r)
    return y


def _encoder_post_ln(ops, p, pre, x, L, heads, eps, K, B, T, D):
    """BERT layers; x [K, B*T, D] (after the embedding LayerNorm)."""
    for i in range(L):
        q = f"{pre}layers.{i}."
        qkv = ops.linear(x, p[q + "qkv.weight"], p[q + "qkv.bias"])
        ctx = ops.attention(qkv.view(K, B, T, 3 * D), heads).view(K, B * T, D)
        a = ops.linear(ctx, p[q + "proj.weight"], p[q + "proj.bias"])
        x, _ = ops.layernorm(x, p[q + "ln1.weight"], p[q + "ln1.bias"], eps, residual=a)
        f = ops.mlp(x, p[q + "fc1.weight"], p[q + "fc1.bias"], p[q + "fc2.weight"], p[q + "fc2.bias"], "gelu")
        x, _ = ops.layernorm(x, p[q + "ln2.weight"], p[q + "ln2.bias"], eps, residual=f)
    return x


def vit_bert_forward(p: Dict[str, torch.Tensor], patches: torch.Tensor, tokens: torch.Tensor, spec,
                     dropout_mask: Optional[torch.Tensor] = None, native: bool = True) -> torch.Tensor:
    """patches [K, B, n_patches, C p p] (flr.models.transformer.patchify of the
    images), tokens [K, B, T] int64 -> logits [K, B, num_classes]."""
    ops = _NativeOps() if native else _TorchOps()
    K, B, NP, _ = patches.shape
    Dv, Db = spec.vit_dim, spec.bert_dim
    Tv = NP + 1
    tok = ops.linear(patches.reshape(K, B * NP, -1), p["vit.patch_embed.weight"], p["vit.patch_embed.bias"])
    x0 = ops.vit_tokens(tok, p["vit.cls_token"], p["vit.pos_embed"].reshape(K, Tv, Dv), B)
    y = _encoder_pre_ln(ops, p, "vit.", x0.reshape(K, B * Tv, Dv), spec.vit_depth, spec.vit_heads, 1e-6,
                        K, B, Tv, Dv)
    img = y.view(K, B, Tv, Dv)[:, :, 0]                      # class-token features [K, B, 384]

    T = tokens.shape[2]
    ids = tokens.reshape(K, B * T)
    type_ids = torch.zeros(B * T, dtype=torch.int64, device=tokens.device)
    pos_ids = torch.arange(T, device=tokens.device).repeat(B)
    e = ops.embed_sum(p["bert.word_embeddings.weight"], p["bert.token_type_embeddings.weight"],
                      p["bert.position_embeddings.weight"], ids, type_ids, pos_ids)
    x = ops.layernorm(e, p["bert.emb_ln.weight"], p["bert.emb_ln.bias"], 1e-12)
    x = _encoder_post_ln(ops, p, "bert.", x, spec.bert_depth, spec.bert_heads, 1e-12, K, B, T, Db)
    txt = ops.linear_act(x.view(K, B, T, Db)[:, :, 0], p["bert.pooler.weight"], p["bert.pooler.bias"], "tanh")

    return ops.mlp((img, txt), p["fc1.weight"], p["fc1.bias"], p["fc2.weight"], p["fc2.bias"], "relu",
                   mask=dropout_mask)
