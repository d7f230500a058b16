"""The multimodal client models.

* family "resnet_gru" (BASELINE.json configs C2/C3): ResNet-18 image trunk +
  1-layer GRU text encoder + late-fusion MLP.
* family "cub" (config C1): the reference's own multimodal model,
  CUB200MultimodalCNN (src/models/cub200_cnn.py:57-118) — three conv3x3 / BN /
  ReLU / MaxPool2 blocks, AdaptiveAvgPool(4, 4), image_fc, the attribute MLP
  over a multi-hot ("BoW") text vector, and the same fusion head.

The reference's only multimodal model is CUB200MultimodalCNN
(src/models/cub200_cnn.py:57-118): conv image branch, a second modality
branch, concat late fusion, Linear -> ReLU -> Dropout -> Linear head.  The
BASELINE configs name ResNet-18 for the image and a 1-layer GRU for the text,
which the reference does not contain; this module keeps the reference's
fusion-head structure (cub200_cnn.py:88-93, 109-117) and uses the standard
ResNet-18 (BasicBlock [2,2,2,2], 7x7/2 stem + 3x3/2 max-pool) and torch GRU
definitions for the branches.

Two forms of the same network:
* ``MultimodalNet`` — a plain ``nn.Module`` for ONE client; its
  ``parameters()`` order defines the client-matrix row layout.  The oracle
  trains it with the reference's loop.
* ``batched_forward`` — the engine's client-batched form: every weight is a
  [K, ...] tensor (a view of the client matrix), activations for all K
  clients travel together (convolutions as grouped convolutions, GRU / MLP as
  batched matmuls), so one launch serves every client of a GPU.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass(frozen=True)
class ModelSpec:
    num_classes: int = 10
    image_size: int = 32
    in_channels: int = 3
    widths: Tuple[int, ...] = (64, 128, 256, 512)
    blocks: Tuple[int, ...] = (2, 2, 2, 2)
    vocab: int = 1000
    seq_len: int = 16
    embed: int = 128
    hidden: int = 256
    fusion: int = 256
    dropout: float = 0.5
    family: str = "resnet_gru"  # "resnet_gru" (C2/C3) | "cub" (C1) | "vit_bert" (C4/C5)
    # vit_bert (flr.models.transformer): ViT-S/4 image encoder + BERT-mini text encoder
    patch: int = 4
    vit_dim: int = 384
    vit_depth: int = 12
    vit_heads: int = 6
    vit_mlp: int = 1536
    bert_dim: int = 256
    bert_depth: int = 4
    bert_heads: int = 4
    bert_ffn: int = 1024
    bert_max_pos: int = 512

    @property
    def name(self) -> str:
        if self.family == "cub":
            return "cub200-multimodal-cnn (conv img + attribute MLP) late-fusion"
        if self.family == "vit_bert":
            return (f"vit-s/{self.patch}(d{self.vit_dim}x{self.vit_depth})-img+bert-mini(d{self.bert_dim}x"
                    f"{self.bert_depth})-text late-fusion")
        return "resnet18-img+gru1-text late-fusion"


TINY = ModelSpec(widths=(8, 16, 16, 32), blocks=(1, 1, 1, 1), vocab=50, embed=8, hidden=16, fusion=16,
                 dropout=0.0)

# C1: CUB200MultimodalCNN at 32x32 with C = 10 classes and the BoW text modality
# as its attribute vector (num_attributes = vocab = 312).  widths = the three
# conv blocks; fusion = image_fc / fusion hidden width; embed, hidden = the
# attribute MLP's widths (cub200_cnn.py:71-93).
CUB = ModelSpec(family="cub", num_classes=10, widths=(32, 64, 128), blocks=(), vocab=312, embed=128,
                hidden=256, fusion=256, dropout=0.5)

# C4/C5: ViT-S/4 (384 x 12, 6 heads, MLP 1536) + BERT-mini (256 x 4, 4 heads, FFN
# 1024, WordPiece vocabulary 30522), fusion 640 -> 256 -> 10 (flr.models.transformer)
VIT_BERT = ModelSpec(family="vit_bert", num_classes=10, vocab=30522, seq_len=16, fusion=256, dropout=0.5)
# the same structure at test size (every layer kind, a few hundred thousand parameters)
VIT_BERT_TINY = ModelSpec(family="vit_bert", num_classes=10, vocab=97, seq_len=16, fusion=32, dropout=0.0,
                          patch=8, vit_dim=64, vit_depth=2, vit_heads=1, vit_mlp=128, bert_dim=128, bert_depth=2,
                          bert_heads=2, bert_ffn=256, bert_max_pos=32)


class BasicBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + idt)


class MultimodalNet(nn.Module):
    def __init__(self, spec: ModelSpec = ModelSpec()):
        super().__init__()
        self.spec = spec
        w = spec.widths
        self.conv1 = nn.Conv2d(spec.in_channels, w[0], 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(w[0])
        layers = []
        cin = w[0]
        for i, (cout, n) in enumerate(zip(w, spec.blocks)):
            blocks = []
            for b in range(n):
                blocks.append(BasicBlock(cin, cout, 2 if (b == 0 and i > 0) else 1))
                cin = cout
            layers.append(nn.Sequential(*blocks))
        self.layers = nn.Sequential(*layers)
        self.embedding = nn.Embedding(spec.vocab, spec.embed)
        self.gru = nn.GRU(spec.embed, spec.hidden, num_layers=1, batch_first=True)
        self.fc1 = nn.Linear(w[-1] + spec.hidden, spec.fusion)
        self.dropout = nn.Dropout(spec.dropout)
        self.fc2 = nn.Linear(spec.fusion, spec.num_classes)

    def forward(self, images: torch.Tensor, tokens: torch.Tensor) -> torch.Tensor:
        x = F.relu(self.bn1(self.conv1(images)))
        x = F.max_pool2d(x, 3, 2, 1)
        x = self.layers(x)
        img = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        _, h = self.gru(self.embedding(tokens))
        txt = h[-1]
        z = torch.cat([img, txt], dim=1)
        z = self.dropout(F.relu(self.fc1(z)))
        return self.fc2(z)


class CubMultimodalNet(nn.Module):
    """The C1 model: layer for layer the structure of CUB200MultimodalCNN
    (cub200_cnn.py:67-93), so parameters() has the reference's names, shapes
    and order (the client-matrix row layout).  forward(images, attributes=None):
    without attributes the image features are padded with zeros
    (cub200_cnn.py:110-115)."""

    def __init__(self, spec: ModelSpec = CUB):
        super().__init__()
        self.spec = spec
        c1, c2, c3 = spec.widths

        def block(cin, cout):
            return [nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(), nn.MaxPool2d(2)]
        self.image_conv = nn.Sequential(*block(spec.in_channels, c1), *block(c1, c2), *block(c2, c3),
                                        nn.AdaptiveAvgPool2d((4, 4)))
        self.image_fc = nn.Linear(c3 * 16, spec.fusion)
        self.attr_fc = nn.Sequential(nn.Linear(spec.vocab, spec.embed), nn.ReLU(),
                                     nn.Linear(spec.embed, spec.hidden), nn.ReLU())
        self.fusion = nn.Sequential(nn.Linear(spec.fusion + spec.hidden, spec.fusion), nn.ReLU(),
                                    nn.Dropout(spec.dropout), nn.Linear(spec.fusion, spec.num_classes))

    def forward(self, images: torch.Tensor, attributes: Optional[torch.Tensor] = None) -> torch.Tensor:
        img = F.relu(self.image_fc(self.image_conv(images).flatten(1)))
        if attributes is None:
            att = torch.zeros(img.shape[0], self.spec.hidden, device=img.device, dtype=img.dtype)
        else:
            att = self.attr_fc(attributes)
        return self.fusion(torch.cat([img, att], dim=1))


def model_class(spec: ModelSpec):
    """The nn.Module of one client for this spec's family."""
    if spec.family == "vit_bert":
        from .transformer import ViTBertNet
        return ViTBertNet
    return CubMultimodalNet if spec.family == "cub" else MultimodalNet


def param_layout(spec: ModelSpec) -> List[Tuple[str, torch.Size]]:
    """(name, shape) in parameters() order — the client-matrix row layout."""
    with torch.device("meta"):
        m = model_class(spec)(spec)
    return [(n, p.shape) for n, p in m.named_parameters()]


def num_params(spec: ModelSpec) -> int:
    return sum(int(s.numel()) for _, s in param_layout(spec))


# ---------------------------------------------------------------------------
# client-batched form
# ---------------------------------------------------------------------------

def split_params(X: torch.Tensor, spec: ModelSpec) -> Dict[str, torch.Tensor]:
    """Views [K, *shape] of the client matrix X [K, >=P] per parameter."""
    out, off = {}, 0
    K = X.shape[0]
    for name, shape in param_layout(spec):
        n = int(shape.numel())
        out[name] = X[:, off:off + n].view(K, *shape)
        off += n
    return out


# "native": the flr HIP layer kernels (conv, GRU gates; default on a GPU);
# "torch": torch ops (MIOpen grouped conv etc.) — the CPU path and A/B timing.
_LAYERS = os.environ.get("FLR_LAYERS", "native")


def tap_major_names(spec: ModelSpec) -> frozenset:
    """Conv weights the engine trains in tap-major layout [K, KH, KW, Cin, Cout]
    (flr_conv2d_*_t kernels): Cin and Cout multiples of 64
    (flr_conv2d_tap_major_ok)."""
    return frozenset(n for n, s in param_layout(spec)
                     if len(s) == 4 and s[0] % 64 == 0 and s[1] % 64 == 0)


def conv_geometry(spec: ModelSpec) -> Dict[str, Tuple[int, int, int, int, int]]:
    """name -> (H_in, kernel, stride, pad, H_out) of every conv weight (square maps)."""
    out = {}
    H = spec.image_size
    if spec.family == "vit_bert":  # no convolutions (the patch embedding is a Linear)
        return out
    if spec.family == "cub":
        for idx in (0, 4, 8):
            out[f"image_conv.{idx}.weight"] = (H, 3, 1, 1, H)
            H //= 2
        return out
    Ho = (H + 6 - 7) // 2 + 1
    out["conv1.weight"] = (H, 7, 2, 3, Ho)
    H = (Ho + 2 - 3) // 2 + 1  # 3x3/2 max-pool
    cin = spec.widths[0]
    for li, (cout, nblk) in enumerate(zip(spec.widths, spec.blocks)):
        for bi in range(nblk):
            s = 2 if (bi == 0 and li > 0) else 1
            pre = f"layers.{li}.{bi}."
            H1 = (H + 2 - 3) // s + 1
            out[pre + "conv1.weight"] = (H, 3, s, 1, H1)
            out[pre + "conv2.weight"] = (H1, 3, 1, 1, H1)
            if s != 1 or cin != cout:
                out[pre + "downsample.0.weight"] = (H, 1, s, 0, (H - 1) // s + 1)
            H, cin = H1, cout
    return out


def live_taps(H: int, k: int, stride: int, pad: int) -> List[int]:
    """Tap indices kh*k + kw that read at least one non-padding pixel (square
    map; the rule of conv_common.h make_geom)."""
    Ho = (H + 2 * pad - k) // stride + 1
    rows = [t for t in range(k) if any(0 <= o * stride - pad + t < H for o in range(Ho))]
    return [kh * k + kw for kh in rows for kw in rows]


def to_tap_major(w: torch.Tensor) -> torch.Tensor:
    """[..., Cout, Cin, KH, KW] -> [..., KH, KW, Cin, Cout] (a view)."""
    d = w.dim()
    return w.permute(*range(d - 4), d - 2, d - 1, d - 3, d - 4)


def from_tap_major(w_t: torch.Tensor) -> torch.Tensor:
    """[..., KH, KW, Cin, Cout] -> [..., Cout, Cin, KH, KW] (a view)."""
    d = w_t.dim()
    return w_t.permute(*range(d - 4), d - 1, d - 2, d - 4, d - 3)


def _gconv(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, need_dx: bool = True,
           tap_major: bool = False, zero_dead: bool = True, norm_slot=None) -> torch.Tensor:
    """w [K, Cout, Cin, kh, kw] (or [K, kh, kw, Cin, Cout] when tap_major).
    Native (flr kernels): x [K*Cin, B, H, W] -> [K*Cout, B, H', W'];
    torch: x [B, K*Cin, H, W] -> [B, K*Cout, H', W'] (grouped conv).
    norm_slot (tap-major): an nn.NormSlot, where the weight gradient's
    clip-norm partials go (flr_conv2d_bwd_weight_t_sq)."""
    if tap_major:
        if not x.is_cuda:
            raise RuntimeError("tap-major conv weights need the HIP kernels (no CPU path)")
        from ..nn import client_conv2d_t
        return client_conv2d_t(x, w, stride, pad, need_dx, zero_dead, norm_slot)
    if _LAYERS == "native" and x.is_cuda:
        from ..nn import client_conv2d
        return client_conv2d(x, w, stride, pad, need_dx)
    K, cout = w.shape[0], w.shape[1]
    return F.conv2d(x, w.reshape(K * cout, *w.shape[2:]), stride=stride, padding=pad, groups=K)


def _gbn(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Per-client BatchNorm in train mode (batch statistics); running stats are
    not part of parameters() and never aggregated (run_experiments.py:238,258)."""
    return F.batch_norm(x, None, None, g.reshape(-1), b.reshape(-1), training=True, momentum=0.0, eps=1e-5)


def _gru_torch(gi: torch.Tensor, whh: torch.Tensor, bhh: torch.Tensor) -> torch.Tensor:
    """The GRU recurrence in torch ops (torch's cell: h' = (h - n) * z + n)."""
    K, B, T, H3 = gi.shape
    H = H3 // 3
    whh_t = whh.transpose(1, 2)
    bias = bhh.unsqueeze(1)
    h = torch.zeros(K, B, H, device=gi.device, dtype=gi.dtype)
    for t in range(T):
        gh = torch.baddbmm(bias, h, whh_t)
        i_r, i_z, i_n = gi[:, :, t].chunk(3, dim=-1)
        h_r, h_z, h_n = gh.chunk(3, dim=-1)
        r = torch.sigmoid(i_r + h_r)
        z = torch.sigmoid(i_z + h_z)
        n = torch.tanh(i_n + r * h_n)
        h = (h - n) * z + n
    return h


def _bn_act(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, residual: Optional[torch.Tensor] = None,
            relu: bool = True, stats: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """act(BN(x) [+ residual]) — the block's BN, shortcut add and ReLU, fused
    into one HIP kernel each way on the native path.  stats = (running_mean,
    running_var) [K*C] selects eval mode (model.eval(): running statistics)."""
    if stats is not None:
        if _LAYERS == "native" and x.is_cuda:
            from ..nn import client_batchnorm_infer
            return client_batchnorm_infer(x, g, b, stats[0], stats[1], residual, relu)
        y = F.batch_norm(x, stats[0], stats[1], g.reshape(-1), b.reshape(-1), training=False, eps=1e-5)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y
    if _LAYERS == "native" and x.is_cuda:
        from ..nn import client_batchnorm
        return client_batchnorm(x, g, b, residual, relu)
    y = _gbn(x, g, b)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def _eval_stats(bn_stats, name: str, gamma: torch.Tensor):
    """(running_mean, running_var) [K*C] of BatchNorm `name` in eval mode, or
    None in training mode.  bn_stats: None (training), or a dict name ->
    (mean, var); a BN missing from the dict gets torch's initial buffers (0, 1),
    which is what the reference's global model holds — the simulation copies
    parameters() only and never updates the global buffers
    (run_experiments.py:257-259)."""
    if bn_stats is None:
        return None
    if name in bn_stats:
        m, v = bn_stats[name]
        return m.reshape(-1), v.reshape(-1)
    n = gamma.numel()
    return (torch.zeros(n, device=gamma.device, dtype=gamma.dtype),
            torch.ones(n, device=gamma.device, dtype=gamma.dtype))


def batched_forward(p: Dict[str, torch.Tensor], images: torch.Tensor, tokens: torch.Tensor, spec: ModelSpec,
                    dropout_mask: Optional[torch.Tensor] = None, tap_major: frozenset = frozenset(),
                    skip_dead: frozenset = frozenset(), bn_stats: Optional[Dict] = None,
                    norm_slots: Optional[Dict] = None) -> torch.Tensor:
    """images [K, B, C, H, W], tokens [K, B, T] -> logits [K, B, num_classes].

    dropout_mask: optional [K, B, fusion] tensor of {0, 1/(1-p)} (explicit masks
    make the step reproducible); None applies no dropout.
    tap_major: names of conv weights given as [K, KH, KW, Cin, Cout].
    skip_dead: tap-major weights whose dead-tap gradient slabs are left
    unwritten (the trainer's optimizer step never reads them).
    bn_stats: None (training: batch statistics) or a dict for eval mode (see
    _eval_stats).
    norm_slots: tap-major weight name -> nn.NormSlot: the weight
    gradient's clip-norm partials are written there (the trainer's fused norm).
    """
    if spec.family == "cub":
        return _cub_forward(p, images, tokens, spec, dropout_mask, tap_major, bn_stats, norm_slots)
    if spec.family == "vit_bert":
        from .transformer import patchify, vit_bert_forward
        patches = patchify(images, spec.patch) if images.dim() == 5 else images
        return vit_bert_forward(p, patches, tokens, spec, dropout_mask, native=_LAYERS == "native" and images.is_cuda)

    def st(bn):
        return _eval_stats(bn_stats, bn, p[bn + ".weight"])

    def conv(name, x, stride, pad, need_dx=True):
        return _gconv(x, p[name], stride, pad, need_dx, name in tap_major, name not in skip_dead,
                      None if norm_slots is None else norm_slots.get(name))

    K, B = images.shape[:2]
    native = _LAYERS == "native" and images.is_cuda
    if native:  # the flr kernels' client-channel-major layout [K*C, B, H, W]
        x = images.transpose(1, 2).reshape(K * spec.in_channels, B, *images.shape[3:])
    else:       # torch's grouped-conv layout [B, K*C, H, W]
        x = images.transpose(0, 1).reshape(B, K * spec.in_channels, *images.shape[3:])
    x = _bn_act(conv("conv1.weight", x, 2, 3, need_dx=False), p["bn1.weight"], p["bn1.bias"], stats=st("bn1"))
    if native:
        from ..nn import client_maxpool2d
        x = client_maxpool2d(x, 3, 2, 1)
    else:
        x = F.max_pool2d(x, 3, 2, 1)
    w = spec.widths
    for li, nblk in enumerate(spec.blocks):
        for bi in range(nblk):
            pre = f"layers.{li}.{bi}."
            stride = 2 if (bi == 0 and li > 0) else 1
            idt = x
            if (pre + "downsample.0.weight") in p:
                idt = _bn_act(conv(pre + "downsample.0.weight", x, stride, 0), p[pre + "downsample.1.weight"],
                              p[pre + "downsample.1.bias"], relu=False, stats=st(pre + "downsample.1"))
            y = _bn_act(conv(pre + "conv1.weight", x, stride, 1), p[pre + "bn1.weight"], p[pre + "bn1.bias"],
                        stats=st(pre + "bn1"))
            x = _bn_act(conv(pre + "conv2.weight", y, 1, 1), p[pre + "bn2.weight"], p[pre + "bn2.bias"],
                        residual=idt, stats=st(pre + "bn2"))
    if native:
        # global average pool: at 32x32 input layer4's map is 1x1, where the mean
        # is the value itself (exact) and the pooled features are a free view
        gap = x.view(K, w[-1], B) if x.shape[2] * x.shape[3] == 1 else x.mean(dim=(2, 3)).view(K, w[-1], B)
        img = gap.transpose(1, 2)  # [K, B, 512]
    else:
        img = x.mean(dim=(2, 3)).view(B, K, w[-1]).transpose(0, 1)

    # text: embedding gather + GRU with per-client weights (gate order r, z, n)
    V, E, H = spec.vocab, spec.embed, spec.hidden
    table = p["embedding.weight"]  # [K, V, E]
    T = tokens.shape[2]
    if native:  # flr_embedding_fwd / _bwd (deterministic index_add order)
        from ..nn import client_embedding
        emb = client_embedding(table, tokens.reshape(K, B * T))
    else:
        kofs = (torch.arange(K, device=tokens.device) * V).view(K, 1, 1)
        emb = table.reshape(K * V, E)[(tokens + kofs).reshape(-1)].view(K, B * T, E)
    if native:  # flr_bgemm (MFMA) for every matrix product of the text branch and the head
        from ..nn import client_linear as _lin
    else:
        def _lin(x, W, b):
            return torch.baddbmm(b.unsqueeze(1), x, W.transpose(1, 2))
    gi = _lin(emb, p["gru.weight_ih_l0"], p["gru.bias_ih_l0"])
    gi = gi.view(K, B, T, 3 * H)
    if _LAYERS == "native" and gi.is_cuda:  # flr HIP gate kernels (one launch per step)
        from ..nn import client_gru
        h = client_gru(gi, p["gru.weight_hh_l0"], p["gru.bias_hh_l0"])
    else:
        h = _gru_torch(gi, p["gru.weight_hh_l0"], p["gru.bias_hh_l0"])

    if native:  # fusion head: [img | h] never concatenated; ReLU + dropout mask in the GEMM epilogues
        from ..nn import client_mlp
        return client_mlp((img, h), p["fc1.weight"], p["fc1.bias"], p["fc2.weight"], p["fc2.bias"], "relu",
                          mask=dropout_mask)
    f = torch.cat([img, h], dim=2)  # [K, B, 512 + H]
    f = F.relu(_lin(f, p["fc1.weight"], p["fc1.bias"]))
    if dropout_mask is not None:
        f = f * dropout_mask
    return _lin(f, p["fc2.weight"], p["fc2.bias"])


def _linear_op(native: bool):
    if native:  # flr_bgemm (MFMA)
        from ..nn import client_linear
        return client_linear

    def lin(x, W, b):
        return torch.baddbmm(b.unsqueeze(1), x, W.transpose(1, 2))
    return lin


def _cub_forward(p: Dict[str, torch.Tensor], images: torch.Tensor, attrs: Optional[torch.Tensor], spec: ModelSpec,
                 dropout_mask: Optional[torch.Tensor], tap_major: frozenset,
                 bn_stats: Optional[Dict] = None, norm_slots: Optional[Dict] = None) -> torch.Tensor:
    """The C1 model (cub200_cnn.py:95-118) for K clients at once: three
    conv3x3(+bias) -> BN -> ReLU -> MaxPool2 blocks, AdaptiveAvgPool(4, 4),
    image_fc + ReLU, the attribute MLP, concat, the fusion head.
    images [K, B, C, H, W], attrs [K, B, V] (multi-hot) or None."""
    K, B = images.shape[:2]
    native = _LAYERS == "native" and images.is_cuda
    C0, H, W = images.shape[2:]
    x = (images.transpose(1, 2).reshape(K * C0, B, H, W) if native
         else images.transpose(0, 1).reshape(B, K * C0, H, W))
    for i, idx in enumerate((0, 4, 8)):
        wn = f"image_conv.{idx}.weight"
        y = _gconv(x, p[wn], 1, 1, need_dx=i > 0, tap_major=wn in tap_major,
                   norm_slot=None if norm_slots is None else norm_slots.get(wn))
        bias = p[f"image_conv.{idx}.bias"].reshape(-1)  # [K * Cout]
        y = y + (bias.view(-1, 1, 1, 1) if native else bias.view(1, -1, 1, 1))
        bn = f"image_conv.{idx + 1}"
        y = _bn_act(y, p[bn + ".weight"], p[bn + ".bias"], stats=_eval_stats(bn_stats, bn, p[bn + ".weight"]))
        if native:
            from ..nn import client_maxpool2d
            x = client_maxpool2d(y, 2, 2, 0)
        else:
            x = F.max_pool2d(y, 2)
    if tuple(x.shape[-2:]) != (4, 4):  # at 32x32 input the map is already 4x4 (identity)
        x = F.adaptive_avg_pool2d(x, (4, 4))
    c3 = spec.widths[-1]
    img = x.reshape(K, c3, B, 16).transpose(1, 2) if native else x.reshape(B, K, c3, 16).transpose(0, 1)
    lin = _linear_op(native)
    img = F.relu(lin(img.reshape(K, B, c3 * 16), p["image_fc.weight"], p["image_fc.bias"]))
    if attrs is None:
        a = torch.zeros(K, B, spec.hidden, device=img.device, dtype=img.dtype)
    else:
        a = F.relu(lin(attrs, p["attr_fc.0.weight"], p["attr_fc.0.bias"]))
        a = F.relu(lin(a, p["attr_fc.2.weight"], p["attr_fc.2.bias"]))
    f = F.relu(lin(torch.cat([img, a], dim=2), p["fusion.0.weight"], p["fusion.0.bias"]))
    if dropout_mask is not None:
        f = f * dropout_mask
    return lin(f, p["fusion.3.weight"], p["fusion.3.bias"])
