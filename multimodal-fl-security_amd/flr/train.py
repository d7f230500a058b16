"""Client-batched local training: every client of a GPU steps together.

Reference semantics (experiments/run_experiments.py:193-240, the fp32 branch
:230-235; contract FLClient.fit / _train, src/client/fl_client.py:76-149):
each client starts from the global model (:203), builds a fresh
SGD(lr, momentum=0.9, wd) (:206-211), and for every batch runs forward, mean
cross-entropy, backward, clip_grad_norm_(1.0) and optimizer.step(); its update
is the parameter list afterwards (:238) and its reported loss the mean of the
per-batch losses (fl_client.py:143-149).

Engine: the K_local clients' parameters are the rows of one client matrix X
([K, P] fp32 in HBM, `model.parameters()` order).  The forward/backward runs
for all rows at once (flr.models.multimodal.batched_forward: grouped
convolutions / batched matmuls); the loss is the HIP cross-entropy kernel; the
training state is parameter-major (one contiguous [K, *shape] block per
parameter), autograd's gradient blocks feed ONE fused HIP kernel that applies
the per-client clip and the SGD-momentum update in place, and the trained
blocks are written once per round into the client-major matrix X the server
aggregates.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import torch

from . import _capi
from .matrix import ClientMatrix
from .models import multimodal as _mm
from .models.multimodal import (ModelSpec, batched_forward, conv_geometry, from_tap_major, live_taps, param_layout,
                                tap_major_names, to_tap_major)


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class CrossEntropy(torch.autograd.Function):
    """Per-client mean cross-entropy on the flr_cross_entropy HIP kernel.
    logits [K, B, C] fp32, labels [K, B] int64 -> loss [K]."""

    @staticmethod
    def forward(ctx, logits, labels):
        K, B, C = logits.shape
        z = logits.contiguous()
        y = labels.contiguous()
        loss = torch.empty(K, dtype=torch.float32, device=z.device)
        dz = torch.empty_like(z)
        rows = torch.empty(K * B, dtype=torch.float32, device=z.device)
        _capi.call("flr_cross_entropy", z.data_ptr(), y.data_ptr(), K, B, C, loss.data_ptr(), dz.data_ptr(),
                   rows.data_ptr(), _stream(z))
        ctx.save_for_backward(dz)
        return loss

    @staticmethod
    def backward(ctx, gk):
        (dz,) = ctx.saved_tensors
        K, B, C = dz.shape
        d = dz.clone()
        gk = gk.contiguous().float()
        _capi.call("flr_scale_client_rows", d.data_ptr(), gk.data_ptr(), K, B, C, _stream(d))
        return d, None


@dataclass
class TrainConfig:
    lr: float = 0.01             # run_experiments.py:41
    momentum: float = 0.9        # :209
    weight_decay: float = 0.0    # :210 (1e-4 only for cub200)
    clip: float = 1.0            # :227, :234
    local_steps: int = 5
    # clients per forward/backward pass (0: automatic).  Activations scale with
    # it, parameters and optimizer state do not; every kernel's per-client
    # result is independent of it (split-K is chosen per client).
    client_chunk: int = 0


class ClientBatchTrainer:
    """Trains K clients of one GPU together.

    Training state is PARAMETER-MAJOR: parameter j of all K clients is one
    contiguous [K, *shape_j] block (W, and momentum Mb alike), so grouped
    convolutions see their weights as free [K*Cout, Cin, kh, kw] views and
    autograd's per-parameter gradients feed the fused clip+SGD kernel with no
    copy.  After the local steps, `export()` writes the client-major client
    matrix X (row k = client k's parameters() vector) once per round for the
    aggregation kernels.
    """

    def __init__(self, spec: ModelSpec, num_clients: int, device, cfg: TrainConfig = TrainConfig(),
                 matrix: Optional[ClientMatrix] = None):
        self.spec = spec
        self.cfg = cfg
        self.device = torch.device(device)
        layout = param_layout(spec)
        self.names = [n for n, _ in layout]
        self.shapes = [s for _, s in layout]
        # conv weights kept tap-major [K, KH, KW, Cin, Cout] during the round
        # (flr_conv2d_*_t); converted at load_global / export only
        native = self.device.type == "cuda" and _mm._LAYERS == "native"
        self.tap_major = tap_major_names(spec) if native else frozenset()
        self.train_shapes = [torch.Size((s[2], s[3], s[1], s[0])) if n in self.tap_major else s
                             for n, s in zip(self.names, self.shapes)]
        self.X = matrix if matrix is not None else ClientMatrix.empty(num_clients, self.shapes, self.device)
        self.K = self.X.K
        self.P = self.X.P
        self.numels = list(self.X.numels)
        self.offsets = list(self.X.offsets)
        # one buffer per state, each block 256-B aligned
        self._boffs, tot = [], 0
        for n in self.numels:
            self._boffs.append(tot)
            tot += (self.K * n + 63) // 64 * 64
        self._wbuf = torch.zeros(tot, dtype=torch.float32, device=self.device)
        self._mbuf = torch.zeros(tot, dtype=torch.float32, device=self.device)
        self.W = [self._wbuf[o:o + self.K * n].view(self.K, *s)
                  for o, n, s in zip(self._boffs, self.numels, self.train_shapes)]
        self.Mb = [self._mbuf[o:o + self.K * n].view(self.K, *s)
                   for o, n, s in zip(self._boffs, self.numels, self.train_shapes)]
        nbytes = int(_capi.lib().flr_clip_sgd_workspace(self.K))
        self._ws = torch.empty(nbytes + 256, dtype=torch.uint8, device=self.device)
        self._ws_off = (-self._ws.data_ptr()) % 256
        self._ws_bytes = nbytes
        self.norms = torch.zeros(self.K, dtype=torch.float32, device=self.device)
        # optimizer blocks: (param j, element offset, numel, client stride).  A
        # tap-major conv weight with dead taps (taps that only read zero padding
        # at this input size) contributes only its live-tap runs: with
        # weight_decay == 0 a dead tap's gradient is exactly 0 at every step,
        # so its weights and momentum never change and the step skips them.
        self.skip_dead = frozenset()
        blocks = []
        self.dead_ranges = []  # (row offset, numel): the dead-tap slabs, in training order
        geo = conv_geometry(spec)
        for j, (name, n, shp) in enumerate(zip(self.names, self.numels, self.shapes)):
            live = None
            if name in self.tap_major and cfg.weight_decay == 0.0:
                H, k, st, pd, _ = geo[name]
                live = live_taps(H, k, st, pd)
                if len(live) == k * k:
                    live = None
            if live is None:
                blocks.append((j, 0, n, n))
                continue
            self.skip_dead = self.skip_dead | {name}
            slab = shp[0] * shp[1]
            runs, t0 = [], live[0]
            for a, b in zip(live, live[1:] + [None]):
                if b != a + 1:
                    runs.append((t0, a + 1))
                    t0 = b
            for lo, hi in runs:
                blocks.append((j, lo * slab, (hi - lo) * slab, n))
            covered = [(lo * slab, hi * slab) for lo, hi in runs]
            e = 0
            for a, b in covered + [(n, n)]:
                if a > e:
                    self.dead_ranges.append((self.offsets[j] + e, a - e))
                e = b
        self.blocks = blocks
        self.live_params = sum(c for _, _, c, _ in blocks)
        nb = len(blocks)
        self._np = (ctypes.c_int64 * nb)(*[c for _, _, c, _ in blocks])
        self._cs = (ctypes.c_int64 * nb)(*[cs for _, _, _, cs in blocks])
        # the last step's output offsets in a training-order client-matrix row
        self._xo = (ctypes.c_int64 * nb)(*[self.offsets[j] + o for j, o, _, _ in blocks])
        chunk = cfg.client_chunk if cfg.client_chunk > 0 else self.auto_chunk(spec, self.K)
        self.chunks = [(c0, min(self.K, c0 + chunk)) for c0 in range(0, self.K, chunk)]
        # fused clip norm: the tap-major conv weights' gradient sums of squares come
        # from the weight-gradient epilogues (flr_conv2d_bwd_weight_t_sq), so the
        # optimizer's own norm pass reads only the other blocks (FLR_FUSED_NORM=0: off)
        self._norm_fused = frozenset(self.tap_major) if (
            cfg.clip > 0 and os.environ.get("FLR_FUSED_NORM", "1") != "0") else frozenset()
        self._normed = (ctypes.c_uint8 * nb)(*[int(self.names[j] in self._norm_fused) for j, _, _, _ in blocks])
        self._sq = None        # [K, sq_ld] fp64 partials, sized at the first step (the slots depend on B)
        self._sq_B = None
        self._sq_slots: Dict[str, tuple] = {}
        # per chunk: the optimizer's block pointers at the chunk's first client
        self._xp, self._mp = [], []
        for c0, _ in self.chunks:
            self._xp.append((ctypes.c_void_p * nb)(*[self.W[j].data_ptr() + 4 * (o + c0 * cs)
                                                     for j, o, _, cs in blocks]))
            self._mp.append((ctypes.c_void_p * nb)(*[self.Mb[j].data_ptr() + 4 * (o + c0 * cs)
                                                     for j, o, _, cs in blocks]))

    @staticmethod
    def auto_chunk(spec: ModelSpec, K: int) -> int:
        """Clients per pass: the encoder family holds ~0.6 GB of activations per
        client at batch 32 (ViT-S over 65 tokens x 12 blocks), so 32 clients per
        pass; the convolutional families fit every client of a GPU at once."""
        return min(K, 32) if spec.family == "vit_bert" else K

    def load_global(self, global_flat: torch.Tensor) -> None:
        """Every client starts from the global model (run_experiments.py:203)."""
        g = global_flat.to(self.device, torch.float32)
        st = _stream(self._wbuf)
        for name, w, off, n, shp in zip(self.names, self.W, self.offsets, self.numels, self.shapes):
            src = g[off:off + n]
            if name in self.tap_major:  # one client's worth, permuted once
                src = to_tap_major(src.view(shp)).contiguous()
            else:
                src = src.contiguous()
            _capi.call("flr_broadcast_rows", src.data_ptr(), n, w.data_ptr(), self.K, n, st)

    # ---- training order: the coordinate order of the training blocks ---------
    # Row k of a training-order client matrix holds client k's blocks at the
    # torch offsets, each block in its training layout (tap-major conv weights
    # [KH, KW, Cin, Cout] instead of torch's [Cout, Cin, KH, KW]).  The hot-path
    # aggregators are indifferent to a common coordinate permutation
    # (BaseDefense.order_free), so the round engine aggregates in this order:
    # the last optimizer step writes X directly (no export pass) and only the
    # aggregated P-vector is permuted back.
    def to_train_order(self, flat: torch.Tensor) -> torch.Tensor:
        """A torch-order parameter vector -> training order (a new tensor)."""
        parts = []
        for name, off, n, shp in zip(self.names, self.offsets, self.numels, self.shapes):
            src = flat[off:off + n]
            parts.append(to_tap_major(src.view(shp)).reshape(-1) if name in self.tap_major else src)
        return torch.cat(parts) if parts else flat.clone()

    def to_torch_order(self, flat: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """A training-order parameter vector -> torch order (into out if given)."""
        if out is None:
            out = torch.empty_like(flat)
        for name, off, n, shp, tshp in zip(self.names, self.offsets, self.numels, self.shapes, self.train_shapes):
            src = flat[off:off + n]
            if name in self.tap_major:
                out[off:off + n].view(shp).copy_(from_tap_major(src.view(tshp)))
            else:
                out[off:off + n].copy_(src)
        return out

    def load_global_train(self, gtrain: torch.Tensor, live_only: bool = True) -> None:
        """load_global from a training-order global vector: a plain broadcast per
        block.  live_only skips the dead-tap slabs: no training kernel reads
        them and the round's client matrix takes them from gtrain directly
        (local_update's out=), so export() is invalid until the next full load."""
        st = _stream(self._wbuf)
        for name, w, off, n in zip(self.names, self.W, self.offsets, self.numels):
            if live_only and name in self.skip_dead:
                continue
            _capi.call("flr_broadcast_rows", gtrain.data_ptr() + 4 * off, n, w.data_ptr(), self.K, n, st)
        if live_only:
            for j, o, c, cs in self.blocks:
                if self.names[j] in self.skip_dead:
                    _capi.call("flr_broadcast_rows", gtrain.data_ptr() + 4 * (self.offsets[j] + o), c,
                               self.W[j].data_ptr() + 4 * o, self.K, cs, st)
        self._dead_stale = live_only and bool(self.skip_dead)

    def export(self, negate_rows: int = 0) -> ClientMatrix:
        """Client-major client matrix for the server (row k = client k); rows
        k < negate_rows are written negated (the sign-flip attackers)."""
        if getattr(self, "_dead_stale", False):
            raise RuntimeError("export() after load_global_train(live_only=True): the dead-tap slabs are not loaded")
        st = _stream(self._wbuf)
        ld = self.X.data.stride(0)
        base = self.X.data.data_ptr()
        for name, w, off, n, shp in zip(self.names, self.W, self.offsets, self.numels, self.shapes):
            if name in self.tap_major:
                cout, cin, kh, kw = shp
                _capi.call("flr_tap_major_to_torch_neg", w.data_ptr(), self.K, kh * kw, cin, cout, base + 4 * off, ld,
                           negate_rows, st)
            else:
                _capi.call("flr_copy_rows_neg", w.data_ptr(), n, n, base + 4 * off, ld, self.K, negate_rows, st)
        return self.X

    def _norm_slots(self, B: int, c0: int, c1: int) -> Optional[Dict[str, tuple]]:
        """name -> (sq pointer, row stride) of every fused-norm conv weight for
        the chunk [c0, c1); allocates the partial buffer for batch size B."""
        if not self._norm_fused:
            return None
        if self._sq_B != B:
            geo = conv_geometry(self.spec)
            lib = _capi.lib()
            bases, tot = {}, 0
            for j, name in enumerate(self.names):
                if name not in self._norm_fused:
                    continue
                cout, cin, kh, kw = self.shapes[j]
                H, k, st, pd, _ = geo[name]
                n = int(lib.flr_conv2d_bwd_weight_t_sq_slots(c1 - c0, B, cin, H, H, cout, kh, kw, st, pd))
                if n < 0:
                    raise RuntimeError(f"no fused-norm slots for {name}")
                bases[name] = tot
                tot += n
            self._sq = torch.zeros(self.K, max(1, tot), dtype=torch.float64, device=self.device)
            self._sq_bases, self._sq_B = bases, B
        from .nn import NormSlot
        ld = self._sq.shape[1]
        return {name: NormSlot(self._sq.data_ptr() + 8 * (c0 * ld + b), ld) for name, b in self._sq_bases.items()}

    # ---- one optimizer step for every client -----------------------------
    def step(self, images, tokens, labels, first: bool, dropout_mask=None, last: bool = False,
             loss_out: Optional[torch.Tensor] = None, out: Optional[ClientMatrix] = None,
             negate_rows: int = 0) -> torch.Tensor:
        """One local step of every client (chunk by chunk); returns the [K] losses.
        With out (a training-order client matrix) and last, the step writes the
        updated live parameters into out's rows (rows < negate_rows negated)."""
        if loss_out is None:
            loss_out = torch.empty(self.K, dtype=torch.float32, device=self.device)
        c = self.cfg
        for (c0, c1), xp, mp in zip(self.chunks, self._xp, self._mp):
            whole = c0 == 0 and c1 == self.K
            leaves = [(w if whole else w[c0:c1]).detach().requires_grad_(True) for w in self.W]
            params: Dict[str, torch.Tensor] = dict(zip(self.names, leaves))
            sl = (lambda t: t) if whole else (lambda t: None if t is None else t[c0:c1])
            slots = self._norm_slots(images.shape[1], c0, c1)
            logits = batched_forward(params, sl(images), sl(tokens), self.spec, sl(dropout_mask), self.tap_major,
                                     self.skip_dead, norm_slots=slots)
            loss_k = CrossEntropy.apply(logits, sl(labels))
            grads = [g.contiguous() for g in torch.autograd.grad(loss_k.sum(), leaves)]
            if slots is not None and not all(s.used for s in slots.values()):
                missed = sorted(n for n, s in slots.items() if not s.used)
                raise RuntimeError(f"fused clip norm: no partials written for {missed}")
            gp = (ctypes.c_void_p * len(self.blocks))(*[grads[j].data_ptr() + 4 * o for j, o, _, _ in self.blocks])
            xo, ld, nneg = None, 0, 0
            if out is not None and last:
                ld = out.data.stride(0)
                xo = out.data.data_ptr() + 4 * c0 * ld
                nneg = max(0, min(negate_rows, c1) - c0)
            sq, nsq = (None, 0) if slots is None else (self._sq.data_ptr() + 8 * c0 * self._sq.shape[1],
                                                       self._sq.shape[1])
            _capi.call("flr_clip_sgd_step_blocked_x", xp, gp, mp, self._np, self._cs, len(self.blocks), c1 - c0,
                       c.lr, c.momentum, c.weight_decay, c.clip, int(first) | (int(last) << 1), xo, self._xo, ld,
                       nneg, None if slots is None else self._normed, sq, nsq, self.norms.data_ptr() + 4 * c0,
                       self._ws.data_ptr() + self._ws_off, self._ws_bytes, _stream(self._wbuf))
            del grads, leaves, params, logits
            _capi.call("flr_copy_rows", loss_k.data_ptr(), c1 - c0, c1 - c0, loss_out.data_ptr() + 4 * c0, c1 - c0, 1,
                       _stream(loss_out))
        return loss_out

    def local_update(self, batches: Sequence, dropout_masks: Optional[Sequence] = None,
                     export: bool = True, negate_rows: int = 0, gtrain: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Runs len(batches) steps; returns each client's mean loss [K]
        (fl_client.py:143-149).  The per-step losses land in one [steps, K]
        buffer and are averaged by one flr_sum_rows pass (sum in step order).
        export: X <- the torch-order client matrix (export()).  gtrain (the
        round's training-order global vector, loaded by load_global_train):
        X <- the TRAINING-order client matrix instead, written by the last
        optimizer step, the untrained dead-tap ranges copied from gtrain."""
        n = max(1, len(batches))
        steps = torch.empty(n, self.K, dtype=torch.float32, device=self.device)
        direct = gtrain is not None and export and len(batches) > 0
        for s, (images, tokens, labels) in enumerate(batches):
            mask = None if dropout_masks is None else dropout_masks[s]
            self.step(images, tokens, labels, first=(s == 0), dropout_mask=mask, last=(s == len(batches) - 1),
                      loss_out=steps[s], out=self.X if direct else None, negate_rows=negate_rows)
        if direct:
            st = _stream(self._wbuf)
            ld = self.X.data.stride(0)
            for off, c in self.dead_ranges:
                _capi.call("flr_broadcast_rows_neg", gtrain.data_ptr() + 4 * off, c, self.X.data.data_ptr() + 4 * off,
                           self.K, ld, negate_rows, st)
        elif export:
            self.export(negate_rows)
        total = torch.empty(1, self.K, dtype=torch.float32, device=self.device)
        _capi.call("flr_mean_rows", steps.data_ptr(), len(batches), self.K, total.data_ptr(), _stream(total))
        return total[0]


def make_dropout_masks(spec: ModelSpec, steps: int, client_ids, B: int, device,
                       seed: int) -> Optional[List[torch.Tensor]]:
    """Explicit inverted-dropout masks {0, 1/(1-p)} per step, [K, B, fusion]
    each.  client_ids: the global ids of the rows (an int K means 0..K-1);
    client c's masks come from its own stream seeded seed + c, so they do not
    depend on how clients are sharded over GPUs."""
    if spec.dropout <= 0:
        return None
    ids = range(client_ids) if isinstance(client_ids, int) else client_ids
    keep = 1.0 - spec.dropout
    u = torch.empty(steps, len(ids), B, spec.fusion)
    for j, c in enumerate(ids):
        g = torch.Generator(device="cpu")
        g.manual_seed(seed + int(c))
        u[:, j] = torch.rand(steps, B, spec.fusion, generator=g)
    m = ((u < keep).float() / keep).to(device)
    return [m[s] for s in range(steps)]


def synthetic_batches(spec: ModelSpec, steps: int, client_ids: Sequence[int], batch: int, device,
                      seed_base: int = 1000):
    """SURVEY §8d inputs: images N(0,1) [B,3,32,32], tokens U{0..V-1} [B,T],
    labels U{0..C-1}; client c's stream seeded 1000 + c (independent of how
    clients are sharded over GPUs).  The C1 ("cub") family gets the tokens as a
    multi-hot [B, V] float vector (its attribute input)."""
    K = len(client_ids)
    imgs = torch.empty(steps, K, batch, spec.in_channels, spec.image_size, spec.image_size, device=device)
    toks = torch.empty(steps, K, batch, spec.seq_len, dtype=torch.int64, device=device)
    labs = torch.empty(steps, K, batch, dtype=torch.int64, device=device)
    for j, c in enumerate(client_ids):
        g = torch.Generator(device="cpu")
        g.manual_seed(seed_base + int(c))
        imgs[:, j] = torch.randn(steps, batch, spec.in_channels, spec.image_size, spec.image_size, generator=g).to(device)
        toks[:, j] = torch.randint(0, spec.vocab, (steps, batch, spec.seq_len), generator=g).to(device)
        labs[:, j] = torch.randint(0, spec.num_classes, (steps, batch), generator=g).to(device)
    if spec.family == "cub":  # C1's text modality: the multi-hot attribute ("BoW") vector of the tokens
        text = torch.zeros(steps, K, batch, spec.vocab, device=device).scatter_(3, toks, 1.0)
        return [(imgs[s], text[s], labs[s]) for s in range(steps)]
    return [(imgs[s], toks[s], labs[s]) for s in range(steps)]
