"""flr_train_clients / flr_train_vit_bert from Python: the C entries that
train a batch of clients of the C2/C3 (ResNet + GRU) and C4/C5 (ViT + BERT)
model families with no torch in the loop (include/flr.h; the
client plugin of SURVEY §8(b), FLClient.fit / _train fl_client.py:76-149 and
the simulation body run_experiments.py:193-240).  This wrapper only marshals
device buffers (torch is the allocator here); a non-torch caller binds the
same symbol over ctypes / cgo / N-API."""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch

from . import _capi
from .models.multimodal import ModelSpec
from .train import TrainConfig


class ResNetGruSpec(ctypes.Structure):
    _fields_ = [("num_classes", ctypes.c_int64), ("image_size", ctypes.c_int64), ("in_channels", ctypes.c_int64),
                ("widths", ctypes.c_int64 * 4), ("blocks", ctypes.c_int64 * 4), ("vocab", ctypes.c_int64),
                ("seq_len", ctypes.c_int64), ("embed", ctypes.c_int64), ("hidden", ctypes.c_int64),
                ("fusion", ctypes.c_int64)]

    @classmethod
    def of(cls, spec: ModelSpec) -> "ResNetGruSpec":
        if spec.family != "resnet_gru" or len(spec.widths) != 4 or len(spec.blocks) != 4:
            raise ValueError(f"flr_train_clients serves the ResNet + GRU family, not {spec.family!r}")
        return cls(spec.num_classes, spec.image_size, spec.in_channels, (ctypes.c_int64 * 4)(*spec.widths),
                   (ctypes.c_int64 * 4)(*spec.blocks), spec.vocab, spec.seq_len, spec.embed, spec.hidden,
                   spec.fusion)


class VitBertSpec(ctypes.Structure):
    """flr_vit_bert_spec (include/flr.h): the C4/C5 family's geometry."""
    _fields_ = [(n, ctypes.c_int64) for n in (
        "num_classes", "image_size", "in_channels", "patch", "vit_dim", "vit_depth", "vit_heads", "vit_mlp", "vocab",
        "seq_len", "bert_dim", "bert_depth", "bert_heads", "bert_ffn", "bert_max_pos", "fusion")]

    @classmethod
    def of(cls, spec: ModelSpec) -> "VitBertSpec":
        if spec.family != "vit_bert":
            raise ValueError(f"flr_train_vit_bert serves the ViT + BERT family, not {spec.family!r}")
        return cls(*[int(getattr(spec, n)) for n, _ in cls._fields_])


def num_params(spec: ModelSpec) -> int:
    return int(_capi.lib().flr_resnet_gru_num_params(ctypes.byref(ResNetGruSpec.of(spec))))


def workspace_bytes(spec: ModelSpec, K: int, B: int, steps: int) -> int:
    return int(_capi.lib().flr_train_clients_workspace(ctypes.byref(ResNetGruSpec.of(spec)), K, B, steps))


def train_clients(spec: ModelSpec, global_flat: torch.Tensor, batches: Sequence, cfg: TrainConfig = TrainConfig(),
                  dropout_masks: Optional[Sequence] = None, negate_rows: int = 0,
                  X: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """K clients' local updates in one flr_train_clients call.  batches: per
    step (images [K,B,C,H,W], tokens [K,B,T] int64, labels [K,B] int64).
    Returns (X [K, P] torch-order rows, loss [K], last-step clip norms [K])."""
    dev = global_flat.device
    images = torch.stack([b[0] for b in batches]).float().contiguous()
    tokens = torch.stack([b[1] for b in batches]).long().contiguous()
    labels = torch.stack([b[2] for b in batches]).long().contiguous()
    steps, K, B = labels.shape
    masks = None if dropout_masks is None else torch.stack(list(dropout_masks)).float().contiguous()
    P = int(global_flat.numel())
    if X is None:
        X = torch.empty(K, P, dtype=torch.float32, device=dev)
    loss = torch.empty(K, dtype=torch.float32, device=dev)
    norms = torch.empty(K, dtype=torch.float32, device=dev)
    sp = ResNetGruSpec.of(spec)
    n = workspace_bytes(spec, K, B, steps)
    if n == 0:
        raise ValueError("flr_train_clients: unsupported model or shape")
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    g = global_flat.float().contiguous()
    _capi.call("flr_train_clients", ctypes.byref(sp), g.data_ptr(), X.data_ptr(), X.stride(0), images.data_ptr(),
               tokens.data_ptr(), labels.data_ptr(), None if masks is None else masks.data_ptr(), steps, K, B,
               cfg.lr, cfg.momentum, cfg.weight_decay, cfg.clip, negate_rows, loss.data_ptr(), norms.data_ptr(),
               ws.data_ptr(), n, torch.cuda.current_stream(dev).cuda_stream)
    return X, loss, norms


def vit_bert_num_params(spec: ModelSpec) -> int:
    return int(_capi.lib().flr_vit_bert_num_params(ctypes.byref(VitBertSpec.of(spec))))


def vit_bert_workspace_bytes(spec: ModelSpec, K: int, B: int, steps: int, chunk: int = 0) -> int:
    return int(_capi.lib().flr_train_vit_bert_workspace(ctypes.byref(VitBertSpec.of(spec)), K, B, steps, chunk))


class NativeRoundTrainer:
    """The round engine's trainer on the one-call C entries: flr_train_clients_ex
    (the ResNet + GRU family) and flr_train_vit_bert (the ViT + BERT family).
    The whole local update of this GPU's clients is one C call (captured into
    the round's HIP graph by flr.round), so no torch kernel runs in the
    training phase.  The same surface RoundEngine uses of
    flr.train.ClientBatchTrainer (X, P, to_train_order / to_torch_order,
    load_global[_train], local_update), with the same bits: the kernel
    schedule is the Python trainer's (ResNet + GRU: plus the residual blocks'
    two gradient paths summed in the dgrad epilogue, one rounding, as
    autograd's add)."""

    def __init__(self, spec: ModelSpec, num_clients: int, device, cfg: TrainConfig = TrainConfig(), batch: int = 32):
        from .matrix import ClientMatrix
        from .models.multimodal import param_layout
        self.spec, self.cfg = spec, cfg
        self.device = torch.device(device)
        self.K = int(num_clients)
        self.B = int(batch)
        self.vit = spec.family == "vit_bert"
        self._sp = VitBertSpec.of(spec) if self.vit else ResNetGruSpec.of(spec)
        shapes = [s for _, s in param_layout(spec)]
        self.X = ClientMatrix.empty(self.K, shapes, self.device)
        self.P = self.X.P
        n = vit_bert_num_params(spec) if self.vit else num_params(spec)
        if n != self.P:
            raise RuntimeError(f"the C trainer lays out {n} parameters, the model {self.P}")
        steps = max(1, cfg.local_steps)
        if self.vit:  # no dead taps, no layout change; passes of `chunk` clients as ClientBatchTrainer
            self.live_params = self.P
            from .train import ClientBatchTrainer
            self._chunk = cfg.client_chunk if cfg.client_chunk > 0 else ClientBatchTrainer.auto_chunk(spec, self.K)
            self.chunks = [(c0, min(self.K, c0 + self._chunk)) for c0 in range(0, self.K, self._chunk)]
            self._ws_bytes = vit_bert_workspace_bytes(spec, self.K, self.B, steps, self._chunk)
        else:
            self.live_params = int(_capi.lib().flr_resnet_gru_live_params(ctypes.byref(self._sp), cfg.weight_decay))
            self.chunks = [(0, self.K)]
            self._ws_bytes = workspace_bytes(spec, self.K, self.B, steps)
        if self._ws_bytes == 0:
            raise ValueError("native trainer: unsupported model or shape")
        self._ws = torch.empty(self._ws_bytes, dtype=torch.uint8, device=self.device)
        self._ws_steps = steps
        self.loss = torch.empty(self.K, dtype=torch.float32, device=self.device)
        self.norms = torch.empty(self.K, dtype=torch.float32, device=self.device)
        self._global = None   # the vector the next local_update starts from, and its order
        self._order = 0
        self._bound = None    # (key, stacked copies) when the inputs are not views of one buffer
        # training order: leave X's dead-tap slabs to fill_dead (FLR_TC_DEFER_DEAD; RoundEngine)
        self.defer_dead = False

    def dead_ranges(self) -> List[Tuple[int, int]]:
        """[(off, n), ...]: the dead-tap ranges of a training-order row (the
        untrained slabs the trainer copies from the global vector)."""
        if self.vit:
            return []
        lib, sp, wd = _capi.lib(), ctypes.byref(self._sp), self.cfg.weight_decay
        n = int(lib.flr_resnet_gru_dead_ranges(sp, wd, None, None, 0))
        if n < 0:
            raise ValueError("flr_resnet_gru_dead_ranges: bad spec")
        off, ln = (ctypes.c_int64 * max(1, n))(), (ctypes.c_int64 * max(1, n))()
        lib.flr_resnet_gru_dead_ranges(sp, wd, off, ln, n)
        return [(int(off[i]), int(ln[i])) for i in range(n)]

    def fill_dead(self, gtrain: torch.Tensor, negate_rows: int = 0) -> None:
        """X's dead-tap ranges <- gtrain's (rows < negate_rows negated), on the
        current stream: what a local_update with defer_dead left out."""
        if gtrain.numel() < self.P or gtrain.dtype != torch.float32 or gtrain.device != self.device:
            raise ValueError("fill_dead: a float32 training-order P-vector on the trainer's device")
        _capi.call("flr_resnet_gru_fill_dead", ctypes.byref(self._sp), self.cfg.weight_decay, gtrain.data_ptr(),
                   self.X.data.data_ptr(), self.X.data.stride(0), self.K, int(negate_rows), self._stream())

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _reorder(self, src: torch.Tensor, dst: torch.Tensor, to_train: bool) -> torch.Tensor:
        src = src.to(self.device, torch.float32).contiguous()
        if self.vit:  # training order is the parameters() order
            _capi.call("flr_copy_rows", src.data_ptr(), self.P, self.P, dst.data_ptr(), self.P, 1, self._stream())
            return dst
        _capi.call("flr_resnet_gru_reorder", ctypes.byref(self._sp), src.data_ptr(), dst.data_ptr(), int(to_train),
                   self._stream())
        return dst

    def to_train_order(self, flat: torch.Tensor) -> torch.Tensor:
        return self._reorder(flat, torch.empty(self.P, dtype=torch.float32, device=self.device), True)

    def to_torch_order(self, flat: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if out is None:
            out = torch.empty(self.P, dtype=torch.float32, device=self.device)
        return self._reorder(flat, out, False)

    def load_global(self, global_flat: torch.Tensor) -> None:
        """Every client starts from global_flat (torch order) at the next local_update."""
        self._global, self._order = global_flat, 0

    def load_global_train(self, gtrain: torch.Tensor, live_only: bool = True) -> None:
        """The same from a training-order vector; the next local_update then
        writes X in training order (FLR_TC_TRAIN_ORDER)."""
        self._global, self._order = gtrain, 1

    @staticmethod
    def _adjacent(ts: Sequence[torch.Tensor], dtype) -> Optional[torch.Tensor]:
        """The [steps, ...] tensor the per-step tensors ts are consecutive
        slices of (synthetic_batches / make_dropout_masks return such views),
        as a view: no copy, so the trainer (and a captured graph) reads the
        caller's tensors live.  None if they are not laid out that way."""
        t0 = ts[0]
        if t0.dtype != dtype or not t0.is_contiguous() or t0.device.type != "cuda":
            return None
        step = t0.numel() * t0.element_size()
        for i, t in enumerate(ts):
            if (t.shape != t0.shape or t.dtype != dtype or not t.is_contiguous()
                    or t.data_ptr() != t0.data_ptr() + i * step):
                return None
        return t0.as_strided((len(ts),) + tuple(t0.shape), (t0.numel(),) + tuple(t0.stride()))

    def _inputs(self, batches: Sequence, masks: Optional[Sequence]):
        """[steps][K][B]... inputs.  Step tensors that are consecutive slices
        of one buffer are bound as views (live data, no copy); otherwise they
        are stacked into a copy, re-made whenever an element tensor changes
        (data pointer or in-place version) — but a HIP graph captured on a copy
        keeps reading that copy, so the round engine's inputs are always views."""
        cols = [[b[i] for b in batches] for i in range(3)]
        dts = (torch.float32, torch.int64, torch.int64)
        views = [self._adjacent(c, dt) for c, dt in zip(cols, dts)]
        mview = None if masks is None else self._adjacent(list(masks), torch.float32)
        if all(v is not None for v in views) and (masks is None or mview is not None):
            imgs, toks, labs = views
            m = mview
        else:
            key = tuple((t.data_ptr(), t._version) for c in cols for t in c) + (
                () if masks is None else tuple((t.data_ptr(), t._version) for t in masks))
            if self._bound is None or self._bound[0] != key:
                stacked = [torch.stack(c).to(dt).contiguous() for c, dt in zip(cols, dts)]
                mm = None if masks is None else torch.stack(list(masks)).float().contiguous()
                self._bound = (key, (*stacked, mm))
            imgs, toks, labs, m = self._bound[1]
        if labs.shape[1:] != (self.K, self.B):
            raise ValueError(f"labels {tuple(labs.shape)}: expected [steps, {self.K}, {self.B}]")
        return imgs, toks, labs, m

    def local_update(self, batches: Sequence, dropout_masks: Optional[Sequence] = None, export: bool = True,
                     negate_rows: int = 0, gtrain: Optional[torch.Tensor] = None) -> torch.Tensor:
        """len(batches) local steps of every client from the loaded global
        vector; X <- the client rows (training order after load_global_train,
        else torch order), rows < negate_rows negated; returns the [K] mean losses."""
        if self._global is None:
            raise RuntimeError("local_update before load_global / load_global_train")
        if gtrain is not None and (self._order != 1 or gtrain.data_ptr() != self._global.data_ptr()):
            raise ValueError("local_update(gtrain=) must follow load_global_train(gtrain)")
        steps = len(batches)
        if steps > self._ws_steps:
            raise ValueError(f"{steps} local steps, workspace sized for {self._ws_steps}")
        imgs, toks, labs, m = self._inputs(batches, dropout_masks)
        c = self.cfg
        g = self._global
        if self.vit:
            _capi.call("flr_train_vit_bert", ctypes.byref(self._sp), g.data_ptr(), self.X.data.data_ptr(),
                       self.X.data.stride(0), imgs.data_ptr(), toks.data_ptr(), labs.data_ptr(),
                       None if m is None else m.data_ptr(), steps, self.K, self.B, c.lr, c.momentum,
                       c.weight_decay, c.clip, int(negate_rows), self.loss.data_ptr(), self.norms.data_ptr(),
                       self._order, self._chunk, self._ws.data_ptr(), self._ws_bytes, self._stream())
            return self.loss
        _capi.call("flr_train_clients_ex", ctypes.byref(self._sp), g.data_ptr(), self.X.data.data_ptr(),
                   self.X.data.stride(0), imgs.data_ptr(), toks.data_ptr(), labs.data_ptr(),
                   None if m is None else m.data_ptr(), steps, self.K, self.B, c.lr, c.momentum, c.weight_decay,
                   c.clip, int(negate_rows), self.loss.data_ptr(), self.norms.data_ptr(),
                   self._order | (2 if self._order == 1 and self.defer_dead else 0),
                   self._ws.data_ptr(), self._ws_bytes, self._stream())
        return self.loss
