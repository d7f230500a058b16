"""flr_train_clients from Python: the C entry that trains a batch of clients
of the C2/C3 model family with no torch in the loop (include/flr.h; the
client plugin of SURVEY §8(b), FLClient.fit / _train fl_client.py:76-149 and
the simulation body run_experiments.py:193-240).  This wrapper only marshals
device buffers (torch is the allocator here); a non-torch caller binds the
same symbol over ctypes / cgo / N-API."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

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
