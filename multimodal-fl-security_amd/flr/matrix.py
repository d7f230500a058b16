"""The client matrix: the engine's one data layout for a round's updates.

K rows (clients, global client order) × P fp32 coordinates, each row the
client's parameters flattened in ``model.parameters()`` order — exactly the
vector ``KrumDefense._flatten_update`` builds per client
(src/defenses/krum.py:55-57).  Rows are padded to a multiple of 64 floats
(256 B) so every row starts 256-B aligned for the LDS-DMA loads; the padding
is never read by the kernels (they take the logical P).

Local training writes each client's parameters straight into its row, so the
server reads the round's updates with no flatten/stack copy; the generic
``List[List[Tensor]]`` interface of the reference is converted on entry.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from .ops import CHUNK


def padded_ld(P: int) -> int:
    return max(CHUNK, (P + CHUNK - 1) // CHUNK * CHUNK)


class ClientMatrix:
    def __init__(self, data: torch.Tensor, P: int, shapes: Sequence[torch.Size],
                 dtypes: Optional[Sequence[torch.dtype]] = None):
        if data.dim() != 2 or data.dtype != torch.float32 or data.stride(1) != 1:
            raise ValueError("client matrix storage must be a row-major float32 2-D tensor")
        self.data = data
        self.P = int(P)
        self.shapes = [torch.Size(s) for s in shapes]
        self.dtypes = list(dtypes) if dtypes is not None else [torch.float32] * len(self.shapes)
        self.numels = [int(torch.Size(s).numel()) for s in self.shapes]
        if sum(self.numels) != self.P:
            raise ValueError(f"shapes hold {sum(self.numels)} elements, P = {self.P}")
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n

    @property
    def K(self) -> int:
        return self.data.shape[0]

    @property
    def X(self) -> torch.Tensor:
        """[K, P] view (row stride = padded ld)."""
        return self.data[:, : self.P]

    @property
    def device(self) -> torch.device:
        return self.data.device

    @classmethod
    def empty(cls, K: int, shapes: Sequence[torch.Size], device, dtypes=None) -> "ClientMatrix":
        P = sum(int(torch.Size(s).numel()) for s in shapes)
        data = torch.zeros((K, padded_ld(P)), dtype=torch.float32, device=device)
        return cls(data, P, shapes, dtypes)

    @classmethod
    def from_updates(cls, client_updates: Sequence[Sequence[torch.Tensor]],
                     device: Optional[torch.device] = None) -> "ClientMatrix":
        """Stack a reference-style ``List[List[Tensor]]`` (one list per client)."""
        if len(client_updates) == 0:
            raise ValueError("no client updates")
        first = client_updates[0]
        shapes = [t.shape for t in first]
        dtypes = [t.dtype for t in first]
        if device is None:
            device = first[0].device if first[0].is_cuda else torch.device("cuda")
        cm = cls.empty(len(client_updates), shapes, device, dtypes)
        for pi in range(len(shapes)):
            off, n = cm.offsets[pi], cm.numels[pi]
            col = torch.stack([u[pi].reshape(-1) for u in client_updates]).to(
                device=device, dtype=torch.float32, non_blocking=True)
            cm.data[:, off:off + n].copy_(col)
        return cm

    def unflatten(self, flat: torch.Tensor, like_device: Optional[torch.device] = None) -> List[torch.Tensor]:
        """Split a [P] vector into per-parameter tensors (views when on device)."""
        out = []
        for off, n, shape in zip(self.offsets, self.numels, self.shapes):
            t = flat[off:off + n].view(shape)
            if like_device is not None and t.device != like_device:
                t = t.to(like_device)
            out.append(t)
        return out

    def row(self, i: int) -> List[torch.Tensor]:
        """Client i's parameters as views into the matrix."""
        return self.unflatten(self.data[i, : self.P])
