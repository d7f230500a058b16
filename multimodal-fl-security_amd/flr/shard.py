"""Coordinate-sharded exchange: the round's one data exchange as an all-to-all.

The reference aggregates one K×P client matrix on one host
(src/defenses/krum.py:55-99, trimmed_mean.py:74-101, base_defense.py:80-97).
With the K clients sharded over G GPUs (flr.dist), the straightforward
exchange is an all-gather of every GPU's (K/G)×P row block: each GPU then
receives (G-1)/G · 4KP bytes (C3 at G = 8: 5.3 GB) and holds all of X.

Every aggregator of the hot path is either coordinate-wise (FedAvg,
trimmed mean, median, the Multi-Krum mean) or a sum over coordinates of
per-coordinate terms (Krum's Gram matrix).  So the exchange here is the
TRANSPOSE of the client sharding instead: GPU g receives all K clients'
values for its own contiguous coordinate range (one all-to-all,
(G-1)/G · 4KP/G bytes received per GPU: 8x less at G = 8), aggregates its
range, and one all-gather of the P-vector slices rebuilds the global model.

Coordinate ranges are unions of the pairwise kernel's canonical slices
(FLR_PW_SLICES = 8, include/flr.h): GPU g owns slices [8g/G, 8(g+1)/G), and
the coordinates past the last full 64-chunk belong to the last GPU.  The
pairwise kernels compute per-slice records that do not depend on G, and the
coordinate-wise kernels compute each coordinate independently, so every
aggregate — and Krum's distance matrix — is bit-identical at G = 1, 2, 4, 8.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from . import _capi
from .ops import CHUNK

PW_SLICES = 8  # FLR_PW_SLICES


def slice_chunks(P: int, q: int) -> Tuple[int, int]:
    """Full-chunk range [c0, c1) of canonical slice q (flr_pw_slice_chunks)."""
    nch = P // CHUNK
    return nch * q // PW_SLICES, nch * (q + 1) // PW_SLICES


@dataclass(frozen=True)
class CoordPlan:
    """Who owns which coordinates when the K×P matrix is split by columns.
    bounds (world + 1 ascending offsets, 0 .. P): explicit rank boundaries
    instead of the canonical slices' — a training-order round of the
    reference-exact Krum distances aligns them to the tap-major blocks
    (aligned_bounds); the Gram path's per-slice records need the canonical
    ones."""
    P: int
    world: int
    bounds: Optional[Tuple[int, ...]] = None

    def __post_init__(self):
        if PW_SLICES % self.world != 0:
            raise ValueError(f"coordinate sharding needs world | {PW_SLICES} (got {self.world})")

    def slices(self, rank: int) -> Tuple[int, int]:
        per = PW_SLICES // self.world
        return rank * per, (rank + 1) * per

    def chunks(self, rank: int) -> Tuple[int, int]:
        q0, q1 = self.slices(rank)
        return slice_chunks(self.P, q0)[0], slice_chunks(self.P, q1 - 1)[1]

    def coords(self, rank: int) -> Tuple[int, int]:
        """[begin, end) of the coordinates rank owns (tail goes to the last rank)."""
        if self.bounds is not None:
            return self.bounds[rank], self.bounds[rank + 1]
        c0, c1 = self.chunks(rank)
        end = self.P if rank == self.world - 1 else c1 * CHUNK
        return c0 * CHUNK, end

    @property
    def ld(self) -> int:
        """Row stride of every exchanged block: the longest range, 64-aligned."""
        n = max(e - b for b, e in (self.coords(r) for r in range(self.world)))
        return max(CHUNK, (n + CHUNK - 1) // CHUNK * CHUNK)


def aligned_bounds(P: int, world: int, blocks) -> Optional[Tuple[int, ...]]:
    """Rank boundaries for a training-order round whose reference-exact chains
    run through the ranks (ops.pairwise_l2_reference_sharded): every rank's
    range must hold whole tap-major blocks (then it is the same SET of
    coordinates in training and in torch order) and start at a chain step.
    Each canonical boundary moves to the nearest 64-coordinate chunk edge
    outside every block, kept strictly increasing where the gaps allow (a
    block longer than a canonical slice can leave a rank an empty range).
    None when a block reaches the last P mod 8 coordinates (the chains' tail)."""
    plan = CoordPlan(P, world)
    spans = sorted((o, o + co * ci * kk) for o, co, ci, kk in blocks)
    if any(e > P - P % 8 for _, e in spans):
        return None
    # the gaps a boundary may sit in: [lo, hi], both chunk edges
    gaps, prev = [], 0
    for o, e in spans + [(P, P)]:
        lo, hi = -(-prev // CHUNK) * CHUNK, (o // CHUNK) * CHUNK
        if o == P:  # the last rank starts at a chunk edge before the tail
            hi = (P // CHUNK) * CHUNK
        if lo <= hi:
            gaps.append((lo, hi))
        prev = max(prev, e)
    out = [0]
    for r in range(1, world):
        t = plan.coords(r)[0]
        cands = []
        for lo, hi in gaps:
            c = min(max(t, lo), hi)
            cands.append((abs(c - t), c))
        cands.sort()
        pick = next((c for _, c in cands if c > out[-1]), None)
        out.append(pick if pick is not None else out[-1])
    out.append(P)
    return tuple(out)


class Comm:
    """The collectives of a sharded round.  ``nccl`` (RCCL over xGMI) runs on
    the device tensors; ``gloo`` stages CUDA tensors through host memory (the
    world_size > 1 rehearsal on one GPU or on CPU)."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.staged = dist.is_initialized() and dist.get_backend(group) == "gloo"

    def _host(self, t: torch.Tensor) -> torch.Tensor:
        return t.cpu() if (self.staged and t.is_cuda) else t

    def all_reduce_sum(self, t: torch.Tensor) -> None:
        if self.world == 1:
            return
        h = self._host(t)
        dist.all_reduce(h, group=self.group)
        if h is not t:
            t.copy_(h)

    def all_gather(self, out: torch.Tensor, t: torch.Tensor) -> None:
        """out [world * n] <- concat over ranks of t [n] (rank order)."""
        if self.world == 1:
            _copy(t, out, t.numel())
            return
        ho, ht = self._host(out), self._host(t.contiguous())
        dist.all_gather_into_tensor(ho, ht, group=self.group)
        if ho is not out:
            out.copy_(ho)

    def send(self, t: torch.Tensor, dst: int) -> None:
        dist.send(self._host(t.contiguous()), dst, group=self.group)

    def recv(self, t: torch.Tensor, src: int) -> None:
        h = self._host(t)
        dist.recv(h, src, group=self.group)
        if h is not t:
            t.copy_(h)

    def broadcast(self, t: torch.Tensor, src: int) -> None:
        if self.world == 1:
            return
        h = self._host(t)
        dist.broadcast(h, src, group=self.group)
        if h is not t:
            t.copy_(h)

    def all_to_all(self, out: torch.Tensor, t: torch.Tensor) -> None:
        """Equal splits along dim 0: block r of t goes to rank r; out block s came from rank s."""
        if self.world == 1:
            out.copy_(t)
            return
        ho, ht = self._host(out), self._host(t.contiguous())
        dist.all_to_all_single(ho, ht, group=self.group)
        if ho is not out:
            out.copy_(ho)


class CoordSlice:
    """All K clients' values of one GPU's coordinate range: data [K, ld], the
    valid columns [:, :n] are global coordinates [begin, begin + n)."""

    def __init__(self, data: torch.Tensor, plan: CoordPlan, rank: int, comm: Comm):
        self.data, self.plan, self.rank, self.comm = data, plan, rank, comm
        self.begin, self.end = plan.coords(rank)
        self.q0, self.q1 = plan.slices(rank)
        self._gbuf = self._gmine = None

    @property
    def K(self) -> int:
        return self.data.shape[0]

    @property
    def n(self) -> int:
        return self.end - self.begin

    @property
    def P(self) -> int:
        """Length of the WHOLE client vector."""
        return self.plan.P

    @property
    def X(self) -> torch.Tensor:
        return self.data[:, : self.n]

    def gather_vector(self, part: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out [P] <- concatenation of every rank's aggregated range (all-gather)."""
        plan, world = self.plan, self.plan.world
        if world == 1:
            _copy(part, out, self.n)
            return out
        if self._gbuf is None or self._gbuf.device != part.device:
            # allocated once; the tail past n stays zero across rounds
            self._gbuf = torch.zeros(world * plan.ld, dtype=torch.float32, device=part.device)
            self._gmine = torch.zeros(plan.ld, dtype=torch.float32, device=part.device)
        buf, mine = self._gbuf, self._gmine
        mine[: self.n].copy_(part[: self.n])
        self.comm.all_gather(buf, mine)
        for r in range(world):
            b, e = plan.coords(r)
            out[b:e].copy_(buf[r * plan.ld: r * plan.ld + (e - b)])
        return out


def _copy(src: torch.Tensor, dst: torch.Tensor, n: int) -> None:
    """dst[:n] <- src[:n] (contiguous, same dtype): flr_copy_rows on the
    device (bytes as float32 words), torch's copy on the host."""
    if src.is_cuda and dst.is_cuda and src.is_contiguous() and dst.is_contiguous() and src.dtype == dst.dtype \
            and (n * src.element_size()) % 4 == 0:
        w = n * src.element_size() // 4
        _capi.call("flr_copy_rows", src.data_ptr(), w, w, dst.data_ptr(), w, 1, _stream(src))
    else:
        dst.reshape(-1)[:n].copy_(src.reshape(-1)[:n])


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else 0


def pack_for_exchange(local: torch.Tensor, P: int, plan: CoordPlan, send: torch.Tensor) -> None:
    """send [world, K_local, ld] <- local [K_local, >=P] cut at the ranks'
    coordinate ranges (block r = columns plan.coords(r)).  Only the gloo
    rehearsal of CUDA tensors uses it (the staged all-to-all needs one
    contiguous send buffer); RCCL and CPU ranks exchange the row pieces as
    they lie (CoordExchange.exchange)."""
    K_l = local.shape[0]
    for r in range(plan.world):
        b, e = plan.coords(r)
        if local.is_cuda:
            _capi.call("flr_copy_rows", local.data_ptr() + 4 * b, local.stride(0), e - b, send[r].data_ptr(),
                       plan.ld, K_l, _stream(local))
        else:
            send[r, :, : e - b].copy_(local[:, b:e])


class CoordExchange:
    """The exchange of a round: client-sharded rows in, coordinate slice out.
    Buffers are allocated once and reused every round.

    The transpose of the client sharding is a set of row pieces: rank s's
    client k sends its columns plan.coords(r) to rank r, where they land as
    row k of block s (recv[s][k][:n_r]).  Each piece is a contiguous run of
    the trainer's own row, so RCCL sends it in place (one batch of p2p
    sends / receives, K_local per peer): no pack copy of the local matrix
    (round 4's all_to_all_single needed one contiguous send buffer: a read
    and a write of the whole local matrix per round).  Only this rank's own
    block is copied, local -> recv."""

    def __init__(self, K: int, K_local: int, P: int, device, comm: Optional[Comm] = None,
                 bounds: Optional[Tuple[int, ...]] = None):
        self.comm = comm or Comm()
        self.plan = CoordPlan(P, self.comm.world, bounds)
        self.K, self.K_local = K, K_local
        ld = self.plan.ld
        world = self.comm.world
        self.send = self.recv = None
        if world > 1:
            self.recv = torch.zeros(world, K_local, ld, dtype=torch.float32, device=device)
            if self.comm.staged and torch.device(device).type == "cuda":
                self.send = torch.zeros(world, K_local, ld, dtype=torch.float32, device=device)

    def exchange(self, local: torch.Tensor) -> CoordSlice:
        if self.comm.world == 1:  # one GPU holds every coordinate: no copy
            return CoordSlice(local, self.plan, 0, self.comm)
        if self.send is not None:  # gloo staging CUDA tensors through the host: one all-to-all
            pack_for_exchange(local, self.plan.P, self.plan, self.send)
            self.comm.all_to_all(self.recv, self.send)  # recv block s = rank s's clients
        else:
            self._exchange_pieces(local)
        return CoordSlice(self.recv.view(self.K, self.plan.ld), self.plan, self.comm.rank, self.comm)

    def _exchange_pieces(self, local: torch.Tensor) -> None:
        plan, me, world = self.plan, self.comm.rank, self.comm.world
        K_l = local.shape[0]
        b, e = plan.coords(me)
        n = e - b
        if local.is_cuda:  # this rank's own block
            _capi.call("flr_copy_rows", local.data_ptr() + 4 * b, local.stride(0), n, self.recv[me].data_ptr(),
                       plan.ld, K_l, _stream(local))
        else:
            self.recv[me, :, :n].copy_(local[:, b:e])
        ops = []
        for step in range(1, world):  # peers in ring order from this rank: every pair's sends interleave
            dst, src = (me + step) % world, (me - step) % world
            bd, ed = plan.coords(dst)
            for k in range(K_l):
                ops.append(dist.P2POp(dist.isend, local[k, bd:ed], dst, group=self.comm.group))
            for k in range(K_l):
                ops.append(dist.P2POp(dist.irecv, self.recv[src, k, :n], src, group=self.comm.group))
        for req in dist.batch_isend_irecv(ops):
            req.wait()
