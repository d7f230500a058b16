"""Tensor-level wrappers over the flr C ABI (device tensors in, device tensors out).

Each op validates shapes on the host, allocates outputs / workspace with the
PyTorch caching allocator on the tensor's device, and enqueues the HIP
kernels on torch's current stream.  No op has a fallback: a CPU tensor, a
wrong dtype or a missing library raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Sequence, Tuple

import torch

from . import _capi

CHUNK = 64  # coordinates per pairwise chunk; client matrices pad ldx to this
PW_SLICES = 8  # FLR_PW_SLICES: canonical coordinate slices of the pairwise kernels
REFINE_ROWS = 128  # far-cluster rows the Gram path refines per call (include/flr.h, a9)


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _check_matrix(X: torch.Tensor, name: str = "X") -> Tuple[int, int, int]:
    if not isinstance(X, torch.Tensor) or not X.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA/HIP tensor (the engine has no CPU path)")
    if X.dtype != torch.float32 or X.dim() != 2 or X.stride(1) != 1 or X.stride(0) < X.shape[1]:
        raise ValueError(f"{name} must be a row-major float32 [K, P] matrix (got {X.dtype}, "
                         f"shape {tuple(X.shape)}, strides {X.stride()})")
    return X.shape[0], X.shape[1], X.stride(0)


def pairwise_l2(X: torch.Tensor, method: str = "gram", events=None, comm=None,
                tap_blocks: Optional[Sequence[Tuple[int, int, int, int]]] = None, dead=None) -> torch.Tensor:
    """K×K float64 distances, D[i][j] = fp32 ||X_i - X_j|| (krum.py:73-99).

    method: "gram" (centred Gram on MFMA), "direct" (exact fp32 differences,
    fp32/fp64 partial sums) or "reference" (the reference's own torch.norm
    accumulation, bit-identical D over the reference's coordinate order:
    X's columns in that order, or tap_blocks [(off, Cout, Cin, KK), ...]
    naming the convolution weights X holds tap-major — a training-order
    matrix, no reordered copy; include/flr.h flr_pairwise_l2_reference_tap).
    events: optional (begin, end) raw hipEvent_t handles recorded around the
    main MFMA kernel (flr.timing.HipEventPair).
    comm: optional flr.shard.Comm for the reference mode: every rank holds the
    whole X, computes 1/world of the pair tiles and one all-reduce (sum, exact:
    one non-zero term per pair) of the 8·K² bytes of D gives every rank D.
    dead: optional (masks, gdead, nneg[, mark]) with tap_blocks — X's dead-tap
    slabs are not written yet (FLR_TC_DEFER_DEAD): bit t of masks[b] reads tap
    t of block b from the training-order vector gdead, negated on rows < nneg
    (flr_pairwise_l2_reference_tap_dead; the same D as on the filled X).
    mark: an object with .event (a recorded-once torch.cuda.Event): recorded
    on the stream once X has been read for the last time, then mark.recorded
    = True (the round engine writes the slabs beside the chains from there)."""
    K, P, ldx = _check_matrix(X)
    D = torch.empty((K, K), dtype=torch.float64, device=X.device)
    if method == "reference":
        if X.data_ptr() % 16 or ldx % 4:  # the kernels load 16-B pieces of 16-B aligned rows
            if dead is not None:
                raise ValueError("pairwise_l2(dead=): the rows must be 16-B aligned (read in place)")
            Xa = torch.zeros((K, (P + 63) // 64 * 64), dtype=torch.float32, device=X.device)
            Xa[:, :P].copy_(X)
            X, ldx = Xa, Xa.stride(0)
        part, nparts = (0, 1) if comm is None else (comm.rank, comm.world)
        wp, nbytes = _ref_workspace(K, P, X.device, _stream(X))
        taps = [int(v) for blk in (tap_blocks or ()) for v in blk]
        tarr = (ctypes.c_int64 * max(1, len(taps)))(*taps)
        if dead is None:
            _capi.call("flr_pairwise_l2_reference_tap", X.data_ptr(), K, P, ldx, ctypes.addressof(tarr),
                       len(taps) // 4, D.data_ptr(), wp, nbytes, part, nparts, _stream(X))
        else:
            masks, gdead, nneg = dead[:3]
            mark = dead[3] if len(dead) > 3 else None
            if len(masks) != len(taps) // 4 or gdead.device != X.device or gdead.dtype != torch.float32 \
                    or gdead.numel() < P:
                raise ValueError("pairwise_l2(dead=): one mask per tap block and a float32 P-vector on X's device")
            marr = (ctypes.c_uint64 * max(1, len(masks)))(*[int(m) for m in masks])
            _capi.call("flr_pairwise_l2_reference_tap_dead", X.data_ptr(), K, P, ldx, ctypes.addressof(tarr),
                       len(taps) // 4, ctypes.addressof(marr), gdead.data_ptr(), int(nneg), D.data_ptr(), wp,
                       nbytes, part, nparts, None if mark is None else mark.event.cuda_event, _stream(X))
            if mark is not None:
                mark.recorded = True
        if nparts > 1:
            comm.all_reduce_sum(D)
        return D
    if method == "gram":
        ws_fn, fn = "flr_pairwise_l2_workspace", "flr_pairwise_l2"
    elif method == "direct":
        ws_fn, fn = "flr_pairwise_l2_direct_workspace", "flr_pairwise_l2_direct"
    else:
        raise ValueError(f"unknown pairwise method {method!r}")
    nbytes = int(getattr(_capi.lib(), ws_fn)(K, P))
    ws = torch.empty(max(nbytes, 256) + 256, dtype=torch.uint8, device=X.device)
    off = (-ws.data_ptr()) % 256
    if events is not None and method == "gram":
        _capi.call("flr_pairwise_l2_ex", X.data_ptr(), K, P, ldx, D.data_ptr(), ws.data_ptr() + off, nbytes,
                   _stream(X), events[0], events[1])
    else:
        _capi.call(fn, X.data_ptr(), K, P, ldx, D.data_ptr(), ws.data_ptr() + off, nbytes, _stream(X))
    return D


def krum_select(D: torch.Tensor, f: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(scores fp64 [K], order int32 [K]) — krum.py:101-131, 149-176."""
    if not D.is_cuda or D.dtype != torch.float64 or D.dim() != 2 or D.shape[0] != D.shape[1]:
        raise ValueError("D must be a square float64 device matrix")
    D = D.contiguous()
    K = D.shape[0]
    scores = torch.empty(K, dtype=torch.float64, device=D.device)
    order = torch.empty(K, dtype=torch.int32, device=D.device)
    _capi.call("flr_krum_select", D.data_ptr(), K, int(f), scores.data_ptr(), order.data_ptr(), _stream(D))
    return scores, order


def rows_mean(X: torch.Tensor, rows: torch.Tensor, divisor: Optional[int] = None,
              out: Optional[torch.Tensor] = None, dead=None) -> torch.Tensor:
    """Ordered fp32 sum of X[rows] divided by `divisor` (krum.py:182-192).
    dead: optional (ranges [(off, n), ...], gdead, nneg) — X's dead-tap ranges
    are not written (FLR_DEFER_DEAD=2): row k's value there is gdead's, negated
    for k < nneg (flr_rows_mean_dead; the same bits as over the filled rows)."""
    K, P, ldx = _check_matrix(X)
    rows = rows.to(device=X.device, dtype=torch.int32).contiguous()
    m = rows.numel()
    divisor = m if divisor is None else int(divisor)
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=X.device)
    if dead is None:
        _capi.call("flr_rows_mean", X.data_ptr(), K, P, ldx, rows.data_ptr(), m, divisor, out.data_ptr(),
                   _stream(X))
        return out
    ranges, gdead, nneg = dead
    off = (ctypes.c_int64 * max(1, len(ranges)))(*[int(o) for o, _ in ranges])
    ln = (ctypes.c_int64 * max(1, len(ranges)))(*[int(n) for _, n in ranges])
    _capi.call("flr_rows_mean_dead", X.data_ptr(), K, P, ldx, rows.data_ptr(), m, divisor, ctypes.addressof(off),
               ctypes.addressof(ln), len(ranges), gdead.data_ptr(), int(nneg), out.data_ptr(), _stream(X))
    return out


def fill_dead_ranges(vec: torch.Tensor, ranges, gdead: torch.Tensor, negate: bool) -> torch.Tensor:
    """vec's dead-tap ranges <- gdead's (negated when `negate`): one row of a
    FLR_DEFER_DEAD=2 matrix made whole (flr_copy_rows_neg per range)."""
    st = _stream(vec)
    for o, n in ranges:
        _capi.call("flr_copy_rows_neg", gdead.data_ptr() + 4 * o, n, n, vec.data_ptr() + 4 * o, n, 1,
                   1 if negate else 0, st)
    return vec


def fedavg(X: torch.Tensor, num_examples, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Example-weighted average (base_defense.py:80-97)."""
    K, P, ldx = _check_matrix(X)
    n = torch.as_tensor(num_examples, dtype=torch.int64).to(X.device).contiguous()
    if n.numel() != K:
        raise ValueError(f"num_examples has {n.numel()} entries for {K} clients")
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=X.device)
    _capi.call("flr_fedavg", X.data_ptr(), K, P, ldx, n.data_ptr(), out.data_ptr(), _stream(X))
    return out


def _rows_arg(rows, device):
    return rows.to(device=device, dtype=torch.int32).contiguous()


def trimmed_mean(X: torch.Tensor, t: int, out: Optional[torch.Tensor] = None,
                 rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Coordinate-wise mean of sorted ranks [t, m-t) (trimmed_mean.py:74-88)
    over all K rows, or over the row subset `rows` (m = len(rows))."""
    K, P, ldx = _check_matrix(X)
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=X.device)
    if rows is None:
        _capi.call("flr_trimmed_mean", X.data_ptr(), K, P, ldx, int(t), out.data_ptr(), _stream(X))
    else:
        r = _rows_arg(rows, X.device)
        _capi.call("flr_trimmed_mean_rows", X.data_ptr(), K, P, ldx, r.data_ptr(), r.numel(), int(t), out.data_ptr(),
                   _stream(X))
    return out


def median_lower(X: torch.Tensor, out: Optional[torch.Tensor] = None,
                 rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Coordinate-wise lower median (trimmed_mean.py:101, 163), optionally of a row subset."""
    K, P, ldx = _check_matrix(X)
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=X.device)
    if rows is None:
        _capi.call("flr_median_lower", X.data_ptr(), K, P, ldx, out.data_ptr(), _stream(X))
    else:
        r = _rows_arg(rows, X.device)
        _capi.call("flr_median_lower_rows", X.data_ptr(), K, P, ldx, r.data_ptr(), r.numel(), out.data_ptr(),
                   _stream(X))
    return out


def row_norms(X: torch.Tensor, center: Optional[torch.Tensor] = None, kind: str = "l2") -> torch.Tensor:
    """float64 [K]: ||X_i - center|| per row (l2 or linf); fp32 differences,
    fp64 accumulation in a fixed order (differential_privacy.py:223-236,
    trimmed_mean.py:234)."""
    K, P, ldx = _check_matrix(X)
    if kind not in ("l2", "linf"):
        raise ValueError(f"unknown norm kind {kind!r}")
    if center is not None:
        if not center.is_cuda or center.dtype != torch.float32 or center.numel() != P:
            raise ValueError("center must be a float32 device vector of length P")
        center = center.contiguous()
    out = torch.empty(K, dtype=torch.float64, device=X.device)
    nbytes = int(_capi.lib().flr_row_norms_workspace(K))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=X.device)
    _capi.call("flr_row_norms", X.data_ptr(), K, P, ldx, _ptr(center), 0 if kind == "l2" else 1, out.data_ptr(),
               ws.data_ptr(), nbytes, _stream(X))
    return out


def row_dots(X: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """float64 [K]: X_i . v (fltrust.py:176), exact products, fp64 fixed-order sum."""
    K, P, ldx = _check_matrix(X)
    if not v.is_cuda or v.dtype != torch.float32 or v.numel() != P:
        raise ValueError("v must be a float32 device vector of length P")
    v = v.contiguous()
    out = torch.empty(K, dtype=torch.float64, device=X.device)
    nbytes = int(_capi.lib().flr_row_norms_workspace(K))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=X.device)
    _capi.call("flr_row_dots", X.data_ptr(), K, P, ldx, v.data_ptr(), out.data_ptr(), ws.data_ptr(), nbytes,
               _stream(X))
    return out


def weighted_rows(X: torch.Tensor, weights, divisor: float, rows=None, scales=None,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = (sum_j fl(fl(X[rows[j]] * scales[j]) * weights[j])) / divisor, in j order
    (the Python-sum weighted averages of differential_privacy.py:141-148, 268-276,
    323-330 and trimmed_mean.py:240)."""
    K, P, ldx = _check_matrix(X)
    w = torch.as_tensor(weights, dtype=torch.float32).to(X.device).contiguous()
    m = w.numel()
    r = None
    if rows is not None:
        r = torch.as_tensor(rows, dtype=torch.int32).to(X.device).contiguous()
        if r.numel() != m:
            raise ValueError("rows and weights differ in length")
    elif m != K:
        raise ValueError(f"{m} weights for {K} rows")
    s = None
    if scales is not None:
        s = torch.as_tensor(scales, dtype=torch.float32).to(X.device).contiguous()
        if s.numel() != m:
            raise ValueError("scales and weights differ in length")
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=X.device)
    _capi.call("flr_weighted_rows", X.data_ptr(), K, P, ldx, _ptr(r), m, w.data_ptr(), _ptr(s), float(divisor),
               out.data_ptr(), _stream(X))
    return out


# ---- coordinate-sharded Krum distances (flr_pairwise_* phases, include/flr.h) ----

# The reference-exact distances' workspace (the chain sums and the chain-major
# copy of X, up to 8 GiB per segment: ~6 GB at C3) is kept per (device,
# stream) and reused by every later call that fits in it, instead of being
# allocated per call.  FLR_REF_WS_CAP (bytes) bounds it: the
# library then runs the chains over more, shorter segments (the same D).
REF_WS_CAP = int(os.environ.get("FLR_REF_WS_CAP", "0")) or None
_REF_WS: Dict[Tuple[int, int], torch.Tensor] = {}


def _ref_workspace(K: int, P: int, device, stream: int) -> Tuple[int, int]:
    nbytes = int(_capi.lib().flr_pairwise_l2_reference_workspace(K, P))
    if REF_WS_CAP is not None:
        nbytes = min(nbytes, REF_WS_CAP)
    key = (torch.device(device).index or 0, stream)
    ws = _REF_WS.get(key)
    if ws is None or ws.numel() < nbytes + 256:
        _REF_WS.pop(key, None)
        ws = torch.empty(max(nbytes, 256) + 256, dtype=torch.uint8, device=device)
        _REF_WS[key] = ws
    return ws.data_ptr() + (-ws.data_ptr()) % 256, nbytes


def release_workspaces() -> None:
    """Drop the cached reference-exact workspaces (their HBM returns to torch's allocator)."""
    _REF_WS.clear()


def _ws(nbytes: int, device) -> Tuple[torch.Tensor, int]:
    ws = torch.empty(max(nbytes, 256) + 256, dtype=torch.uint8, device=device)
    return ws, ws.data_ptr() + (-ws.data_ptr()) % 256


def pairwise_l2_reference_sharded(cs, tap_blocks=None) -> torch.Tensor:
    """The reference-exact distances (pairwise_l2 "reference") from coordinate
    slices (flr.shard.CoordSlice, the reference's coordinate order): the
    chains run through the ranks in order — rank r continues every pair's 8
    chains over its coordinate range from where rank r-1 left them (the
    8·K² fp32 sums passed on), the last rank adds the P mod 8 tail and takes
    the square roots, and D is broadcast.  Each chain step is the same fp32
    operation in the same order as on one GPU, so D is bit-identical to
    pairwise_l2(X, "reference") at every world size.  A chain cannot be split,
    so the ranks run one after another: the phase costs about the one-GPU
    chain time at any G, with only this rank's 1/G of the rows transposed.
    tap_blocks (a training-order round): the matrix's tap-major blocks
    [(off, Cout, Cin, KK), ...]; the rank boundaries must not cut one
    (shard.aligned_bounds), and the blocks inside this slice are read in
    place (flr_pairwise_l2_reference_partial_tap)."""
    lib = _capi.lib()
    K, P, dev = cs.K, cs.P, cs.data.device
    X, ld = cs.data, cs.data.stride(0)
    comm, rank, world = cs.comm, cs.comm.rank, cs.comm.world
    R = P // 8
    full_end = min(cs.end, 8 * R)
    steps = max(0, full_end - cs.begin) // 8
    if cs.begin % 8:
        raise ValueError("coordinate slices must start at a multiple of 8 coordinates")
    if X.data_ptr() % 16 or ld % 4:
        raise ValueError("coordinate slice rows must be 16-B aligned")
    taps = []
    for o, co, ci, kk in (tap_blocks or ()):
        e = o + co * ci * kk
        if e <= cs.begin or o >= cs.end:
            continue
        if o < cs.begin or e > cs.begin + 8 * steps:
            raise ValueError(f"tap block [{o}, {e}) crosses this rank's chain range [{cs.begin}, "
                             f"{cs.begin + 8 * steps}): the rank boundaries must be tap-block aligned")
        taps += [o - cs.begin, co, ci, kk]
    tarr = (ctypes.c_int64 * max(1, len(taps)))(*taps)
    nbytes = int(lib.flr_pairwise_l2_reference_workspace(K, 8 * steps))
    ws, wp = _ws(nbytes, dev)
    st = _stream(X)
    A = torch.empty(0, dtype=torch.float32, device=dev)
    if K > 1:
        A = torch.as_strided(ws, (8 * K * K * 4,), (1,), (wp - ws.data_ptr())).view(torch.float32)
        if rank > 0:
            comm.recv(A, rank - 1)
        _capi.call("flr_pairwise_l2_reference_partial_tap", X.data_ptr(), K, steps, ld, ctypes.addressof(tarr),
                   len(taps) // 4, int(rank == 0), wp, nbytes, st)
        if rank < world - 1:
            comm.send(A, rank + 1)
    D = torch.empty((K, K), dtype=torch.float64, device=dev)
    if rank == world - 1:
        ntail = P - 8 * R
        xt = X.data_ptr() + 4 * (8 * R - cs.begin)
        _capi.call("flr_pairwise_l2_reference_finish", xt, K, ntail, ld, int(R > 0), wp, D.data_ptr(), st)
    comm.broadcast(D, world - 1)
    return D


def pairwise_l2_sharded(cs, events=None) -> torch.Tensor:
    """K×K float64 distances from a coordinate slice (flr.shard.CoordSlice):
    every rank ends with the same D, bit-identical to pairwise_l2 on the
    whole matrix.  Collectives: one exact sum of the pivot sample, one exact
    sum of the tail term, one all-gather of the per-slice Gram sums."""
    if cs.plan.bounds is not None:
        raise ValueError("the Gram path's per-slice records need the canonical rank boundaries "
                         "(this slice's are tap-block aligned: a training-order reference-exact round)")
    lib = _capi.lib()
    K, P, dev = cs.K, cs.P, cs.data.device
    X, ld = cs.data, cs.data.stride(0)
    st = _stream(X)
    c0, c1 = cs.plan.chunks(cs.rank)
    S = int(lib.flr_pairwise_sample_len(P))
    D = torch.empty((K, K), dtype=torch.float64, device=dev)
    tail = torch.empty((K, K), dtype=torch.float64, device=dev)
    # tail: coordinates past the last full chunk (held by the last rank)
    t0 = (P // CHUNK) * CHUNK - cs.begin
    t0 = min(max(t0, 0), cs.n)
    _capi.call("flr_pairwise_tail", X.data_ptr(), K, ld, t0, cs.n, tail.data_ptr(), st)
    if S == 0:  # no full chunk anywhere: the tail is everything
        cs.comm.all_reduce_sum(tail)
        gsum = torch.zeros(PW_SLICES * int(lib.flr_pairwise_gsum_len(K)), dtype=torch.float64, device=dev)
        _capi.call("flr_pairwise_finish", gsum.data_ptr(), tail.data_ptr(), K, D.data_ptr(), st)
        return D
    Xs = torch.empty((K, S), dtype=torch.float32, device=dev)
    _capi.call("flr_pairwise_sample", X.data_ptr(), K, ld, P, c0, c1, Xs.data_ptr(), st)
    cs.comm.all_reduce_sum(Xs)
    nsl = cs.q1 - cs.q0
    nbytes = int(lib.flr_pairwise_sliced_workspace(K, P, nsl))
    ws, wp = _ws(nbytes, dev)
    pivot = torch.empty(int(lib.flr_pairwise_pivot_len()), dtype=torch.int32, device=dev)  # the pivot record
    _capi.call("flr_pairwise_pivot", Xs.data_ptr(), K, P, pivot.data_ptr(), wp, nbytes, st)
    glen = int(lib.flr_pairwise_gsum_len(K))
    mine = torch.empty(nsl * glen, dtype=torch.float64, device=dev)
    ev = (None, None) if events is None else events
    _capi.call("flr_pairwise_gram_slices", X.data_ptr(), K, ld, P, cs.q0, cs.q1, pivot.data_ptr(), mine.data_ptr(),
               wp, nbytes, st, ev[0], ev[1])
    cs.comm.all_reduce_sum(tail)
    gsum = torch.empty(PW_SLICES * glen, dtype=torch.float64, device=dev)
    cs.comm.all_gather(gsum, mine)
    _capi.call("flr_pairwise_finish", gsum.data_ptr(), tail.data_ptr(), K, D.data_ptr(), st)
    return D
