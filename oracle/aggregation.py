"""ORACLE (test infrastructure only) — CPU restatement of the aggregation rules.

Each function follows the cited reference lines with the same torch / numpy
operations in the same order, so on this image it reproduces the reference's
numbers.  Inputs are reference-style ``List[List[Tensor]]`` on the CPU.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

Update = Sequence[torch.Tensor]


def flat(update: Update) -> torch.Tensor:
    """krum.py:55-57 — one fp32 vector per client."""
    return torch.cat([p.flatten().float() for p in update])


def distance_matrix(updates: Sequence[Update]) -> np.ndarray:
    """krum.py:73-99 — fp64 matrix of fp32 torch.norm(.).item() per pair."""
    n = len(updates)
    vecs = [flat(u) for u in updates]
    out = np.zeros((n, n))
    for a in range(n):
        for b in range(a + 1, n):
            v = torch.norm(vecs[a] - vecs[b]).item()
            out[a, b] = v
            out[b, a] = v
    return out


def krum_scores(dist: np.ndarray, num_neighbors: int) -> List[float]:
    """krum.py:101-131 and :165-169 — sum of sorted row entries 1..m."""
    scores = []
    for a in range(dist.shape[0]):
        row_sorted = np.sort(dist[a].copy())
        scores.append(np.sum(row_sorted[1:num_neighbors + 1]))
    return scores


def krum(updates: Sequence[Update], num_malicious: int, multi_k: int):
    """krum.py:149-192.  Returns (aggregate, scores, selected, rejected, dist)."""
    n, f = len(updates), num_malicious
    if n < 2 * f + 3:
        raise ValueError(f"Krum requires n >= 2f + 3. Got n={n}, f={f}.")
    dist = distance_matrix(updates)
    scores = krum_scores(dist, n - f - 2)
    order = np.argsort(scores)
    selected = order[:multi_k].tolist()
    rejected = order[multi_k:].tolist()
    if multi_k == 1:
        return list(updates[selected[0]]), scores, selected, rejected, dist
    chosen = [updates[i] for i in selected]
    agg = []
    for pi in range(len(chosen[0])):
        total = sum(u[pi] for u in chosen)
        agg.append(total / multi_k)
    return agg, scores, selected, rejected, dist


def fedavg(updates: Sequence[Update], num_examples: Sequence[int]) -> List[torch.Tensor]:
    """base_defense.py:80-97 (== run_experiments.py:246-254)."""
    total_examples = sum(num_examples)
    agg = []
    for pi in range(len(updates[0])):
        weighted = sum(num_examples[i] * updates[i][pi] for i in range(len(updates)))
        agg.append(weighted / total_examples)
    return agg


def median(updates: Sequence[Update]) -> List[torch.Tensor]:
    """trimmed_mean.py:92-103 / 156-166 — torch.median(dim=0) (lower median)."""
    agg = []
    for pi in range(len(updates[0])):
        stacked = torch.stack([u[pi].float() for u in updates])
        agg.append(torch.median(stacked, dim=0)[0])
    return agg


def trimmed_mean(updates: Sequence[Update], trim_ratio: float) -> Tuple[List[torch.Tensor], int]:
    """trimmed_mean.py:63-90.  Returns (aggregate, num_trimmed_per_end)."""
    n = len(updates)
    t = max(1, int(n * trim_ratio))
    if n - 2 * t < 1:
        return median(updates), t
    agg = []
    for pi in range(len(updates[0])):
        stacked = torch.stack([u[pi].float() for u in updates])
        sorted_vals, _ = torch.sort(stacked, dim=0)
        agg.append(sorted_vals[t:n - t].mean(dim=0))
    return agg, t


def _weighted_avg(updates: Sequence[Update], num_examples: Sequence[int]) -> List[torch.Tensor]:
    total_examples = sum(num_examples)
    agg = []
    for pi in range(len(updates[0])):
        weighted = sum(num_examples[i] * updates[i][pi] for i in range(len(updates)))
        agg.append(weighted / total_examples)
    return agg


def gradient_clipping(updates: Sequence[Update], num_examples: Sequence[int], clip_norm: float = 1.0,
                      clip_type: str = "l2"):
    """differential_privacy.py:223-283.  Returns (aggregate, original_norms, clipped_count)."""
    norms, clipped, count = [], [], 0
    for u in updates:
        f = torch.cat([t.flatten().float() for t in u])
        norm = torch.max(torch.abs(f)).item() if clip_type == "linf" else torch.norm(f).item()
        norms.append(norm)
        if norm > clip_norm:
            scale = clip_norm / norm
            count += 1
            clipped.append([t * scale for t in u])
        else:
            clipped.append(list(u))
    return _weighted_avg(clipped, num_examples), norms, count


def norm_bounding(updates: Sequence[Update], num_examples: Sequence[int], max_norm: float = 10.0,
                  min_norm: float = 0.0):
    """differential_privacy.py:299-334.  Returns (aggregate, rejected_clients)."""
    rejected, valid, valid_n = [], [], []
    for i, u in enumerate(updates):
        norm = torch.norm(torch.cat([t.flatten() for t in u])).item()
        if min_norm <= norm <= max_norm:
            valid.append(u)
            valid_n.append(num_examples[i])
        else:
            rejected.append(i)
    if not valid:
        valid, valid_n = list(updates), list(num_examples)
    return _weighted_avg(valid, valid_n), rejected


def dp_sgd_clipped_mean(updates: Sequence[Update], num_examples: Sequence[int], clip_norm: float = 10.0):
    """differential_privacy.py:74-96, 127-152 without the noise (steps 1-2).
    Returns (aggregate before noise, norms)."""
    clipped, norms = [], []
    for u in updates:
        f = torch.cat([t.flatten().float() for t in u])
        norm = torch.norm(f)
        if norm > clip_norm:
            scale = clip_norm / norm
            clipped.append([t * scale for t in u])
        else:
            clipped.append(list(u))
        norms.append(norm.item())
    return _weighted_avg(clipped, num_examples), norms


def geometric_median(updates: Sequence[Update], max_iters: int = 100, tolerance: float = 1e-5):
    """trimmed_mean.py:216-251 (Weiszfeld from the coordinate median).
    Returns (flat aggregate, num_iters)."""
    U = torch.stack([torch.cat([p.flatten().float() for p in u]) for u in updates])
    current = torch.median(U, dim=0)[0]
    num_iters = max_iters
    for it in range(max_iters):
        d = torch.clamp(torch.norm(U - current, dim=1), min=1e-10)
        w = 1.0 / d
        new = (w.unsqueeze(1) * U).sum(dim=0) / w.sum()
        change = torch.norm(new - current)
        current = new
        if change < tolerance:
            num_iters = it + 1
            break
    return current, num_iters


def fltrust(updates: Sequence[Update], server_gradient: Update):
    """fltrust.py:158-270 given the server update g.  Returns (aggregate, trust_scores)."""
    sflat = torch.cat([t.flatten().float() for t in server_gradient])
    trust = []
    for u in updates:
        cflat = torch.cat([t.flatten().float() for t in u])
        dot = torch.dot(cflat, sflat)
        cn, sn = torch.norm(cflat), torch.norm(sflat)
        if cn < 1e-10 or sn < 1e-10:
            trust.append(0.0)
        else:
            trust.append(max(0.0, (dot / (cn * sn)).item()))
    normalized = []
    for u in updates:
        un = torch.norm(torch.cat([t.flatten().float() for t in u]))
        if un < 1e-10:
            normalized.append(list(u))
        else:
            scale = torch.norm(sflat) / un
            normalized.append([t * scale for t in u])
    total = sum(trust)
    if total < 1e-10:
        return list(server_gradient), trust
    agg = []
    for pi in range(len(normalized[0])):
        weighted = sum(trust[i] * normalized[i][pi] for i in range(len(normalized)))
        agg.append(weighted / total)
    return agg, trust


def sign_flip(update: Update) -> List[torch.Tensor]:
    """model_poisoning.py:274-276 — IPM without a benign mean negates the update."""
    return [-p for p in update]


# ---- op-level semantics the kernels restate (pinned in tests/test_oracle.py) ----

def numpy_pairwise_sum(a: np.ndarray) -> float:
    """numpy's float64 pairwise summation (what np.sum does on a contiguous slice)."""
    n = len(a)
    if n < 8:
        res = 0.0
        for i in range(n):
            res += a[i]
        return res
    if n <= 128:
        r = [a[j] for j in range(8)]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += a[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return numpy_pairwise_sum(a[:n2]) + numpy_pairwise_sum(a[n2:])


def torch_outer_sum(rows: torch.Tensor) -> torch.Tensor:
    """torch's CPU vectorised outer reduction (cascade_sum / multi_row_sum):
    16-row blocks accumulated from zero, folded through 4 levels."""
    R = rows.shape[0]
    acc = [torch.zeros(rows.shape[1:], dtype=rows.dtype) for _ in range(4)]
    i = 0
    while i + 16 <= R:
        for _ in range(16):
            acc[0] = acc[0] + rows[i]
            i += 1
        for j in range(1, 4):
            acc[j] = acc[j] + acc[j - 1]
            acc[j - 1] = torch.zeros_like(acc[0])
            if i & (15 << (4 * j)):
                break
    while i < R:
        acc[0] = acc[0] + rows[i]
        i += 1
    for j in range(1, 4):
        acc[0] = acc[0] + acc[j]
    return acc[0]
