"""Synthetic workloads — generated on the device, never timed.

Aggregation-only client matrix:
  g ~ N(0, 0.05^2) (seed), X[i] = g + sigma_i * N(0, 1), sigma_i = 0.01 (1 + 0.5 i / K),
  sign-flip attackers i < f submit -(g + sigma_i N) (model_poisoning.py:274-276 applied
  as in malicious_client.py:103-115).
The heteroscedastic sigma spreads benign Krum scores by ~0.4 % per rank, far
above the fp32 rounding of the reference's torch.norm, so reference indices
are well conditioned.
"""
from __future__ import annotations

import torch

from .matrix import padded_ld


def update_matrix(K: int, P: int, f: int = 0, seed: int = 7, device="cuda",
                  ld: int = None) -> torch.Tensor:
    """[K, ld] float32 with the first P columns filled (padding zero)."""
    ld = padded_ld(P) if ld is None else ld
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    X = torch.zeros((K, ld), dtype=torch.float32, device=device)
    g = torch.randn(P, generator=gen, device=device, dtype=torch.float32) * 0.05
    for i in range(K):
        sigma = 0.01 * (1.0 + 0.5 * i / K)
        row = X[i, :P]
        row.normal_(0.0, 1.0, generator=gen)
        row.mul_(sigma).add_(g)
        if i < f:
            row.neg_()
    return X


def split_rows(X: torch.Tensor, P: int, shapes):
    """Reference-style List[List[Tensor]] views of a client matrix."""
    out = []
    for i in range(X.shape[0]):
        off, parts = 0, []
        for s in shapes:
            n = int(torch.Size(s).numel())
            parts.append(X[i, off:off + n].view(s))
            off += n
        out.append(parts)
    return out
