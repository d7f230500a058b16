"""Host side of the pairwise-space Weiszfeld (flr.defenses.geometric_median):
the coefficient iteration over K x K distances must reproduce the oracle's
direct loop over the full vectors (trimmed_mean.py:216-251) — same iteration
count and the same estimate to fp32 precision.  CPU only (numpy distances)."""
import numpy as np
import pytest
import torch

from flr.defenses.geometric_median import weiszfeld_pairwise
from oracle import aggregation as ref


def _case(K, P, seed, outliers=0):
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(P, generator=g) * 0.05
    rows = [base + torch.randn(P, generator=g) * 0.01 * (1 + 0.5 * i / K) for i in range(K)]
    for i in range(outliers):
        rows[i] = -rows[i] * 3
    return [[r[: P // 2].clone(), r[P // 2:].clone()] for r in rows]


@pytest.mark.parametrize("K,P,seed,outliers,tol", [(5, 300, 1, 0, 1e-5), (16, 2000, 2, 3, 1e-5),
                                                   (33, 1000, 3, 6, 1e-6), (7, 64, 4, 1, 1e-3)])
def test_pairwise_weiszfeld_matches_direct(K, P, seed, outliers, tol):
    ups = _case(K, P, seed, outliers)
    want, iters = ref.geometric_median(ups, max_iters=100, tolerance=tol)
    U = torch.stack([torch.cat([p.flatten() for p in u]) for u in ups]).double()
    D = torch.cdist(U, U).numpy()
    med = torch.median(U.float(), dim=0)[0].double()
    d0 = torch.norm((U.float() - med.float()).double(), dim=1).numpy()
    w, W, n = weiszfeld_pairwise(D, d0, 100, tol)
    got = (torch.from_numpy(w).double() @ U) / float(W)
    assert abs(n - iters) <= 1, (n, iters)
    err = (got - want.double()).abs().max().item()
    assert err <= 1e-5 * max(1.0, want.abs().max().item()), err


def test_zero_iters_case_returns_median_weights_shape():
    ups = _case(4, 40, 5)
    U = torch.stack([torch.cat([p.flatten() for p in u]) for u in ups]).double()
    D = torch.cdist(U, U).numpy()
    w, W, n = weiszfeld_pairwise(D, np.ones(4), 1, 1e-5)
    assert w.shape == (4,) and n == 1


def test_duplicate_clients_trigger_direct_fallback():
    """Colluding clients sending the same vector: the Weiszfeld iterate moves
    onto their point, dist2 = (D2 a)_i - a^T D2 a / 2 cancels, and the
    pairwise form declines (None -> the defense runs the direct passes)."""
    ups = _case(9, 500, 6)
    for i in range(1, 4):  # 4 of 9 identical: the iterate converges onto their point (44 iterations)
        ups[i] = [t.clone() for t in ups[0]]
    U = torch.stack([torch.cat([p.flatten() for p in u]) for u in ups]).double()
    D = torch.cdist(U, U).numpy()
    med = torch.median(U.float(), dim=0)[0].double()
    d0 = torch.norm((U.float() - med.float()).double(), dim=1).numpy()
    assert weiszfeld_pairwise(D, d0, 100, 1e-5) is None
