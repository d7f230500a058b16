"""GPU parity for the §8(f) defenses: gradient clipping (l2 / linf), norm
bounding, DP-SGD (clipped mean exact-path + noise statistics) and the
geometric median (pairwise-space and direct Weiszfeld) vs the oracle.

Bars: clip counts / rejected clients / iteration counts exact (inputs are
built with norms well away from the thresholds); aggregates within 1e-5 x
scale (norms differ from the reference's fp32 torch.norm by its own drift,
~1e-7 at these sizes, which moves clip scales by the same relative amount).
"""
import numpy as np
import pytest
import torch

from oracle import aggregation as orc
from flr import ops
from flr.defenses import get_defense
from flr.matrix import ClientMatrix

pytestmark = pytest.mark.gpu


def _updates(K, P, seed, spread=True):
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(P, generator=g) * 0.05
    rows = []
    for i in range(K):
        s = 0.01 * (1 + 0.5 * i / K) if spread else 0.01
        r = base + torch.randn(P, generator=g) * s
        if i % 4 == 0:
            r = r * (1 + i)  # a range of norms for the clip / bound decisions
        rows.append(r)
    a, b = P // 3, P - P // 3
    return [[r[:a].view(-1).clone(), r[a:b].clone(), r[b:].clone()] for r in rows]


def _close(got, want, tol=1e-5):
    got = got.detach().double().cpu()
    want = want.detach().double().cpu()
    err = (got - want).abs().max().item()
    assert err <= tol * max(1.0, want.abs().max().item()), err


def _flat(ts):
    return torch.cat([t.reshape(-1) for t in ts])


def test_row_norms_vs_fp64(cuda):
    for K, P in [(1, 1), (3, 7), (17, 4099), (64, 100003)]:
        X = torch.randn(K, P, generator=torch.Generator().manual_seed(K)).to(cuda)
        c = torch.randn(P, generator=torch.Generator().manual_seed(P)).to(cuda)
        for center in (None, c):
            got = ops.row_norms(X, center=center).cpu()
            d = (X - center) if center is not None else X
            want = torch.linalg.vector_norm(d.double().cpu(), dim=1)
            assert torch.allclose(got, want, rtol=1e-12, atol=0), (got - want).abs().max()
            gi = ops.row_norms(X, center=center, kind="linf").cpu()
            assert torch.equal(gi, d.abs().max(dim=1)[0].double().cpu())


def test_row_norms_unaligned_and_strided(cuda):
    X = torch.randn(9, 1001, generator=torch.Generator().manual_seed(3)).to(cuda)
    sub = X[:, 1:1000]  # misaligned base, odd ld
    got = ops.row_norms(sub).cpu()
    want = torch.linalg.vector_norm(sub.double().cpu(), dim=1)
    assert torch.allclose(got, want, rtol=1e-12, atol=0)


@pytest.mark.parametrize("clip_type", ["l2", "linf"])
@pytest.mark.parametrize("K,P", [(5, 333), (16, 4099), (40, 20000)])
def test_gradient_clipping_vs_oracle(cuda, K, P, clip_type):
    ups = _updates(K, P, seed=K + P)
    n = [10 + 3 * i for i in range(K)]
    norms = [(_flat(u).abs().max() if clip_type == "linf" else _flat(u).norm()).item() for u in ups]
    clip = float(np.median(norms))
    if min(abs(v - clip) / clip for v in norms) < 1e-4:
        clip *= 1.01
    want, wnorms, wcount = orc.gradient_clipping(ups, n, clip, clip_type)
    d = get_defense("gradient_clipping", {"clip_norm": clip, "clip_type": clip_type})
    got = d.aggregate([[t.to(cuda) for t in u] for u in ups], n)
    assert d.clipped_count == wcount
    assert np.allclose(d.original_norms, wnorms, rtol=1e-5)
    for a, b in zip(got, want):
        _close(a, b)


@pytest.mark.parametrize("K,P", [(6, 500), (32, 8192)])
def test_norm_bounding_vs_oracle(cuda, K, P):
    ups = _updates(K, P, seed=7 * K)
    n = [100] * K
    norms = sorted(_flat(u).norm().item() for u in ups)
    lo, hi = (norms[1] + norms[2]) / 2, (norms[-3] + norms[-2]) / 2
    want, wrej = orc.norm_bounding(ups, n, hi, lo)
    d = get_defense("norm_bounding", {"max_norm": hi, "min_norm": lo})
    got = d.aggregate([[t.to(cuda) for t in u] for u in ups], n)
    assert d.rejected_clients == wrej and len(wrej) == 4
    for a, b in zip(got, want):
        _close(a, b)
    # nothing kept -> mean of all (differential_privacy.py:320-323)
    want2, _ = orc.norm_bounding(ups, n, 1e-9, 0.0)
    d2 = get_defense("norm_bounding", {"max_norm": 1e-9})
    got2 = d2.aggregate([[t.to(cuda) for t in u] for u in ups], n)
    assert d2.rejected_clients == list(range(K))
    for a, b in zip(got2, want2):
        _close(a, b)


def test_dp_sgd_clipped_mean_and_noise(cuda):
    K, P = 12, 30000
    ups = _updates(K, P, seed=5)
    n = [50] * K
    clip = float(np.median([_flat(u).norm().item() for u in ups])) * 1.003
    want, _ = orc.dp_sgd_clipped_mean(ups, n, clip)
    d = get_defense("dp_sgd", {"clip_norm": clip, "noise_multiplier": 0.5, "seed": 3})
    cm = ClientMatrix.from_updates([[t.to(cuda) for t in u] for u in ups])
    clean = d.clipped_mean(cm, n)
    _close(clean, _flat(want))
    noisy = d.aggregate_flat(cm, n)
    resid = (noisy - clean).double()
    std = clip * 0.5 / K
    assert abs(resid.mean().item()) < 5 * std / np.sqrt(P)
    assert abs(resid.std().item() / std - 1) < 0.03
    assert d.rounds_completed == 1 and d.privacy_spent > 0


@pytest.mark.parametrize("method", ["pairwise", "direct"])
@pytest.mark.parametrize("K,P,tol", [(5, 300, 1e-5), (16, 4099, 1e-5), (33, 2000, 1e-6), (64, 65536, 1e-5)])
def test_geometric_median_vs_oracle(cuda, K, P, tol, method):
    ups = _updates(K, P, seed=K * 3 + 1)
    for i in range(K // 5):
        ups[i] = [-3 * t for t in ups[i]]
    want, iters = orc.geometric_median(ups, 100, tol)
    d = get_defense("geometric_median", {"tolerance": tol, "method": method})
    got = d.aggregate([[t.to(cuda) for t in u] for u in ups], [1] * K)
    assert abs(d.num_iters - iters) <= 1, (d.num_iters, iters)
    _close(_flat(got), want)


def test_geometric_median_duplicate_clients(cuda):
    """Duplicated / colluding client rows: the pairwise identity cancels near
    the shared point, so the defense falls back to the direct passes and
    matches the oracle (trimmed_mean.py:216-251)."""
    K, P = 9, 500
    g = torch.Generator().manual_seed(6)
    base = torch.randn(P, generator=g) * 0.05
    rows = [base + torch.randn(P, generator=g) * 0.01 * (1 + 0.5 * i / K) for i in range(K)]
    ups = [[r[: P // 2].clone(), r[P // 2:].clone()] for r in rows]
    for i in range(1, 4):  # 4 of 9 identical: the iterate converges onto their point
        ups[i] = [t.clone() for t in ups[0]]
    want, iters = orc.geometric_median(ups, 100, 1e-5)
    d = get_defense("geometric_median", {"tolerance": 1e-5})
    got = d.aggregate([[t.to(cuda) for t in u] for u in ups], [1] * K)
    assert d.used_direct
    assert abs(d.num_iters - iters) <= 1, (d.num_iters, iters)
    _close(_flat(got), want)
