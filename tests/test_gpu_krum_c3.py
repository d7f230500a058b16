"""GPU parity of the Krum path at the shapes the benchmark runs.

The Gram kernel picks its bf16 split from P (agg_pairwise.hip gram_terms):
3 terms below 2^20 coordinates, 2 terms at and above — and every BASELINE
config (P = 11.8M, 33M) runs the 2-term variant.  These tests put that
variant (and the 3-term one, forced through FLR_GRAM_TERMS, which the kernel
reads on every call) against:

* the C3-shaped golden fixtures (tests/golden/c3krum_*.npz, make_golden.py
  main_c3): K = 128, f = 25 sign-flipped clients, multi_k = 64, the §8d
  generator, outputs of the oracle (krum.py:73-192, run_experiments.py:155-162)
  — selected / rejected indices and the Multi-Krum mean bit-exact;
* fp64 distances at the full C3 size P = 11,800,394.

Each case prints the selection-boundary margin next to the measured distance
error ("report the minimum boundary margin alongside every
index-parity check") and asserts the score shift stays below a quarter of it.
"""
import hashlib

import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden
from oracle import aggregation as orc
from flr import ops
from flr.defenses import KrumDefense
from flr.matrix import ClientMatrix, padded_ld
from flr.workload import update_matrix

pytestmark = pytest.mark.gpu

# relative distance error vs fp64 (DESIGN.md §3 error model): pairs near the
# pivot ~1e-7; pairs inside the far sign-flipped cluster (cancellation factor
# ~100 against the pivot) up to ~1e-5
TOL_BULK = 2e-6
TOL_ALL = 5e-5


def _margin(scores, mk):
    s = np.sort(np.asarray(scores))
    return float((s[mk] - s[mk - 1]) / abs(s[mk]))


def _rel_offdiag(D, ref):
    K = D.shape[0]
    off = ~np.eye(K, dtype=bool)
    return np.abs(D - ref)[off] / ref[off]


@pytest.mark.parametrize("terms", ["auto", "2", "3"])
@pytest.mark.parametrize("path", golden_files("c3krum"), ids=lambda p: p.split("/")[-1])
def test_c3_krum_fixture_bitexact_selection(cuda, path, terms, knob):
    if terms != "auto":
        knob("FLR_GRAM_TERMS", terms)
    fx = load_golden(path)
    K, P, f, mk = (int(fx[k]) for k in ("K", "P", "f", "multi_k"))
    X = update_matrix(K, P, f=f, seed=int(fx["seed"]), device="cpu")[:, :P]
    Xd = X.double()
    assert float(Xd.sum()) == float(fx["x_sum"])  # same CPU generator stream as the fixture
    data = torch.zeros((K, padded_ld(P)), dtype=torch.float32, device=cuda)
    data[:, :P] = X.to(cuda)
    cm = ClientMatrix(data, P, [(P,)])
    d = KrumDefense({"num_malicious": f, "multi_k": mk, "pairwise_method": "gram"})
    flat = d.aggregate_flat(cm, [1] * K)
    D = d.distances.cpu().numpy()
    assert np.all(np.diag(D) == 0) and np.array_equal(D, D.T)
    err_exact = _rel_offdiag(D, fx["exact"])
    err_ref = _rel_offdiag(D, fx["dist"])
    benign = np.arange(K) >= f
    bulk = _rel_offdiag(D[np.ix_(benign, benign)], fx["exact"][np.ix_(benign, benign)])
    scores = np.asarray(orc.krum_scores(D, K - f - 2))
    shift = float(np.max(np.abs(scores - fx["scores"]) / fx["scores"]))
    margin = float(fx["margin"])
    gram_terms = terms if terms != "auto" else ("3" if P < (1 << 20) else "2")
    print(f"\n[c3krum K={K} P={P} gram_terms={gram_terms}] boundary margin {margin:.3e} | distance error vs fp64: "
          f"all {err_exact.max():.2e}, benign {bulk.max():.2e} | vs reference fp32 norm {err_ref.max():.2e} "
          f"(reference's own error {float(fx['ref_err']):.2e}) | score shift {shift:.2e}")
    assert err_exact.max() < TOL_ALL and bulk.max() < TOL_BULK
    assert err_ref.max() < float(fx["ref_err"]) + TOL_ALL
    assert shift < margin / 4
    assert d.selected_clients == fx["selected"].tolist()
    assert d.rejected_clients == fx["rejected"].tolist()
    assert hashlib.sha256(flat.cpu().numpy().tobytes()).hexdigest() == str(fx["agg_sha256"])


def _exact_fp64(X: torch.Tensor) -> np.ndarray:
    """fp64 distances of a device matrix via a centred fp64 Gram (chunked)."""
    K, P = X.shape
    G = torch.zeros(K, K, dtype=torch.float64, device=X.device)
    step = 1 << 22
    for c in range(0, P, step):  # centring per column is exact for distances
        Y = X[:, c:c + step].double()
        Y = Y - Y.mean(dim=0, keepdim=True)
        G += Y @ Y.T
    dg = torch.diag(G)
    D = (dg[:, None] + dg[None, :] - 2 * G).clamp_min(0).sqrt().cpu().numpy()
    np.fill_diagonal(D, 0.0)
    return D


@pytest.mark.parametrize("K,P", [(128, 11_800_394), (128, 1 << 20), (64, 3_000_017)])
def test_gram_two_term_production_size_vs_fp64(cuda, K, P):
    """The default (2-term) Gram path at the C3 size against fp64 and against
    the direct-difference kernel; Krum selection from it equals the selection
    from the fp64 distances (numpy scores restated, krum.py:101-131, 174)."""
    f = int(0.2 * K)
    mk = K // 2
    X = update_matrix(K, P, f=f, seed=K + P % 1000, device=cuda)[:, :P]
    Dg = ops.pairwise_l2(X, "gram").cpu().numpy()
    Dd = ops.pairwise_l2(X, "direct").cpu().numpy()
    exact = _exact_fp64(X)
    benign = np.arange(K) >= f
    eg, ed = _rel_offdiag(Dg, exact), _rel_offdiag(Dd, exact)
    bulk = _rel_offdiag(Dg[np.ix_(benign, benign)], exact[np.ix_(benign, benign)])
    s_exact = orc.krum_scores(exact, K - f - 2)
    margin = _margin(s_exact, mk)
    s_gram = np.asarray(orc.krum_scores(Dg, K - f - 2))
    shift = float(np.max(np.abs(s_gram - np.asarray(s_exact)) / np.asarray(s_exact)))
    print(f"\n[gram 2-term K={K} P={P}] margin {margin:.3e} | gram vs fp64: all {eg.max():.2e}, benign {bulk.max():.2e}"
          f" | direct vs fp64 {ed.max():.2e} | score shift {shift:.2e}")
    assert eg.max() < TOL_ALL and bulk.max() < TOL_BULK
    # the direct kernel accumulates each segment's squares in fp32: ~1e-5 at 1e7
    # coordinates (the reference's torch.norm: ~3e-4)
    assert ed.max() < 3e-5
    assert shift < margin / 4
    _, order = ops.krum_select(torch.from_numpy(Dg).to(cuda), f)
    ref_order = np.argsort(s_exact, kind="stable")
    got = order.cpu().numpy()
    assert got[:mk].tolist() == ref_order[:mk].tolist()
    assert sorted(got[mk:].tolist()) == sorted(ref_order[mk:].tolist())
    assert not set(got[:mk].tolist()) & set(range(f))
