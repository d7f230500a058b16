"""GPU parity: the HIP aggregation kernels vs the oracle / golden fixtures.

Bars (north_star): Krum/Multi-Krum indices bit-exact; Krum
scores bit-exact given the same distance matrix; distances within 2e-5
relative of the reference's fp32 torch.norm (whose own error vs exact is
~1e-5 at 1e6 and ~3e-4 at 1e7 coordinates); median bit-exact; Multi-Krum
mean and FedAvg bit-exact; trimmed mean bit-exact on the coordinates torch
sums with its vectorised cascade (every K up to 512), within 1e-5 on its
scalar tail columns.
"""
import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden, shapes_of
from oracle import aggregation as orc
from flr import ops
from flr.defenses import get_defense, KrumDefense
from flr.matrix import ClientMatrix, padded_ld
from flr.workload import split_rows, update_matrix

pytestmark = pytest.mark.gpu


def to_matrix(X_np, device):
    K, P = X_np.shape
    data = torch.zeros((K, padded_ld(P)), dtype=torch.float32, device=device)
    data[:, :P] = torch.from_numpy(X_np).to(device)
    return data[:, :P]


# ---------------- pairwise distances ----------------

@pytest.mark.parametrize("path", golden_files("krum"), ids=lambda p: p.split("/")[-1])
@pytest.mark.parametrize("method", ["gram", "direct"])
def test_pairwise_vs_golden(cuda, path, method):
    fx = load_golden(path)
    X = to_matrix(fx["X"], cuda)
    D = ops.pairwise_l2(X, method).cpu().numpy()
    ref = fx["dist"]
    assert np.all(np.diag(D) == 0) and np.array_equal(D, D.T)
    rel = np.abs(D - ref) / np.maximum(ref, 1e-30)
    np.fill_diagonal(rel, 0)
    assert rel.max() < 2e-5, rel.max()


@pytest.mark.parametrize("K,P", [(1, 100), (2, 64), (3, 1), (33, 129), (64, 4096), (100, 6400),
                                 (128, 65536 + 17), (129, 3000), (200, 2048), (300, 1111)])
def test_pairwise_gram_vs_direct_and_fp64(cuda, K, P):
    """Error model of the Gram path: relative error on a pair's
    distance scales with its cancellation factor w.r.t. the medoid pivot —
    ~1e-7 for pairs near the bulk, up to ~1e-5 for pairs inside a far outlier
    cluster (here the f = K/5 sign-flipped clients).  The direct path has no
    cancellation."""
    f = K // 5
    X = update_matrix(K, P, f=f, seed=K + P, device=cuda)[:, :P]
    Dg = ops.pairwise_l2(X, "gram").cpu().numpy()
    Dd = ops.pairwise_l2(X, "direct").cpu().numpy()
    Xd = X.double().cpu()
    exact = torch.cdist(Xd, Xd).numpy() if K > 1 else np.zeros((1, 1))
    benign = np.arange(K) >= f
    for D, tol_bulk, tol_all in ((Dg, 2e-6, 2e-5), (Dd, 2e-6, 2e-6)):
        rel = np.abs(D - exact) / np.maximum(exact, 1e-30)
        np.fill_diagonal(rel, 0)
        assert rel.max() < tol_all, rel.max()
        assert rel[np.ix_(benign, np.ones(K, bool))].max() < tol_bulk
        assert np.all(np.diag(D) == 0) and np.array_equal(D, D.T)


@pytest.mark.parametrize("K", [129, 300, 512])
def test_pairwise_two_term_gram_wide(cuda, knob, K):
    """The 2-term split that every BASELINE-size call runs (P >= 2^20), forced
    at a small P for K > 128 (the diagonal 128-row groups and the cross
    groups).  Against fp64 distances: 1e-4 for every pair, 2e-5 for the benign
    rows (measured 3.9e-6 / 1.3e-7)."""
    knob("FLR_GRAM_TERMS", "2")
    P = 65536 + 17
    f = K // 5
    X = update_matrix(K, P, f=f, seed=K, device=cuda)[:, :P]
    D = ops.pairwise_l2(X, "gram").cpu().numpy()
    Xd = X.double().cpu()
    exact = torch.cdist(Xd, Xd).numpy()
    rel = np.abs(D - exact) / np.maximum(exact, 1e-30)
    np.fill_diagonal(rel, 0)
    benign = np.arange(K) >= f
    print(f"\n[2-term Gram K={K}] max rel {rel.max():.2e}, benign rows {rel[benign].max():.2e}")
    assert rel.max() < 1e-4, rel.max()
    assert rel[benign].max() < 2e-5
    assert np.all(np.diag(D) == 0) and np.array_equal(D, D.T)


def _far_cluster_matrix(K, P, f, seed, device):
    """A trained round's geometry (SURVEY §8 a16 sign flip on full weights):
    every client close to a large common vector g, the f attackers at -x, so
    |x_i - x_j| ~ 1e-4 |x| inside both clusters."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    X = torch.zeros((K, padded_ld(P)), dtype=torch.float32, device=device)
    g = torch.randn(P, generator=gen, device=device)
    for i in range(K):
        row = X[i, :P]
        row.normal_(0.0, 1e-4 * (1.0 + 0.5 * i / K), generator=gen)
        row.add_(g)
        if i < f:
            row.neg_()
    return X


def _fp64_dist(X):
    Xd = X.double()
    G = (Xd - Xd[0:1]) @ (Xd - Xd[0:1]).T
    d = G.diagonal()
    return (d[:, None] + d[None, :] - 2 * G).clamp_min(0).sqrt().fill_diagonal_(0)


@pytest.mark.parametrize("K,P,f", [(40, 64 * 1000 + 7, 8), (128, 200_000, 25), (128, 70_000, 40),
                                   (130, 64 * 900, 30), (300, 64 * 700, 60), (300, 64 * 700 + 5, 80),
                                   (320, 64 * 500, 100), (128, 64 * 300, 60)])
def test_pairwise_far_cluster_refined(cuda, K, P, f):
    """Pairs inside a cluster far from the medoid pivot (cancellation factor ~1e8
    here) come from the exact-difference refine, every pair within 2e-5 of
    fp64 — including row lists of 33..128 rows (two to four row-list blocks,
    diagonal and off-diagonal block pairs) and K > 128."""
    X = _far_cluster_matrix(K, P, f, seed=K + f, device=cuda)
    D = ops.pairwise_l2(X[:, :P], "gram")
    ref = _fp64_dist(X[:, :P])
    off = ~torch.eye(K, dtype=torch.bool, device=cuda)
    err = ((D - ref).abs()[off] / ref[off]).max().item()
    assert err < 2e-5, err
    # the sharded composition (the phases over any split of the slices) stays bit-identical
    from test_gpu_shard import _phases
    for world in (2, 8):
        assert torch.equal(_phases(X, K, P, world), D)


def test_pairwise_far_cluster_overflow_is_loud(cuda):
    """More far-cluster rows than the refine list holds (140 > 128, only
    possible at K > 128): every distance is NaN, the diagonal included (the
    marker), and Krum raises on the device path itself — with publish=False
    (the round engine's call) too — never a silently inaccurate selection."""
    from flr._capi import FlrError
    K, P, f = 300, 64 * 200, 140
    X = _far_cluster_matrix(K, P, f, seed=3, device=cuda)
    D = ops.pairwise_l2(X[:, :P], "gram")
    assert torch.isnan(D).all()
    for publish in (True, False):
        d = KrumDefense({"num_malicious": f, "multi_k": K // 2, "pairwise_method": "gram"})
        with pytest.raises(FlrError):
            d.aggregate_flat(ClientMatrix(X, P, [(P,)]), [1] * K, publish=publish)
    # the exact paths have no such limit (the reference mode: the default)
    Dd = ops.pairwise_l2(X[:, :P], "direct")
    assert not torch.isnan(Dd).any()
    d = KrumDefense({"num_malicious": f, "multi_k": K // 2})
    d.aggregate_flat(ClientMatrix(X, P, [(P,)]), [1] * K)
    assert not torch.isnan(d.distances).any()


@pytest.mark.parametrize("method,bad", [("direct", 5), ("gram", 5), ("gram", 0), ("reference", 0)])
def test_krum_nan_client_is_rejected(cuda, method, bad):
    """A client that sends NaN (krum.py:89-131 on numpy): its distances are
    NaN, np.sort puts them last in every row, its own score is NaN and
    np.argsort ranks it last — rejected, every order slot written, the other
    clients' scores and order those of the oracle.  Gram mode with the NaN
    client at row 0 (an attacker index): the pivot is chosen among the rows
    with finite sample distances, not row 0 by default."""
    K, P, f = 12, 3000, 2
    g = torch.Generator().manual_seed(11)
    X = torch.randn(K, P, generator=g) * 0.1
    X[bad, 17] = float("nan")
    data = torch.zeros((K, 3008), dtype=torch.float32)
    data[:, :P] = X
    d = KrumDefense({"num_malicious": f, "multi_k": 4, "pairwise_method": method})
    d.aggregate_flat(ClientMatrix(data.to(cuda), P, [(P,)]), [1] * K)
    assert sorted(d.selected_clients + d.rejected_clients) == list(range(K))
    assert d.rejected_clients[-1] == bad and d.client_scores[bad] != d.client_scores[bad]
    Dh = d.distances.cpu().numpy()
    fin = [i for i in range(K) if i != bad]
    assert np.isfinite(Dh[np.ix_(fin, fin)]).all()
    scores = np.asarray(orc.krum_scores(Dh, K - f - 2))
    order = np.argsort(scores, kind="stable")
    assert d.selected_clients + d.rejected_clients == order.tolist()
    assert np.array_equal(np.asarray(d.client_scores)[fin], scores[fin])
    ref = np.asarray(orc.krum_scores(orc.distance_matrix([[X[k]] for k in range(K)]), K - f - 2))
    assert np.argsort(ref, kind="stable").tolist()[-1] == bad


def test_pairwise_large_offset_centering(cuda):
    # a large common component (weights, not deltas) must not cost accuracy
    K, P = 48, 50000
    X = update_matrix(K, P, f=0, seed=5, device=cuda)[:, :P] + 3.0
    D = ops.pairwise_l2(X).cpu().double()
    Xd = X.double().cpu()
    exact = torch.cdist(Xd, Xd)
    rel = ((D - exact).abs() / exact.clamp_min(1e-30)).fill_diagonal_(0)
    assert rel.max().item() < 5e-6


def test_pairwise_unaligned_rows(cuda):
    K, P = 9, 1001
    base = torch.randn(K * P + 1, device=cuda)
    X = base[1:].view(K, P)  # 4-B aligned only, ld = P (odd): the tail path does all of it
    D = ops.pairwise_l2(X).cpu().double()
    exact = torch.cdist(X.double().cpu(), X.double().cpu())
    assert ((D - exact).abs() / exact.clamp_min(1e-30)).fill_diagonal_(0).max().item() < 5e-6


# ---------------- selection ----------------

@pytest.mark.parametrize("path", golden_files("krum"), ids=lambda p: p.split("/")[-1])
def test_krum_select_bitexact_given_distances(cuda, path):
    fx = load_golden(path)
    D = torch.from_numpy(fx["dist"]).to(cuda)
    scores, order = ops.krum_select(D, int(fx["f"]))
    np.testing.assert_array_equal(scores.cpu().numpy(), fx["scores"])
    mk = int(fx["multi_k"])
    assert order.cpu().tolist()[:mk] == fx["selected"].tolist()


def test_krum_select_random_rows_bitexact(cuda):
    rng = np.random.default_rng(1)
    for K, f in [(5, 1), (50, 10), (128, 25), (257, 50), (512, 100)]:
        A = rng.random((K, K)) * 10
        D = np.triu(A, 1) + np.triu(A, 1).T
        scores = orc.krum_scores(D, K - f - 2)
        s, o = ops.krum_select(torch.from_numpy(D).to(cuda), f)
        np.testing.assert_array_equal(s.cpu().numpy(), np.asarray(scores))
        assert o.cpu().tolist() == np.argsort(scores, kind="stable").tolist()


def test_krum_rejects_small_n(cuda):
    with pytest.raises(ValueError):
        get_defense("krum", {"num_malicious": 2}).aggregate(
            [[torch.randn(4, device=cuda)] for _ in range(3)], [1] * 3)


# ---------------- end-to-end defenses vs golden ----------------

@pytest.mark.parametrize("path", golden_files("krum"), ids=lambda p: p.split("/")[-1])
def test_krum_defense_vs_golden(cuda, path):
    fx = load_golden(path)
    shapes = shapes_of(fx)
    X = torch.from_numpy(fx["X"]).to(cuda)
    ups = split_rows(X, X.shape[1], shapes)
    d = KrumDefense({"num_malicious": int(fx["f"]), "multi_k": int(fx["multi_k"])})
    agg = d.aggregate(ups, [100] * len(ups))
    assert d.selected_clients == fx["selected"].tolist()
    assert d.rejected_clients == fx["rejected"].tolist()
    flat = torch.cat([a.reshape(-1) for a in agg]).cpu().numpy()
    np.testing.assert_array_equal(flat, fx["agg"])  # same rows, same order -> bit-exact
    if int(fx["multi_k"]) == 1:
        assert agg is ups[d.selected_clients[0]]  # reference returns the caller's list


@pytest.mark.parametrize("path", golden_files("stat"), ids=lambda p: p.split("/")[-1])
def test_stat_defenses_vs_golden(cuda, path):
    fx = load_golden(path)
    shapes = shapes_of(fx)
    X = torch.from_numpy(fx["X"]).to(cuda)
    ups = split_rows(X, X.shape[1], shapes)
    cat = lambda lst: torch.cat([a.reshape(-1) for a in lst]).cpu().numpy()  # noqa: E731
    med = cat(get_defense("median", {}).aggregate(ups, []))
    np.testing.assert_array_equal(med, fx["median"])
    tmd = get_defense("trimmed_mean", {"trim_ratio": float(fx["trim_ratio"])})
    tm = cat(tmd.aggregate(ups, []))
    assert tmd.num_trimmed_per_end == int(fx["t"])
    np.testing.assert_allclose(tm, fx["trimmed"], rtol=1e-5, atol=1e-6)
    fa = cat(get_defense("fedavg", {}).aggregate(ups, fx["num_examples"].tolist()))
    np.testing.assert_array_equal(fa, fx["fedavg"])


@pytest.mark.parametrize("K", [2, 3, 5, 8, 9, 16, 31, 64, 100, 128, 129, 200, 255, 256, 300, 511, 512])
def test_order_stats_vs_torch(cuda, K):
    P = 5003
    X = torch.randn(K, P, device=cuda)
    X[0, :10] = float("inf")
    X[1 % K, 10:20] = -float("inf")
    ref_sorted = torch.sort(X.cpu(), dim=0)[0]
    np.testing.assert_array_equal(ops.median_lower(X).cpu().numpy(), torch.median(X.cpu(), dim=0)[0].numpy())
    t = max(1, int(K * 0.1))
    if K - 2 * t >= 1:
        Xf = X.clone()
        Xf[~torch.isfinite(Xf)] = 0.0
        ref = torch.sort(Xf.cpu(), dim=0)[0][t:K - t].mean(dim=0)
        got = ops.trimmed_mean(Xf, t).cpu()
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
        # bit-exact on the vectorised columns (all but the scalar tail), the
        # multi-lane path (K > 128) included: the cascade runs across its lanes
        ncol = (P // 64) * 64
        cas = orc.torch_outer_sum(torch.sort(Xf.cpu(), dim=0)[0][t:K - t]) / (K - 2 * t)
        assert torch.equal(got[:ncol], cas[:ncol])
    del ref_sorted


@pytest.mark.parametrize("K", [5, 16, 100, 128, 200, 256, 512])
def test_order_stats_nan_like_torch(cuda, K):
    """A Byzantine client sending NaN: torch.sort orders NaN last, torch.median
    returns NaN for a column with any NaN, and the trimmed mean is NaN only
    when more NaN than t survive the trim (trimmed_mean.py:74-101)."""
    P = 3001
    X = torch.randn(K, P, device=cuda)
    nan = float("nan")
    X[0, :700] = nan                      # one NaN per column: trimmed away when t >= 1
    X[1 % K, 100:200] = nan               # two NaN in these columns
    X[2 % K, 200:300] = float("inf")      # NaN / +inf ties
    X[3 % K, 300:400] = -nan              # negative-signed NaN sorts last too
    # K = 256 / 512 screen each lane's four 32-client quarters separately: NaN
    # in every quarter of some lane (client % 128 = 40, 100, 72, 44, 16, 127)
    for r in (40, 100, 200, 300, 400, K - 1):
        if r < K and r > 3:
            X[r, 500 + r % 97: 600 + r % 97] = nan
            X[r, 650:660] = nan
    t = max(1, int(K * 0.1))
    cpu = X.cpu()
    med_ref = torch.median(cpu, dim=0)[0]
    med = ops.median_lower(X).cpu()
    np.testing.assert_array_equal(med.numpy(), med_ref.numpy())  # NaN == NaN positions, bit-exact elsewhere
    if K - 2 * t >= 1:
        ref = torch.sort(cpu, dim=0)[0][t:K - t].mean(dim=0)
        got = ops.trimmed_mean(X, t).cpu()
        assert torch.equal(torch.isnan(got), torch.isnan(ref))
        fin = ~torch.isnan(ref)
        torch.testing.assert_close(got[fin], ref[fin], rtol=1e-5, atol=1e-6)


def test_trimmed_falls_back_to_median(cuda):
    ups = [[torch.randn(7, device=cuda)] for _ in range(3)]
    d = get_defense("trimmed_mean", {"trim_ratio": 0.5})
    out = d.aggregate(ups, [])
    ref = orc.median([[u[0].cpu()] for u in ups])[0]
    assert torch.equal(out[0].cpu(), ref)


def test_rows_mean_and_fedavg_bitexact(cuda):
    K, P = 37, 10007
    X = torch.randn(K, P, device=cuda)
    rows = torch.tensor([5, 3, 30, 0, 12], dtype=torch.int32)
    got = ops.rows_mean(X, rows, divisor=5).cpu()
    ups = [[X[i].cpu()] for i in range(K)]
    ref = sum(ups[i][0] for i in rows.tolist()) / 5
    assert torch.equal(got, ref)
    n = [int(v) for v in torch.randint(1, 100000, (K,))]
    assert torch.equal(ops.fedavg(X, n).cpu(), orc.fedavg(ups, n)[0])


@pytest.mark.parametrize("P", [4097, 4098, 4099, 11_800_394 // 100])
def test_rows_mean_fedavg_vector_path_with_tail(cuda, P):
    K = 9
    data = torch.zeros((K, padded_ld(P)), device=cuda)
    data[:, :P] = torch.randn(K, P, device=cuda)
    X = data[:, :P]
    rows = torch.tensor([4, 0, 7], dtype=torch.int32)
    ref = (0 + X[4].cpu() + X[0].cpu() + X[7].cpu()) / 3
    assert torch.equal(ops.rows_mean(X, rows).cpu(), ref)
    n = list(range(1, K + 1))
    assert torch.equal(ops.fedavg(X, n).cpu(), orc.fedavg([[X[i].cpu()] for i in range(K)], n)[0])


def test_client_matrix_zero_copy_defense(cuda):
    K, P = 20, 3000
    cm = ClientMatrix(update_matrix(K, P, f=4, device=cuda), P, [(P,)])
    d = get_defense("krum", {"num_malicious": 4, "multi_k": 10})
    out = d.aggregate(cm, [1] * K)
    assert out[0].shape == (P,)
    assert not set(d.selected_clients) & set(range(4))  # sign-flipped clients rejected


@pytest.mark.parametrize("K,m", [(40, 20), (200, 100), (512, 256), (300, 7), (512, 200), (600, 400), (512, 512)])
def test_order_stats_row_subset(cuda, K, m):
    P = 2049
    X = torch.randn(K, P, device=cuda)
    g = torch.Generator().manual_seed(K)
    rows = torch.randperm(K, generator=g)[:m].to(torch.int32)
    sub = X.cpu()[rows.long()]
    np.testing.assert_array_equal(ops.median_lower(X, rows=rows).cpu().numpy(),
                                  torch.median(sub, dim=0)[0].numpy())
    t = max(1, int(m * 0.1))
    if m - 2 * t >= 1:
        ref = torch.sort(sub, dim=0)[0][t:m - t].mean(dim=0)
        torch.testing.assert_close(ops.trimmed_mean(X, t, rows=rows).cpu(), ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("K,P", [(40, 4099), (128, 20_011), (512, 4099)])
def test_krum_trimmed_mean_vs_oracle(cuda, K, P):
    """Multi-Krum selection (krum.py:149-176) then the trimmed mean of the
    selected updates (trimmed_mean.py:63-90), both halves on the oracle."""
    f = int(0.2 * K)
    mk = K // 2
    X = update_matrix(K, P, f=f, seed=K, device=cuda)[:, :P]
    ups = [[X[i].cpu()] for i in range(K)]
    _, _, sel, rej, _ = orc.krum(ups, f, mk)
    want, t = orc.trimmed_mean([ups[i] for i in sel], 0.1)
    d = get_defense("krum_trimmed_mean", {"num_malicious": f, "multi_k": mk, "trim_ratio": 0.1})
    got = d.aggregate(ClientMatrix(update_matrix(K, P, f=f, seed=K, device=cuda), P, [(P,)]), [1] * K)
    assert d.selected_clients == sel and d.rejected_clients == rej
    assert d.num_trimmed_per_end == t
    torch.testing.assert_close(got[0].cpu(), want[0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("K,P,ranges,nneg,m", [
    (12, 4096 + 13, [(64, 512), (1024, 1000), (3000, 3)], 3, 6),
    (40, 70_001, [(1, 7), (100, 40_000), (60_000, 10_001)], 0, 17),
    (8, 1029, [(1024, 5)], 8, 8)])
def test_rows_mean_dead_ranges(cuda, K, P, ranges, nneg, m):
    """flr_rows_mean_dead (FLR_DEFER_DEAD=2): the dead ranges are NaN in X and
    come from the global vector (negated on rows < nneg) — bit-identical to
    flr_rows_mean over the filled rows, also in the float4 groups a range
    only partly covers and in the scalar tail; and the selected-row fill
    (ops.fill_dead_ranges) equals the filled row."""
    g = torch.Generator().manual_seed(K + P)
    ld = padded_ld(P)
    data = torch.zeros(K, ld)
    data[:, :P] = torch.randn(K, P, generator=g)
    gv = torch.randn(P, generator=g)
    filled, holes = data.clone(), data.clone()
    for o, n in ranges:
        filled[:, o:o + n] = gv[o:o + n]
        filled[:nneg, o:o + n] = -gv[o:o + n]
        holes[:, o:o + n] = float("nan")
    filled, holes, gvd = filled.to(cuda), holes.to(cuda), gv.to(cuda)
    rows = torch.randperm(K, generator=g)[:m].to(torch.int32).to(cuda)
    want = ops.rows_mean(filled[:, :P], rows, divisor=m + 1)
    got = ops.rows_mean(holes[:, :P], rows, divisor=m + 1, dead=(ranges, gvd, nneg))
    assert torch.isfinite(want).all() and torch.equal(got, want)
    for i in (0, K - 1):
        row = ops.fill_dead_ranges(holes[i, :P].clone(), ranges, gvd, i < nneg)
        assert torch.equal(row, filled[i, :P])
