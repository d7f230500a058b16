"""CPU: pin the oracle — reference property tests restated, op semantics, golden vectors."""
import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden, shapes_of
from oracle import aggregation as orc
from flr.workload import split_rows


def mock_updates(n, shapes=((10, 10), (10,)), seed=0):
    g = torch.Generator().manual_seed(seed)
    return [[torch.randn(s, generator=g) for s in shapes] for _ in range(n)]


# ---- tests/test_defenses.py of the reference, restated against the oracle ----

def test_ref_single_krum():  # test_defenses.py:40-52
    ups = mock_updates(5)
    agg, scores, sel, rej, _ = orc.krum(ups, 1, 1)
    assert len(agg) == len(ups[0]) and len(sel) == 1


def test_ref_multi_krum():  # :54-63
    agg, _, sel, _, _ = orc.krum(mock_updates(5), 1, 2)
    assert len(agg) == 2 and len(sel) == 2


def test_ref_malicious_detection():  # :65-81
    g = torch.Generator().manual_seed(3)
    ups = [[torch.zeros(10, 10) + torch.randn(10, 10, generator=g) * 0.01] for _ in range(4)]
    ups.append([torch.randn(10, 10, generator=g) * 100])
    _, _, sel, _, _ = orc.krum(ups, 1, 1)
    assert 4 not in sel


def test_ref_insufficient_clients():  # :83-91
    with pytest.raises(ValueError):
        orc.krum(mock_updates(3), 2, 1)


def test_ref_trimmed_outliers():  # :112-129
    base = torch.zeros(10)
    ups = [[base + 0.1], [base + 0.2], [base], [base + 100], [base - 100]]
    agg, t = orc.trimmed_mean(ups, 0.2)
    assert t == 1 and agg[0].abs().mean() < 1.0


def test_ref_median_outlier():  # :145-160
    ups = [[torch.tensor([1.0, 1.0])], [torch.tensor([1.1, 0.9])], [torch.tensor([0.9, 1.1])],
           [torch.tensor([100.0, 100.0])], [torch.tensor([1.0, 1.0])]]
    assert torch.allclose(orc.median(ups)[0], torch.tensor([1.0, 1.0]), atol=0.2)


def test_ref_lower_median_even():  # torch.median(dim=0) is the lower median
    ups = [[torch.tensor([float(v)])] for v in (4, 1, 3, 2)]
    assert orc.median(ups)[0].item() == 2.0


def test_sign_flip_negates():  # model_poisoning.py:274-276
    u = [torch.ones(3), -2 * torch.ones(2)]
    assert all(torch.equal(a, -b) for a, b in zip(orc.sign_flip(u), u))


# ---- op semantics restated by the kernels ----

@pytest.mark.parametrize("n", [0, 1, 5, 7, 8, 9, 63, 64, 101, 127, 128, 129, 200, 255, 511, 1000])
def test_numpy_pairwise_sum_exact(n):
    a = np.random.default_rng(n).standard_normal(n) * 10
    assert orc.numpy_pairwise_sum(a) == np.sum(a) or (n == 0 and np.sum(a) == 0)
    assert 0.0 + orc.numpy_pairwise_sum(a) == np.sum(a)


@pytest.mark.parametrize("R", [1, 5, 15, 16, 17, 33, 104, 206, 300])
def test_torch_outer_sum_cascade(R):
    x = torch.randn(R, 4096, generator=torch.Generator().manual_seed(R))
    got = orc.torch_outer_sum(x)
    ref = x.sum(dim=0)
    assert torch.equal(got, ref)
    assert torch.equal(x.mean(dim=0), ref / R)


def test_scalar_division_is_ieee():
    x = torch.randn(100003)
    for k in (3, 7, 64, 101):
        assert torch.equal(x / k, (x.double() / k).float())


# ---- golden fixtures reproduce ----

@pytest.mark.parametrize("path", golden_files("krum"), ids=lambda p: p.split("/")[-1])
def test_golden_krum_reproduces(path):
    fx = load_golden(path)
    shapes = shapes_of(fx)
    X = torch.from_numpy(fx["X"])
    ups = split_rows(X, X.shape[1], shapes)
    agg, scores, sel, rej, dist = orc.krum(ups, int(fx["f"]), int(fx["multi_k"]))
    assert sel == fx["selected"].tolist() and rej == fx["rejected"].tolist()
    np.testing.assert_array_equal(np.asarray(scores), fx["scores"])
    np.testing.assert_array_equal(dist, fx["dist"])
    flat = torch.cat([a.reshape(-1) for a in agg]).numpy()
    np.testing.assert_array_equal(flat, fx["agg"])


@pytest.mark.parametrize("path", golden_files("stat"), ids=lambda p: p.split("/")[-1])
def test_golden_stats_reproduce(path):
    fx = load_golden(path)
    shapes = shapes_of(fx)
    X = torch.from_numpy(fx["X"])
    ups = split_rows(X, X.shape[1], shapes)
    tm, t = orc.trimmed_mean(ups, float(fx["trim_ratio"]))
    assert t == int(fx["t"])
    cat = lambda lst: torch.cat([a.reshape(-1) for a in lst]).numpy()  # noqa: E731
    np.testing.assert_array_equal(cat(tm), fx["trimmed"])
    np.testing.assert_array_equal(cat(orc.median(ups)), fx["median"])
    np.testing.assert_array_equal(cat(orc.fedavg(ups, fx["num_examples"].tolist())), fx["fedavg"])


@pytest.mark.parametrize("path", golden_files("c3krum"), ids=lambda p: p.split("/")[-1])
def test_golden_c3_krum_regenerates(path):
    """The C3-shaped fixtures store the seed, not X: the CPU generator must
    reproduce X exactly (checksums), and — at the smaller P — the oracle must
    reproduce the stored distances, scores and selection bit for bit."""
    import hashlib
    from flr.workload import update_matrix
    fx = load_golden(path)
    K, P, f, mk = (int(fx[k]) for k in ("K", "P", "f", "multi_k"))
    X = update_matrix(K, P, f=f, seed=int(fx["seed"]), device="cpu")[:, :P].contiguous()
    Xd = X.double()
    assert float(Xd.sum()) == float(fx["x_sum"]) and float((Xd * Xd).sum()) == float(fx["x_sumsq"])
    # selection from the stored D (krum.py:101-131, 174)
    scores = orc.krum_scores(fx["dist"], K - f - 2)
    np.testing.assert_array_equal(np.asarray(scores), fx["scores"])
    order = np.argsort(scores)
    assert order[:mk].tolist() == fx["selected"].tolist() and order[mk:].tolist() == fx["rejected"].tolist()
    assert not set(fx["selected"].tolist()) & set(range(f))  # every sign-flipped client rejected
    if P < 100_000:
        agg, sc, sel, rej, dist = orc.krum(split_rows(X, P, [(P,)]), f, mk)
        np.testing.assert_array_equal(dist, fx["dist"])
        assert sel == fx["selected"].tolist()
        flat = torch.cat([a.reshape(-1) for a in agg]).numpy()
        assert hashlib.sha256(flat.tobytes()).hexdigest() == str(fx["agg_sha256"])


def test_golden_krum_margins_recorded():
    for path in golden_files("krum"):
        fx = load_golden(path)
        assert float(fx["margin"]) > 0  # no exact tie at the selection boundary


# ---- the reference's per-pair norm (krum.py:95) restated in C (oracle/norm_ref.c) ----

@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 63, 1000, 4099, 65537, 1 << 20, 3_000_001])
def test_norm_ref_model_equals_torch_norm(n):
    """SURVEY App. C's accumulation model of fp32 torch.norm (8 sequential-fma
    lanes, lanes summed in order, tail mul + add, sqrt_f32) reproduces
    torch.norm(a - b).item() bit for bit, at every length and magnitude mix
    (several seeds per length; the heavy-tailed cases make order matter)."""
    from oracle import normref
    for seed in range(6):
        g = torch.Generator().manual_seed(1000 * n + seed)
        a = torch.randn(n, generator=g) * (10.0 ** (seed - 3))
        b = a + torch.randn(n, generator=g) * 1e-3 * torch.exp(2 * torch.randn(n, generator=g))
        want = torch.norm(a - b).item()
        got = normref.norm_diff(a.numpy(), b.numpy())
        assert got == want, (n, seed, got, want)


@pytest.mark.parametrize("n", list(range(1, 17)) + [20, 23, 100, 1001, 4099])
def test_norm_ref_model_tail_lengths(n):
    """The P mod 8 tail (every length 0..7 after 0..N full 8-lane steps), 200
    seeds each: a 4-element group as separate multiply + add, the rest fma."""
    from oracle import normref
    for seed in range(200):
        g = torch.Generator().manual_seed(n * 1000 + seed)
        a = torch.randn(n, generator=g) * 3
        b = torch.randn(n, generator=g)
        assert normref.norm_diff(a.numpy(), b.numpy()) == torch.norm(a - b).item(), (n, seed)


def test_norm_ref_model_thread_independent():
    """A single-output fp32 norm is one sequential reduction whatever the
    intra-op thread count (C3's P = 11,800,394)."""
    from oracle import normref
    g = torch.Generator().manual_seed(5)
    n = 11_800_394
    a = torch.randn(n, generator=g) * 0.05
    b = a + 0.01 * torch.randn(n, generator=g)
    got = normref.norm_diff(a.numpy(), b.numpy())
    prev = torch.get_num_threads()
    try:
        for th in (1, max(2, prev)):
            torch.set_num_threads(th)
            assert torch.norm(a - b).item() == got
    finally:
        torch.set_num_threads(prev)


def test_norm_ref_distance_matrix_equals_oracle():
    """The OpenMP pair matrix == oracle.aggregation.distance_matrix (torch.norm per pair)."""
    from oracle import normref
    g = torch.Generator().manual_seed(9)
    X = torch.randn(9, 3001, generator=g)
    X[:3] = -X[:3]
    want = orc.distance_matrix([[X[k]] for k in range(9)])
    assert np.array_equal(normref.distance_matrix(X.numpy()), want)


_CAP_SCRIPT = r"""
import sys, json, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from oracle import normref
g = np.random.default_rng(5)
bad = 0
for n in (7, 8, 15, 16, 17, 31, 33, 100, 1023, 4101, 100003, 1 << 20):
    for t in range(4):
        a = g.standard_normal(n).astype(np.float32) * np.float32(10.0 ** g.uniform(-3, 3))
        b = g.standard_normal(n).astype(np.float32)
        bad += torch.norm(torch.from_numpy(a) - torch.from_numpy(b)).item() != normref.norm_diff(a, b)
print(json.dumps({"capability": torch.backends.cpu.get_cpu_capability(), "mismatches": int(bad)}))
"""


@pytest.mark.parametrize("cap", [None, "avx2", "avx512"])
def test_norm_ref_model_cpu_capability(cap):
    """the 8-lane accumulation is ATen's Vectorized<float> width on
    the AVX2 path; pinned here under each SIMD dispatch this torch offers
    (ATEN_CPU_CAPABILITY), the capability recorded: the same bits on AVX2 and
    AVX512 (this container reports AVX512 by default, the GPU boxes' EPYC 9575F
    too).  A capability whose torch.norm differed would fail here."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    if cap:
        env["ATEN_CPU_CAPABILITY"] = cap
    out = subprocess.run([sys.executable, "-c", _CAP_SCRIPT, root], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    print(f"\n[torch.norm capability] requested {cap}: {rec}")
    if cap:
        assert rec["capability"].lower() == cap
    assert rec["mismatches"] == 0, rec


def test_relu_ties_resolve_only_the_given_gates():
    """oracle.training relu_ties (the gate-tie resolution of the step-2 parity
    check): the reference's own decisions given back leave the step bit-identical;
    one decision forced the other way changes it; relu_inputs reads the inputs."""
    from oracle import training as otrain
    from flr.models.multimodal import TINY, MultimodalNet, param_layout
    torch.manual_seed(0)
    P = sum(int(np.prod(s)) for _, s in param_layout(TINY))
    glob = torch.randn(P) * 0.1
    im = torch.randn(4, TINY.in_channels, 32, 32)
    tk = torch.randint(0, TINY.vocab, (4, TINY.seq_len))
    lb = torch.randint(0, TINY.num_classes, (4,))
    cb = [(im, tk, lb)]
    base, _ = otrain.local_update(MultimodalNet, TINY, glob, cb)
    z = otrain.relu_inputs(MultimodalNet, TINY, glob, im, tk)
    assert len(z) >= 2 and z[1].dim() == 4
    idx = torch.arange(0, z[1].numel(), 7)
    same, _ = otrain.local_update(MultimodalNet, TINY, glob, cb, relu_ties={1: (idx, z[1].reshape(-1)[idx] > 0)})
    assert all(torch.equal(a, b) for a, b in zip(base, same))
    j = int((z[1].reshape(-1) > 0).nonzero()[0])
    off, _ = otrain.local_update(MultimodalNet, TINY, glob, cb, relu_ties={1: (torch.tensor([j]), torch.tensor([False]))})
    assert not all(torch.equal(a, b) for a, b in zip(base, off))
