"""GPU: BASELINE.json configs C3 / C4 / C5 at round level, against the oracle.

* C3 — the Krum indices of a TRAINED round (K = 128, batch 32, 5 local steps,
  P = 11,800,394, 25 sign-flip attackers) against the reference's own
  distances: fp32 ``torch.norm(fi - fj).item()`` per pair (krum.py:73-99,
  restated by oracle.aggregation.distance_matrix's op), its scores and
  ``np.argsort`` (krum.py:101-131, 174).  The selection boundary margin and the
  reference's own fp32 error against fp64 are asserted and written to a record
  (profiles/ keeps the committed copy).
* C4 — a K = 256 trimmed-mean round of the ViT-S/4 + BERT-mini model
  (trimmed_mean.py:48-90, run_experiments.py:188-259): sampled clients' rows
  against the oracle loop, the aggregate against oracle.trimmed_mean on a
  strided sample of > 1M coordinates.
* C5 — a K = 512 backdoor round (backdoor.py:253-290 on clients 0..101) with
  Multi-Krum then the trimmed mean of the selection (krum.py:133-192 +
  trimmed_mean.py:48-90): the GPU's distance matrix against fp64, the
  selection against the oracle's scores and argsort, the aggregate against
  the oracle's trimmed mean of the selected rows.
"""
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from oracle import aggregation as orc
from oracle import training as otrain
from flr import ops
from flr.matrix import padded_ld
from flr.models.multimodal import VIT_BERT, ModelSpec, model_class, param_layout
from parity import aggregate_report, check_delta, delta_report, tensor_sample
from flr.round import RoundConfig, RoundEngine
from flr.train import TrainConfig, make_dropout_masks, synthetic_batches

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _record(name: str, payload: dict) -> None:
    d = os.environ.get("FLR_RECORD_DIR", os.path.join(ROOT, "gpurun_out", "records"))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name), "w") as fh:
        json.dump(payload, fh, indent=1)
    print(f"\n[record {name}] " + json.dumps({k: v for k, v in payload.items() if not isinstance(v, list)}))


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def fp64_distances(X: torch.Tensor, P: int, chunk: int = 1 << 20) -> torch.Tensor:
    """K×K ℓ2 distances in fp64 on the device: the Gram matrix of the rows
    centred on row 0, accumulated over coordinate chunks in fp64 (cancellation
    costs at most ~1e-9 relative here)."""
    K = X.shape[0]
    G = torch.zeros(K, K, dtype=torch.float64, device=X.device)
    for c0 in range(0, P, chunk):
        c1 = min(P, c0 + chunk)
        y = X[:, c0:c1].double() - X[0:1, c0:c1].double()
        G += y @ y.T
        del y
    d = G.diagonal()
    return (d[:, None] + d[None, :] - 2.0 * G).clamp_min(0.0).sqrt().fill_diagonal_(0.0)


def reference_distances(rows, threads: int = 16) -> np.ndarray:
    """krum.py:89-97 on host rows: fp64 matrix of fp32 torch.norm(fi - fj).item().
    The pairs run on a thread pool with torch's intra-op pool at one thread; a
    single-output fp32 norm is one sequential reduction and the
    subtraction is elementwise, so the values are the reference's."""
    n = len(rows)
    out = np.zeros((n, n))
    prev = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        def row(a):
            return a, [torch.norm(rows[a] - rows[b]).item() for b in range(a + 1, n)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            for a, vals in ex.map(row, range(n)):
                for j, v in enumerate(vals):
                    out[a, a + 1 + j] = v
                    out[a + 1 + j, a] = v
                if a % 16 == 15:  # progress (a long host loop must not look hung)
                    print(f"[reference norms] rows 0..{a} done, {time.perf_counter() - t0:.1f} s", flush=True)
    finally:
        torch.set_num_threads(prev)
    return out


def _order_report(scores_a, scores_b, scores64, multi_k):
    """Compare two Krum orders (np.argsort of the two score vectors) given the
    fp64 scores: positions that differ must be swaps within the combined score
    error (ill-conditioned, both orders equally right)."""
    sa, sb, s64 = (np.asarray(s, dtype=np.float64) for s in (scores_a, scores_b, scores64))
    oa, ob = np.argsort(sa), np.argsort(sb)
    e = np.abs(sa - s64) + np.abs(sb - s64)  # per client: how far the two orders' scores can disagree
    diff = [int(r) for r in np.nonzero(oa != ob)[0]]
    ill = all(abs(s64[oa[r]] - s64[ob[r]]) <= e[oa[r]] + e[ob[r]] for r in diff)
    o64 = np.argsort(s64, kind="stable")
    s_sorted = s64[o64]
    out = {"order_a": oa, "order_b": ob, "positions_differing": diff, "differences_within_error": ill,
           "score_err_abs_max": float(e.max())}
    if multi_k < len(s64):
        lo, hi = o64[multi_k - 1], o64[multi_k]
        gap = float(s_sorted[multi_k] - s_sorted[multi_k - 1])
        out.update({"boundary_margin_rel": gap / float(s_sorted[multi_k]), "boundary_margin_abs": gap,
                    "boundary_score_err_abs": float(e[lo] + e[hi]),
                    "boundary_well_conditioned": bool(gap > e[lo] + e[hi])})
    gaps = np.diff(s_sorted) / s_sorted[1:]
    out.update({"min_adjacent_gap_rel": float(gaps.min()), "median_adjacent_gap_rel": float(np.median(gaps))})
    return out


@pytest.mark.timeout(900)
def test_c3_trained_round_krum_indices_vs_reference_norms(cuda):
    """C3 exactly as bench.py runs it (K = 128, B = 32, 5 local steps, full
    P; the default reference-exact distances over the training-order matrix):
    the engine's D is the reference's bit for bit — fp32 torch.norm distances
    of the trained (sign-flipped) rows in torch order — so its scores, selected
    and rejected lists are the reference's (krum.py:89-97, 126-129, 174).  The
    Gram path's D on the same rows is recorded beside it (selection equal where
    the scores are well conditioned)."""
    spec = ModelSpec()
    K, f, B, steps, mk = 128, 25, 32, 5, 64
    rc = RoundConfig(num_clients=K, batch=B, defense="krum", attack="sign_flip", num_attackers=f)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=steps), cuda)
    glob = eng.global_flat.clone().cpu()
    new = eng.run_round().clone().cpu()
    eng.defense.publish()
    eng.materialize()  # the client matrix whole (the dead-tap ranges, FLR_DEFER_DEAD)
    torch.cuda.synchronize()
    P = eng.trainer.P
    X = eng.trainer.X.data[:, :P]
    D_gpu = eng.defense.distances.double()
    D64 = fp64_distances(X, P)
    t0 = time.perf_counter()
    rows = []
    Xt = torch.zeros((K, padded_ld(P)), dtype=torch.float32, device=cuda)  # torch-order device copy
    for k in range(K):  # the reference's flattened updates: torch (parameters()) order
        r = eng.trainer.to_torch_order(X[k]) if eng.train_order else X[k]
        Xt[k, :P].copy_(r)
        rows.append(r.cpu())
    t_copy = time.perf_counter() - t0
    # the reference-exact mode on the torch-order copy (the engine read the
    # training-order matrix through its tap-major blocks), and the Gram path
    assert eng.defense.pairwise_method == "reference" and eng.train_order
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()  # the op's kernels run on torch's current stream
    D_mode = ops.pairwise_l2(Xt[:, :P], "reference")
    ev1.record()
    torch.cuda.synchronize()
    mode_ms = ev0.elapsed_time(ev1)
    D_gram = ops.pairwise_l2(Xt[:, :P], "gram").cpu().numpy()
    _, order_mode = ops.krum_select(D_mode, f)
    order_mode = order_mode.cpu().tolist()
    D_mode = D_mode.cpu().numpy()
    del Xt
    t0 = time.perf_counter()
    D_ref = reference_distances(rows)
    t_ref = time.perf_counter() - t0
    # the Multi-Krum mean of the reference's selection (krum.py:182-192: Python
    # sum of the selected rows in selection order, / multi_k), whole vector, per tensor
    order_ref0 = np.argsort(orc.krum_scores(D_ref, K - f - 2)).tolist()
    want = sum(rows[i] for i in order_ref0[:mk]) / mk
    agg_rep = aggregate_report(new, want, glob, param_layout(spec))
    del rows
    D64h = D64.cpu().numpy()
    off = ~np.eye(K, dtype=bool)
    err_ref = float(np.max(np.abs(D_ref - D64h)[off] / D64h[off]))
    err_gpu = float(np.max(np.abs(D_gpu.cpu().numpy() - D64h)[off] / D64h[off]))
    m = K - f - 2
    s_ref = orc.krum_scores(D_ref, m)
    s_gpu = orc.krum_scores(D_gpu.cpu().numpy(), m)
    s64 = orc.krum_scores(D64h, m)
    rep = _order_report(s_ref, s_gpu, s64, mk)
    order_ref = rep.pop("order_a").tolist()
    rep.pop("order_b")
    sel_ref, rej_ref = order_ref[:mk], order_ref[mk:]
    # the engine's published selection is its device order (krum.py:171-176)
    assert eng.defense.client_scores == pytest.approx(s_gpu, rel=1e-12)
    payload = {
        "config": "C3: K=128, f=25 sign-flip, multi_k=64, B=32, 5 local steps, P=11800394, one trained round",
        "torch": torch.__version__, "numpy": np.__version__,
        "distance_rel_err_reference_fp32_vs_fp64": err_ref, "distance_rel_err_gpu_vs_fp64": err_gpu,
        "selected_identical": eng.defense.selected_clients == sel_ref,
        "rejected_identical": eng.defense.rejected_clients == rej_ref,
        "selected_set_identical": set(eng.defense.selected_clients) == set(sel_ref),
        "attackers_selected": sorted(set(eng.defense.selected_clients) & set(range(f))),
        "host_copy_s": t_copy, "reference_norms_s": t_ref, **rep,
        "reference_mode_D_bit_identical": bool(np.array_equal(D_mode, D_ref)),
        "reference_mode_D_max_abs_diff": float(np.abs(D_mode - D_ref).max()),
        "reference_mode_selected_identical": order_mode[:mk] == sel_ref,
        "reference_mode_rejected_identical": order_mode[mk:] == rej_ref,
        "reference_mode_kernel_ms": mode_ms,
        "selected_reference": sel_ref, "selected_gpu": eng.defense.selected_clients,
        "engine_D_bit_identical": bool(np.array_equal(D_gpu.cpu().numpy(), D_ref)),
        "gram_distance_rel_err_vs_fp64": float(np.max(np.abs(D_gram - D64h)[off] / D64h[off])),
        "gram_selected_identical": np.argsort(np.asarray(orc.krum_scores(D_gram, m)))[:mk].tolist() == sel_ref,
        "aggregate_per_tensor": agg_rep, "aggregate_bit_identical": bool(torch.equal(new, want)),
    }
    _record("c3_krum_trained_round.json", payload)
    # the aggregate: every tensor's Δ_agg against the oracle's mean of the same rows
    check_delta({"aggregate": agg_rep})
    assert torch.equal(new, want)
    # the reference-exact mode: the reference's D bit for bit, so its whole order
    assert np.array_equal(D_mode, D_ref)
    assert order_mode[:mk] == sel_ref and order_mode[mk:] == rej_ref
    # the engine (the default reference-exact distances): D, scores and the
    # whole order are the reference's
    assert np.array_equal(D_gpu.cpu().numpy(), D_ref)
    assert eng.defense.client_scores == [float(v) for v in s_ref]
    assert eng.defense.selected_clients == sel_ref and eng.defense.rejected_clients == rej_ref
    assert not set(eng.defense.selected_clients) & set(range(f))


def _trimmed_cascade(sub: torch.Tensor, trim_ratio: float = 0.1):
    """trimmed_mean.py:63-90 on the sampled [n_rows, n] host matrix: torch.sort
    along the clients, rows [t, n_rows - t), summed in torch's vectorised
    outer-reduction order (oracle.aggregation.torch_outer_sum: every column of
    a real parameter but the last numel % 16, i.e. all but fc2.bias's 10 in
    both models) / R.  Returns (mean, t)."""
    n = sub.shape[0]
    t = max(1, int(n * trim_ratio))
    srt = torch.sort(sub, dim=0)[0][t:n - t]
    return orc.torch_outer_sum(srt) / (n - 2 * t), t


def _tail_param_report(eng, spec, new, rows, glob, name="fc2.bias"):
    """The scalar-tail parameter (numel % 16 columns torch reduces with its
    4-way row_sum instead of the vectorised cascade): the reference's own
    per-parameter trimmed mean (torch on the [n_rows, numel] stack) against
    the engine's, and against the vectorised order the engine restates."""
    off = 0
    for nm, shp in param_layout(spec):
        k = int(np.prod(shp))
        if nm == name:
            break
        off += k
    idx = torch.arange(off, off + k, dtype=torch.int64)
    sub = _sample_rows(eng, rows, idx)
    t = max(1, int(len(rows) * 0.1))
    ref_torch = torch.sort(sub, dim=0)[0][t:len(rows) - t].mean(dim=0)  # trimmed_mean.py:85-88, this parameter
    vec, _ = _trimmed_cascade(sub)
    got = new[idx.to(new.device)].cpu()
    d_gpu = (got - ref_torch).abs()
    d_vec = (vec - ref_torch).abs()
    return {"param": name, "coords": k, "engine_equals_vectorised_order": bool(torch.equal(got, vec)),
            "max_abs_engine_vs_torch": float(d_gpu.max()), "max_abs_vectorised_vs_torch": float(d_vec.max()),
            "max_delta_ref": float((ref_torch - glob[idx]).abs().max()), "ok": bool((d_gpu <= d_vec).all())}


def _sample_rows(eng, clients, idx: torch.Tensor) -> torch.Tensor:
    """[len(clients), len(idx)] host copy of the client rows' torch-order
    coordinates idx (one row converted at a time)."""
    eng.materialize()
    X = eng.trainer.X.data[:, : eng.trainer.P]
    di = idx.to(X.device)
    out = []
    for k in clients:
        r = eng.trainer.to_torch_order(X[k]) if eng.train_order else X[k]
        out.append(r[di].cpu())
    return torch.stack(out)


def _check_clients(eng, spec, glob, clients, batches_dev, masks_dev, negate=(), losses=False):
    """Sampled clients' rows vs the oracle loop: whole vector at 1e-5 and the
    per-tensor update report (tests/parity.py); returns the reports."""
    reps = {}
    eng.materialize()
    for k in clients:
        j = k - eng.lo
        cb = [(im[j].cpu(), tk[j].cpu(), lb[j].cpu()) for im, tk, lb in batches_dev]
        cm = None if masks_dev is None else [m[j].cpu() for m in masks_dev]
        upd, ref_loss = otrain.local_update(model_class(spec), spec, glob, cb, masks=cm)
        ref = torch.cat([u.reshape(-1) for u in upd])
        row = eng.trainer.X.data[j, : eng.trainer.P]
        row = eng.trainer.to_torch_order(row) if eng.train_order else row
        reps[f"client{k}"] = delta_report(-row if k in negate else row, ref, glob, param_layout(spec))
        if losses:
            got = eng.losses[j].item()
            reps[f"client{k}"]["loss_rel_err"] = abs(got - ref_loss) / max(1.0, abs(ref_loss))
            assert reps[f"client{k}"]["loss_rel_err"] <= 1e-5
        if k in negate:
            ref = -ref
        assert _rel(row.cpu(), ref) < 1e-5, (k, _rel(row.cpu(), ref))
    return reps


@pytest.mark.timeout(600)
def test_c4_round_trimmed_mean_vit_bert(cuda):
    """C4: trimmed mean (trim 0.1 -> t = 25 of 256) over K = 256 clients of
    ViT-S/4 + BERT-mini, 1 local step at batch 8."""
    spec = VIT_BERT
    K, B, steps = 256, 8, 1
    rc = RoundConfig(num_clients=K, batch=B, defense="trimmed_mean", defense_cfg={"trim_ratio": 0.1},
                     attack="none", num_attackers=0)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=steps), cuda)
    glob = eng.global_flat.clone().cpu()
    new = eng.run_round().clone()
    torch.cuda.synchronize()
    assert eng.defense.num_trimmed_per_end == 25
    reps = _check_clients(eng, spec, glob, [0, 77, 200, 255], eng.batches, eng.masks)
    _record("c4_update_parity_b8_1step.json", {"config": "C4 round, B=8, 1 step", **reps})
    check_delta(reps)
    P = eng.trainer.P
    idx, lay = tensor_sample(param_layout(spec))
    sub = _sample_rows(eng, range(K), idx)
    want, t = _trimmed_cascade(sub)
    assert t == 25
    got = new[idx.to(cuda)].cpu()
    agg_rep = aggregate_report(got, want, glob[idx], lay)
    tail = _tail_param_report(eng, spec, new, range(K), glob)
    _record("c4_trimmed_round.json", {"config": "C4: K=256 trimmed mean (t=25), ViT-S/4 + BERT-mini, B=8, 1 step",
                                      "P": P, "coords_checked": int(idx.numel()),
                                      "aggregate_rel_err": _rel(got, want), "aggregate_per_tensor": agg_rep,
                                      "tail_parameter": tail})
    # per tensor: Δ_agg within the bar of the oracle's aggregate of the same rows
    # (bit-identical expected: the same sort, torch's cascade order)
    check_delta({"aggregate": agg_rep})
    assert agg_rep["bit_identical_coords"] == agg_rep["coords"], agg_rep["bit_identical_coords"]
    assert tail["ok"], tail


@pytest.mark.timeout(900)
def test_c5_round_backdoor_krum_trimmed_mean(cuda):
    """C5: K = 512, backdoor on clients 0..101 (f = int(0.2 K)), Multi-Krum
    (multi_k = 256) then the trimmed mean (t = 25) of the selected rows."""
    spec = VIT_BERT
    K, B, steps = 512, 32, 1
    f = int(0.2 * K)
    rc = RoundConfig(num_clients=K, batch=B, defense="krum_trimmed_mean", defense_cfg={"trim_ratio": 0.1},
                     attack="backdoor", num_attackers=f)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=steps), cuda)
    # the attackers' data is poisoned (backdoor.py:253-290), the benign clients' is not
    clean = synthetic_batches(spec, steps, [0, 101, 102, 511], B, cuda)
    for j, k in enumerate([0, 101, 102, 511]):
        same = all(torch.equal(c[0][j], e[0][k]) and torch.equal(c[2][j], e[2][k])
                   for c, e in zip(clean, eng.batches))
        assert same == (k >= f), k
    glob = eng.global_flat.clone().cpu()
    new = eng.run_round().clone()
    eng.defense.publish()
    torch.cuda.synchronize()
    reps = _check_clients(eng, spec, glob, [0, 101, 102, 511], eng.batches, eng.masks)
    _record("c5_update_parity_b32_1step.json", {"config": "C5 round, B=32, 1 step (backdoor clients 0, 101)",
                                                **reps})
    check_delta(reps)
    P = eng.trainer.P
    X = eng.trainer.X.data[:, :P]
    D_gpu = eng.defense.distances.double()
    D64 = fp64_distances(X, P)
    off = ~torch.eye(K, dtype=torch.bool, device=cuda)
    dist_err = ((D_gpu - D64).abs()[off] / D64[off]).max().item()
    # the default reference-exact distances: sampled pairs bit-identical to the
    # reference's fp32 torch.norm accumulation (oracle/norm_ref.c) of the
    # torch-order rows; the whole D within the reference's own fp32 error of fp64
    assert eng.defense.pairwise_method == "reference"
    from oracle import normref
    Dh = D_gpu.cpu().numpy()

    def torch_row(k):
        return (eng.trainer.to_torch_order(X[k]) if eng.train_order else X[k]).cpu().numpy()
    # two whole rows of D (an attacker's and a benign client's: 2 x 511 pairs)
    # against the reference's fp32 accumulation (oracle/norm_ref.c), bit for bit
    t0 = time.perf_counter()
    row_pairs = 0
    for i in (0, 300):
        ri = torch_row(i)
        for c0 in range(0, K, 32):
            js = [j for j in range(c0, min(K, c0 + 32)) if j != i]
            rj = {j: torch_row(j) for j in js}
            with ThreadPoolExecutor(16) as ex:
                vals = list(ex.map(lambda j: normref.norm_diff(ri, rj[j]), js))
            for j, v in zip(js, vals):
                assert Dh[i, j] == v and Dh[j, i] == v, (i, j, Dh[i, j], v)
            row_pairs += len(js)
            del rj
        print(f"[D row {i}] {K - 1} pairs bit-identical, {time.perf_counter() - t0:.1f} s", flush=True)
    del ri
    assert dist_err < 1e-2, dist_err
    m, mk = K - f - 2, K // 2
    s_gpu = orc.krum_scores(D_gpu.cpu().numpy(), m)
    s64 = orc.krum_scores(D64.cpu().numpy(), m)
    order = np.argsort(s_gpu, kind="stable")
    assert eng.defense.selected_clients == order[:mk].tolist()
    rep = _order_report(s_gpu, s64, s64, mk)
    rep.pop("order_a"), rep.pop("order_b")
    sel = eng.defense.selected_clients
    idx, lay = tensor_sample(param_layout(spec))
    sub = _sample_rows(eng, sel, idx)  # in selection (score) order, as the reference stacks them
    want, t = _trimmed_cascade(sub)
    assert t == eng.defense.num_trimmed_per_end == 25
    got = new[idx.to(cuda)].cpu()
    agg_rep = aggregate_report(got, want, glob[idx], lay)
    tail = _tail_param_report(eng, spec, new, sel, glob)
    _record("c5_backdoor_round.json", {
        "config": "C5: K=512, backdoor clients 0..101, Multi-Krum (multi_k=256) + trimmed mean (t=25), "
                  "ViT-S/4 + BERT-mini, B=32, 1 step",
        "P": P, "distance_rel_err_gpu_vs_fp64": dist_err, "D_pairs_bit_identical_to_reference": row_pairs,
        "coords_checked": int(idx.numel()), "aggregate_rel_err": _rel(got, want),
        "aggregate_per_tensor": agg_rep, "tail_parameter": tail,
        "backdoor_clients_selected": sorted(set(sel) & set(range(f))), **rep})
    check_delta({"aggregate": agg_rep})
    assert agg_rep["bit_identical_coords"] == agg_rep["coords"], agg_rep["bit_identical_coords"]
    assert tail["ok"], tail


@pytest.mark.timeout(900)
def test_c4_round_bench_shape_update_parity(cuda):
    """C4 at the bench's own training shape (B = 32, 5 local steps, K = 256
    trimmed mean, ViT-S/4 + BERT-mini): two sampled clients' updates per
    tensor and their losses against the oracle loop (run_experiments.py:
    206-238), and the aggregate against oracle.trimmed_mean on a strided
    sample."""
    spec = VIT_BERT
    K, B, steps = 256, 32, 5
    rc = RoundConfig(num_clients=K, batch=B, defense="trimmed_mean", defense_cfg={"trim_ratio": 0.1},
                     attack="none", num_attackers=0)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=steps), cuda)
    glob = eng.global_flat.clone().cpu()
    new = eng.run_round().clone()
    torch.cuda.synchronize()
    reps = _check_clients(eng, spec, glob, [3, 250], eng.batches, eng.masks, losses=True)
    idx, lay = tensor_sample(param_layout(spec), 2048)
    sub = _sample_rows(eng, range(K), idx)
    want, t = _trimmed_cascade(sub)
    got = new[idx.to(cuda)].cpu()
    agg_rep = aggregate_report(got, want, glob[idx], lay)
    _record("c4_update_parity_bench_shape.json", {"config": "C4 round at the bench shape: K=256 trimmed mean, "
                                                            "ViT-S/4 + BERT-mini, B=32, 5 local steps",
                                                  "aggregate_rel_err": _rel(got, want),
                                                  "aggregate_per_tensor": agg_rep, **reps})
    check_delta(reps)
    check_delta({"aggregate": agg_rep})
    assert agg_rep["bit_identical_coords"] == agg_rep["coords"], agg_rep["bit_identical_coords"]
