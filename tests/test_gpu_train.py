"""GPU parity of local training: the client-batched engine vs the oracle's
per-client reference loop (run_experiments.py:195-240), training loss and
trained parameters within 1e-5 (north_star)."""
import pytest
import torch

from parity import check_conditioned, check_delta, conditioned_report, delta_report, record

from oracle import training as otrain
from flr.client import Client
from flr.models.multimodal import CUB, TINY, ModelSpec, MultimodalNet, model_class, num_params, param_layout
from flr.round import initial_global
from flr.train import ClientBatchTrainer, TrainConfig, make_dropout_masks, synthetic_batches

pytestmark = pytest.mark.gpu

SPEC = TINY
SPEC_DROP = ModelSpec(widths=(8, 16, 16, 32), blocks=(1, 1, 1, 1), vocab=50, embed=8, hidden=16, fusion=16,
                      dropout=0.5)
# channel counts that put every non-stem conv on the tap-major kernels
SPEC_WIDE = ModelSpec(widths=(64, 64, 128, 128), blocks=(1, 1, 1, 1), vocab=50, embed=8, hidden=16, fusion=16,
                      dropout=0.0)


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("spec", [SPEC, SPEC_DROP, SPEC_WIDE], ids=["p0", "dropout-masks", "tap-major"])
def test_batched_training_matches_reference_loop(cuda, spec):
    K, B, steps = 3, 8, 3
    glob = initial_global(spec, 42, cuda)
    tr = ClientBatchTrainer(spec, K, cuda, TrainConfig(local_steps=steps))
    batches = synthetic_batches(spec, steps, range(K), B, cuda)
    masks = make_dropout_masks(spec, steps, K, B, cuda, seed=3)
    tr.load_global(glob)
    loss = tr.local_update(batches, masks).cpu()
    for k in range(K):
        cb = [(im[k].cpu(), tk[k].cpu(), lb[k].cpu()) for im, tk, lb in batches]
        cm = None if masks is None else [m[k].cpu() for m in masks]
        upd, ref_loss = otrain.local_update(MultimodalNet, spec, glob.cpu(), cb, masks=cm)
        ref = torch.cat([u.reshape(-1) for u in upd])
        got = tr.X.data[k, : tr.P].cpu()
        assert abs(loss[k].item() - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
        assert _rel(got, ref) < 1e-5, _rel(got, ref)


def test_client_api_mirror(cuda):
    spec = SPEC
    glob = initial_global(spec, 42, cuda)
    batches = [(im[0], tk[0], lb[0]) for im, tk, lb in synthetic_batches(spec, 2, [7], 8, cuda)]
    c = Client(7, batches, spec, cuda)
    shapes = [p.shape for p in MultimodalNet(spec).parameters()]
    parts, off = [], 0
    for s in shapes:
        n = int(torch.Size(s).numel())
        parts.append(glob[off:off + n].view(s))
        off += n
    params, n, metrics = c.local_update(parts, {"local_epochs": 1, "learning_rate": 0.01})
    assert n == 16 and metrics["client_id"] == 7 and isinstance(metrics["loss"], float)
    assert [p.shape for p in params] == shapes
    cpu_b = [(a.cpu(), b.cpu(), y.cpu()) for a, b, y in batches]
    upd, ref_loss = otrain.fl_client_train(MultimodalNet, spec, glob.cpu(), cpu_b)  # fl_client.py:109-149, no clip
    assert abs(metrics["loss"] - ref_loss) < 1e-5
    ref = torch.cat([u.reshape(-1) for u in upd])
    got = torch.cat([p.reshape(-1) for p in params]).cpu()
    assert _rel(got, ref) < 1e-5, _rel(got, ref)
    nd, _, _ = c.fit([p.cpu().numpy() for p in parts], {})
    assert len(nd) == len(shapes)
    # clip = 1.0: the simulation loop's clip_grad_norm_ (run_experiments.py:234)
    c1 = Client(7, batches, spec, cuda, clip=1.0, learning_rate=0.5)
    params1, _, m1 = c1.local_update(parts, {"local_epochs": 1})
    upd1, loss1 = otrain.local_update(MultimodalNet, spec, glob.cpu(), cpu_b, lr=0.5, max_norm=1.0)
    assert abs(m1["loss"] - loss1) < 1e-5
    ref1 = torch.cat([u.reshape(-1) for u in upd1])
    assert _rel(torch.cat([p.reshape(-1) for p in params1]).cpu(), ref1) < 1e-5


def test_full_model_single_step_runs(cuda):
    spec = ModelSpec()
    assert num_params(spec) == 11_800_394
    tr = ClientBatchTrainer(spec, 2, cuda, TrainConfig(local_steps=1))
    tr.load_global(initial_global(spec, 42, cuda))
    b = synthetic_batches(spec, 1, [0, 1], 4, cuda)
    loss = tr.local_update(b, make_dropout_masks(spec, 1, 2, 4, cuda, 1))
    assert torch.isfinite(loss).all()


def test_full_model_matches_reference_loop(cuda):
    """The C3 model itself (every ResNet-18 layer shape: tap-major convs, dead
    taps at 1x1, split-K) for 2 clients x 2 steps vs the oracle loop."""
    spec = ModelSpec()
    K, B, steps = 2, 4, 2
    glob = initial_global(spec, 42, cuda)
    tr = ClientBatchTrainer(spec, K, cuda, TrainConfig(local_steps=steps))
    assert len(tr.tap_major) == 19  # all convs but the 7x7 stem
    batches = synthetic_batches(spec, steps, range(K), B, cuda)
    masks = make_dropout_masks(spec, steps, K, B, cuda, seed=5)
    tr.load_global(glob)
    loss = tr.local_update(batches, masks).cpu()
    for k in range(K):
        cb = [(im[k].cpu(), tk[k].cpu(), lb[k].cpu()) for im, tk, lb in batches]
        upd, ref_loss = otrain.local_update(MultimodalNet, spec, glob.cpu(), cb, masks=[m[k].cpu() for m in masks])
        ref = torch.cat([u.reshape(-1) for u in upd])
        got = tr.X.data[k, : tr.P].cpu()
        assert abs(loss[k].item() - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
        assert _rel(got, ref) < 1e-5, _rel(got, ref)


def test_layout_kernels(cuda):
    """flr_broadcast_rows / flr_copy_rows / flr_tap_major_to_torch on odd sizes
    and unaligned bases (scalar paths) as well as aligned ones."""
    from flr import _capi
    from flr.models.multimodal import to_tap_major
    st = torch.cuda.current_stream().cuda_stream
    for n, off in [(7, 0), (1000, 0), (1001, 1), (64, 3)]:
        src = torch.randn(n + off, device=cuda)[off:]
        dst = torch.full((5, n + 9), -1.0, device=cuda)
        _capi.call("flr_broadcast_rows", src.data_ptr(), n, dst.data_ptr() + 4 * off, 5, n + 9, st)
        assert torch.equal(dst[:, off:off + n], src.expand(5, n))
        out = torch.zeros(5, n + 9 + off, device=cuda)
        _capi.call("flr_copy_rows", dst.data_ptr(), n + 9, n + 9, out.data_ptr(), n + 9 + off, 5, st)
        assert torch.equal(out[:, : n + 9], dst)
    for K, cout, cin, k in [(3, 64, 64, 3), (2, 70, 20, 3), (2, 128, 64, 1), (1, 5, 3, 2)]:
        w = torch.randn(K, cout, cin, k, k, device=cuda)
        wt = to_tap_major(w).contiguous()
        n = cout * cin * k * k
        X = torch.zeros(K, n + 13, device=cuda)
        _capi.call("flr_tap_major_to_torch", wt.data_ptr(), K, k * k, cin, cout, X.data_ptr() + 4 * 5, n + 13, st)
        assert torch.equal(X[:, 5:5 + n], w.reshape(K, n))


def test_cub_c1_model_matches_reference_loop(cuda):
    """Config C1's model — the reference's CUB200MultimodalCNN structure (conv
    blocks with bias, attribute MLP over the multi-hot text, fusion head with
    dropout masks) — with the cub200 optimizer (weight decay 1e-4,
    run_experiments.py:210), 3 clients x 3 steps vs the oracle loop."""
    spec = CUB
    K, B, steps = 3, 8, 3
    glob = initial_global(spec, 42, cuda)
    tr = ClientBatchTrainer(spec, K, cuda, TrainConfig(local_steps=steps, weight_decay=1e-4))
    assert tr.tap_major == {"image_conv.8.weight"}  # 64 -> 128: the tap-major kernels
    batches = synthetic_batches(spec, steps, range(K), B, cuda)
    masks = make_dropout_masks(spec, steps, K, B, cuda, seed=9)
    tr.load_global(glob)
    loss = tr.local_update(batches, masks).cpu()
    for k in range(K):
        cb = [(im[k].cpu(), tx[k].cpu(), lb[k].cpu()) for im, tx, lb in batches]
        upd, ref_loss = otrain.local_update(model_class(spec), spec, glob.cpu(), cb, weight_decay=1e-4,
                                            masks=[m[k].cpu() for m in masks])
        ref = torch.cat([u.reshape(-1) for u in upd])
        got = tr.X.data[k, : tr.P].cpu()
        assert abs(loss[k].item() - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
        assert _rel(got, ref) < 1e-5, _rel(got, ref)


def test_c1_round_fedavg_matches_reference(cuda):
    """Config C1 end to end: K = 4 clients, 2 local steps, FedAvg write-back
    (run_experiments.py:193-259) on the engine vs the oracle's per-client loop
    + FedAvg (base_defense.py:80-97)."""
    from oracle import aggregation as orc
    from flr.round import RoundConfig, RoundEngine
    spec = CUB
    K, steps, B = 4, 2, 8
    rc = RoundConfig(num_clients=K, batch=B, defense="fedavg", attack="none", num_attackers=0)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=steps, weight_decay=1e-4), cuda)
    glob = eng.global_flat.clone().cpu()
    new = eng.run_round().cpu()
    batches = synthetic_batches(spec, steps, range(K), B, "cpu")
    masks = make_dropout_masks(spec, steps, range(K), B, "cpu", seed=rc.seed + 7919)
    ups = []
    for k in range(K):
        cb = [(im[k], tx[k], lb[k]) for im, tx, lb in batches]
        upd, _ = otrain.local_update(model_class(spec), spec, glob, cb, weight_decay=1e-4,
                                     masks=[m[k] for m in masks])
        ups.append(upd)
    ref = torch.cat([t.reshape(-1) for t in orc.fedavg(ups, [steps * B] * K)])
    assert _rel(new, ref) < 1e-5, _rel(new, ref)


def test_vit_bert_tiny_matches_reference_loop(cuda):
    """The C4/C5 family (ViT + BERT encoders, every kernel of train_xfmr.hip
    and the fused GEMM epilogues) at test size: 3 clients x 3 steps with
    dropout masks vs the oracle loop on one ViTBertNet per client."""
    from flr.models.multimodal import VIT_BERT_TINY
    spec = VIT_BERT_TINY.__class__(**{**VIT_BERT_TINY.__dict__, "dropout": 0.5})
    K, B, steps = 3, 8, 3
    glob = initial_global(spec, 42, cuda)
    tr = ClientBatchTrainer(spec, K, cuda, TrainConfig(local_steps=steps))
    batches = synthetic_batches(spec, steps, range(K), B, cuda)
    masks = make_dropout_masks(spec, steps, K, B, cuda, seed=4)
    tr.load_global(glob)
    loss = tr.local_update(batches, masks).cpu()
    for k in range(K):
        cb = [(im[k].cpu(), tk[k].cpu(), lb[k].cpu()) for im, tk, lb in batches]
        upd, ref_loss = otrain.local_update(model_class(spec), spec, glob.cpu(), cb, masks=[m[k].cpu() for m in masks])
        ref = torch.cat([u.reshape(-1) for u in upd])
        got = tr.X.data[k, : tr.P].cpu()
        assert abs(loss[k].item() - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
        assert _rel(got, ref) < 1e-5, _rel(got, ref)


def test_vit_bert_full_model_matches_reference_loop(cuda):
    """The C4/C5 model itself (ViT-S/4 + BERT-mini, P = 32,675,722): 2 clients
    x 2 steps vs the oracle loop."""
    from flr.models.multimodal import VIT_BERT
    spec = VIT_BERT
    assert num_params(spec) == 32_675_722
    K, B, steps = 2, 4, 2
    glob = initial_global(spec, 42, cuda)
    tr = ClientBatchTrainer(spec, K, cuda, TrainConfig(local_steps=steps))
    batches = synthetic_batches(spec, steps, range(K), B, cuda)
    masks = make_dropout_masks(spec, steps, K, B, cuda, seed=6)
    tr.load_global(glob)
    loss = tr.local_update(batches, masks).cpu()
    assert torch.isfinite(loss).all()
    for k in range(K):
        cb = [(im[k].cpu(), tk[k].cpu(), lb[k].cpu()) for im, tk, lb in batches]
        upd, ref_loss = otrain.local_update(model_class(spec), spec, glob.cpu(), cb, masks=[m[k].cpu() for m in masks])
        ref = torch.cat([u.reshape(-1) for u in upd])
        got = tr.X.data[k, : tr.P].cpu()
        assert abs(loss[k].item() - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
        assert _rel(got, ref) < 1e-5, _rel(got, ref)


@pytest.mark.parametrize("spec_name", ["wide", "vit_tiny"])
def test_client_chunking_bit_identical(cuda, spec_name):
    """Training the clients in chunks (TrainConfig.client_chunk) gives the
    same bits as one pass: every kernel's per-client result is independent of
    how many clients share its launch."""
    from flr.models.multimodal import VIT_BERT_TINY
    spec = SPEC_WIDE if spec_name == "wide" else VIT_BERT_TINY
    K, B, steps = 5, 4, 2
    glob = initial_global(spec, 42, cuda)
    batches = synthetic_batches(spec, steps, range(K), B, cuda)
    out = []
    for chunk in (0 if spec_name == "wide" else K, 2):
        tr = ClientBatchTrainer(spec, K, cuda, TrainConfig(local_steps=steps, client_chunk=chunk))
        assert len(tr.chunks) == (1 if chunk in (0, K) else 3)
        tr.load_global(glob)
        loss = tr.local_update(batches)
        out.append((loss.cpu(), tr.X.data[:, : tr.P].cpu()))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


def test_c2_round_fedavg_matches_reference(cuda):
    """Config C2 end to end: FedAvg over K = 32 clients of the ResNet-18 + GRU
    model (2 local steps at the reference batch 32, dropout masks): the
    engine's round vs the oracle's per-client loop (run_experiments.py:193-240)
    + oracle.fedavg (base_defense.py:80-97) at 1e-5."""
    from oracle import aggregation as orc
    from flr.round import RoundConfig, RoundEngine
    spec = ModelSpec()
    K, steps, B = 32, 2, 32
    rc = RoundConfig(num_clients=K, batch=B, defense="fedavg", attack="none", num_attackers=0)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=steps), cuda)
    glob = eng.global_flat.clone().cpu()
    new = eng.run_round().cpu()
    batches = synthetic_batches(spec, steps, range(K), B, "cpu")
    masks = make_dropout_masks(spec, steps, range(K), B, "cpu", seed=rc.seed + 7919)
    ups, ups64, losses = [], [], []
    for k in range(K):
        cb = [(im[k], tk[k], lb[k]) for im, tk, lb in batches]
        upd, ref_loss = otrain.local_update(MultimodalNet, spec, glob, cb, masks=[m[k] for m in masks])
        ups.append(upd)
        losses.append(ref_loss)
        # the same loop in fp64: how far the reference's own fp32 result is from exact
        ups64.append(otrain.local_update(MultimodalNet, spec, glob, cb, masks=[m[k] for m in masks],
                                         dtype=torch.float64)[0])
    ref = torch.cat([t.reshape(-1) for t in orc.fedavg(ups, [steps * B] * K)])
    ref64 = torch.cat([t.reshape(-1) for t in orc.fedavg(ups64, [steps * B] * K)])
    assert _rel(new, ref) < 1e-5, _rel(new, ref)
    layout = param_layout(spec)
    reps = {"aggregate": delta_report(new, ref, glob, layout)}
    X = eng.trainer.X.data[:, : eng.trainer.P]
    for k in (0, 31):
        row = eng.trainer.to_torch_order(X[k]) if eng.train_order else X[k]
        reps[f"client{k}"] = delta_report(row, torch.cat([u.reshape(-1) for u in ups[k]]), glob, layout)
    # the aggregate per tensor against the reference's own fp32 conditioning
    # (VERDICT r4 item 5): its fp32 weighted sum (32 terms of n_i * w ~ 64)
    # rounds by several ulp of w, so the bar is the fp32 reference's distance
    # from the same FedAvg in fp64 (tests/parity.py check_conditioned)
    cond = {"aggregate": conditioned_report(new, ref, ref64, glob, layout)}
    for k in (0, 31):
        row = eng.trainer.to_torch_order(X[k]) if eng.train_order else X[k]
        cond[f"client{k}"] = conditioned_report(row, torch.cat([u.reshape(-1) for u in ups[k]]),
                                                torch.cat([u.reshape(-1) for u in ups64[k]]), glob, layout)
    record("c2_update_parity.json", {"config": "C2: FedAvg K=32, ResNet-18 + GRU, B=32, 2 local steps",
                                     **{c: r for c, r in reps.items()},
                                     "conditioned": {c: r for c, r in cond.items()}})
    check_delta({c: r for c, r in reps.items() if c != "aggregate"})
    check_conditioned(cond)
    got_loss = eng.losses.cpu()
    err = max(abs(got_loss[k].item() - losses[k]) / max(1.0, abs(losses[k])) for k in range(K))
    print(f"\n[C2 round] weights rel err {_rel(new, ref):.2e}, max loss rel err {err:.2e}")
    assert err <= 1e-5


def test_c3_round_multikrum_signflip(cuda):
    """Config C3's round: K = 128 clients (f = 25 sign-flipped, multi_k = 64),
    1 local step.  Four sampled clients' trained rows (attackers and benign)
    match the oracle loop at 1e-5 (before the sign flip the row is the
    reference's local update; after it, its negation, model_poisoning.py:274-276);
    the Krum selection equals the oracle's scores and argsort on the GPU's
    distance matrix (krum.py:101-131, 174) and rejects every attacker."""
    from oracle import aggregation as orc
    from flr.round import RoundConfig, RoundEngine
    spec = ModelSpec()
    K, f, steps, B = 128, 25, 1, 8
    rc = RoundConfig(num_clients=K, batch=B, defense="krum", attack="sign_flip", num_attackers=f)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=steps), cuda)
    assert eng.defense.multi_k == 64
    glob = eng.global_flat.clone().cpu()
    eng.run_round()
    eng.defense.publish()
    eng.materialize()  # the client matrix whole (the dead-tap ranges, FLR_DEFER_DEAD)
    X = eng.trainer.X.data[:, : eng.trainer.P]
    batches = synthetic_batches(spec, steps, [0, 24, 25, 127], B, "cpu")
    masks = make_dropout_masks(spec, steps, [0, 24, 25, 127], B, "cpu", seed=rc.seed + 7919)
    reps = {}
    for j, k in enumerate([0, 24, 25, 127]):
        cb = [(im[j], tk[j], lb[j]) for im, tk, lb in batches]
        upd, _ = otrain.local_update(MultimodalNet, spec, glob, cb, masks=[m[j] for m in masks])
        ref = torch.cat([u.reshape(-1) for u in upd])
        row = eng.trainer.to_torch_order(X[k]) if eng.train_order else X[k]  # X is in training order
        # the update is compared before the sign flip (the attackers submit -row)
        reps[f"client{k}"] = delta_report(-row if k < f else row, ref, glob, param_layout(spec))
        if k < f:
            ref = -ref
        assert _rel(row.cpu(), ref) < 1e-5, (k, _rel(row.cpu(), ref))
    record("c3_update_parity_1step.json", {"config": "C3 round: K=128 Multi-Krum sign flip, B=8, 1 local step",
                                           **reps})
    check_delta(reps)
    D = eng.defense.distances.cpu().numpy()
    scores = orc.krum_scores(D, K - f - 2)
    import numpy as np
    order = np.argsort(scores, kind="stable")
    assert eng.defense.selected_clients == order[:64].tolist()
    assert not set(eng.defense.selected_clients) & set(range(f))
    s = np.sort(np.asarray(scores))
    print(f"\n[C3 round] selection-boundary margin {(s[64] - s[63]) / s[64]:.3e}")


def test_fused_clip_norm_matches_optimizer_pass(cuda, monkeypatch):
    """The clip norm from the conv weight-gradient epilogues' partials
    (flr_conv2d_bwd_weight_t_sq + flr_clip_sgd_step_blocked_x extra_sq) equals
    the optimizer's own sum-of-squares pass (FLR_FUSED_NORM=0) up to fp64
    summation order: per-client norms within 1e-6, trained rows within 1e-6."""
    spec = ModelSpec()
    K, B, steps = 3, 8, 2
    glob = initial_global(spec, 42, cuda)
    batches = synthetic_batches(spec, steps, range(K), B, cuda)
    out = []
    for fused in ("0", "1"):
        monkeypatch.setenv("FLR_FUSED_NORM", fused)
        tr = ClientBatchTrainer(spec, K, cuda, TrainConfig(local_steps=steps))
        assert bool(tr._norm_fused) == (fused == "1")
        tr.load_global(glob)
        tr.local_update(batches)
        out.append((tr.norms.cpu().clone(), tr.X.data[:, : tr.P].cpu().clone()))
    (n0, x0), (n1, x1) = out
    assert torch.all(n0 > 1.0)  # the clip is active (max_norm 1.0)
    assert ((n0 - n1).abs() / n0).max().item() <= 1e-6
    assert _rel(x1, x0) <= 1e-6, _rel(x1, x0)
