"""GPU: the round engine's auxiliary paths.

* checkpoint / resume — the reference's dict {'round', 'model_state_dict',
  'accuracy', 'loss'} (run_experiments.py:268-279), loadable into the
  reference-structured module, and a resumed engine continues bit-identically;
* FedAvg fallback when the defense raises (robust_server.py:120-122);
* FLTrust through the round engine (the global_params plumbing the
  reference's simulation lacks, fltrust.py:235-238).
"""
import pytest
import torch

from oracle import aggregation as orc
from flr.models.multimodal import TINY, MultimodalNet
from flr.round import RoundConfig, RoundEngine
from flr.train import TrainConfig

pytestmark = pytest.mark.gpu


def test_checkpoint_resume_bit_identical(cuda, tmp_path):
    rc = RoundConfig(num_clients=4, batch=4, defense="fedavg", attack="none", num_attackers=0, graph=False)
    eng = RoundEngine(TINY, rc, TrainConfig(local_steps=2), cuda)
    eng.run_round()
    path = str(tmp_path / "ck.pt")
    eng.save_checkpoint(path, accuracy=0.25, loss=2.0)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert set(ck) == {"round", "model_state_dict", "accuracy", "loss"} and ck["round"] == 1
    m = MultimodalNet(TINY)
    m.load_state_dict(ck["model_state_dict"])  # strict: every parameter and buffer
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert torch.equal(flat, eng.global_flat.cpu())
    eng2 = RoundEngine(TINY, rc, TrainConfig(local_steps=2), cuda)
    assert eng2.load_checkpoint(path) == 1
    assert torch.equal(eng.run_round(), eng2.run_round())
    assert eng2.round_index == 2


def test_fedavg_fallback_when_defense_raises(cuda):
    # Krum with f = 1 needs n >= 5: at n = 4 it raises (krum.py:153-157)
    kw = dict(num_clients=4, batch=4, attack="sign_flip", num_attackers=1, graph=False)
    eng = RoundEngine(TINY, RoundConfig(defense="krum", fallback_fedavg=True, **kw), TrainConfig(local_steps=1), cuda)
    out = eng.run_round().clone()
    assert eng.fell_back and eng.fallback_error == "ValueError"
    ref = RoundEngine(TINY, RoundConfig(defense="fedavg", **kw), TrainConfig(local_steps=1), cuda).run_round()
    assert torch.equal(out, ref)
    strict = RoundEngine(TINY, RoundConfig(defense="krum", **kw), TrainConfig(local_steps=1), cuda)
    with pytest.raises(ValueError):
        strict.run_round()
    # a device / library failure: falls back by default, as the reference's
    # `except Exception` (fallback_device_errors=True); False keeps it loud
    from flr._capi import FlrError

    def _fail(*a, **k):
        raise FlrError("flr_fedavg", -3, "injected")
    for loud in (False, True):
        boom = RoundEngine(TINY, RoundConfig(defense="fedavg", fallback_fedavg=True,
                                             fallback_device_errors=not loud, **kw),
                           TrainConfig(local_steps=1), cuda)
        boom.defense.aggregate_flat = _fail
        boom.defense.aggregate_sharded = _fail
        if loud:
            with pytest.raises(FlrError):
                boom.run_round()
        else:
            assert torch.equal(boom.run_round(), ref) and boom.fallback_error == "FlrError"


def test_round_refine_overflow_raises(cuda):
    """K = 300 with 140 sign-flipped clients — more far-cluster rows
    than the Gram path refines.  The round raises on its own device path
    (run_round never calls publish), instead of ranking a NaN matrix; with the
    FedAvg fallback on it falls back (the default, as the reference's `except
    Exception`) unless fallback_device_errors=False."""
    from flr._capi import FlrError
    kw = dict(num_clients=300, batch=4, defense="krum", attack="sign_flip", num_attackers=140, graph=False,
              defense_cfg={"pairwise_method": "gram"})
    for fb, dev in ((False, True), (True, False)):
        eng = RoundEngine(TINY, RoundConfig(fallback_fedavg=fb, fallback_device_errors=dev, **kw),
                          TrainConfig(local_steps=1), cuda)
        with pytest.raises(FlrError):
            eng.run_round()
    # the default with the fallback on: FedAvg, as the reference's `except Exception`
    eng = RoundEngine(TINY, RoundConfig(fallback_fedavg=True, **kw), TrainConfig(local_steps=1), cuda)
    eng.run_round()
    assert eng.fell_back and eng.fallback_error == "FlrError"


def test_fltrust_round(cuda):
    """FLTrust in the round loop: the engine hands the defense a copy of the
    round's global vector; the result equals the oracle's trust-weighted
    aggregate of the same client rows given the same server update."""
    spec = TINY
    g = torch.Generator().manual_seed(5)
    N = 24
    root = (torch.randn(N, spec.in_channels, spec.image_size, spec.image_size, generator=g),
            torch.randint(0, spec.vocab, (N, spec.seq_len), generator=g),
            torch.randint(0, spec.num_classes, (N,), generator=g))
    rc = RoundConfig(num_clients=6, batch=4, defense="fltrust", attack="sign_flip", num_attackers=1,
                     defense_cfg={"batch_size": 8, "shuffle": False}, graph=False)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=2), cuda)
    eng.defense.set_root_dataset(*root)
    eng.defense.set_model(spec)
    assert eng.exchange == "allgather"
    before = eng.global_flat.clone()
    out = eng.run_round().clone()
    assert not torch.equal(out, before)
    X = eng.full.X.cpu()
    ups = [[X[i]] for i in range(X.shape[0])]
    want, trust = orc.fltrust(ups, [eng.defense.server_gradient.cpu()])
    # every client's trust score matches the oracle's (fltrust.py:158-214); the
    # simulation's updates are weights, so the sign-flipped row's cosine against
    # the server delta has no fixed sign and is checked like the others
    assert len(eng.defense.trust_scores) == len(trust) == 6
    for got_t, want_t in zip(eng.defense.trust_scores, trust):
        assert abs(got_t - want_t) <= 1e-4 * max(1.0, abs(want_t)) + 1e-6
    err = (out.cpu().double() - want[0].double()).abs().max().item()
    assert err <= 1e-5 * max(1.0, want[0].abs().max().item()), err


@pytest.mark.parametrize("defense,cfg,attack,f", [
    ("fedavg", {}, "none", 0),
    ("median", {}, "sign_flip", 2),
    ("trimmed_mean", {"trim_ratio": 0.2}, "sign_flip", 2),
    ("krum", {"multi_k": 4}, "sign_flip", 1),
])
def test_training_order_round_equals_torch_order(cuda, monkeypatch, defense, cfg, attack, f):
    """Training-order rounds (BaseDefense.order_free: the last optimizer step
    writes the client matrix in the trainer's coordinate order, dead-tap ranges
    from the global vector, the attackers' rows negated) give the global model
    of the torch-order export path: bit-identical for coordinate-wise rules
    (FedAvg, median), the same Krum selection, and the trimmed mean within
    1e-6 (its torch-restated cascade sum depends on a column's position in
    torch's vectorised loop).  Full ResNet-18 + GRU model (tap-major convs,
    dead taps), 2 rounds with HIP-graph replay."""
    from flr.models.multimodal import ModelSpec
    spec = ModelSpec()
    rc = RoundConfig(num_clients=8, batch=4, defense=defense, defense_cfg=dict(cfg), attack=attack, num_attackers=f)
    outs, sels = [], []
    for order in ("torch", "train"):
        monkeypatch.setenv("FLR_ORDER", order)
        eng = RoundEngine(spec, rc, TrainConfig(local_steps=2), cuda)
        assert eng.train_order == (order == "train")
        for _ in range(2):
            eng.run_round()
        outs.append(eng.global_flat.clone().cpu())
        sels.append(list(getattr(eng.defense, "selected_clients", [])))
    a, b = outs
    assert torch.isfinite(a).all()
    if defense == "trimmed_mean":
        err = ((a - b).abs().max() / a.abs().max()).item()
        assert err <= 1e-6, err
    elif defense == "krum":
        assert sorted(sels[0]) == sorted(sels[1]) and not set(sels[1]) & set(range(f))
        err = ((a - b).abs().max() / a.abs().max()).item()
        assert err <= 1e-6, err
    else:
        assert torch.equal(a, b)


@pytest.mark.parametrize("order", ["train", "torch"])
def test_native_trainer_round_equals_python_trainer(cuda, monkeypatch, order):
    """The round engine's ResNet + GRU trainer is the one C entry
    flr_train_clients_ex (training order: live-only load, the last step
    writing X, dead-tap ranges from the global vector; torch order: the
    export pass), with the residual blocks' two gradient paths summed in the
    dgrad epilogue.  Against the Python autograd composition of the same
    kernels (FLR_TRAINER=python): the same global model bit for bit, the
    same per-client losses, over 2 rounds of HIP-graph replay with sign-flip
    attackers, on the full ResNet-18 + GRU model (tap-major convs, dead taps)."""
    from flr.models.multimodal import ModelSpec
    spec = ModelSpec()
    rc = RoundConfig(num_clients=6, batch=4, defense="median", attack="sign_flip", num_attackers=2)
    monkeypatch.setenv("FLR_ORDER", order)
    res = []
    for trainer in ("python", "native"):
        monkeypatch.setenv("FLR_TRAINER", trainer)
        eng = RoundEngine(spec, rc, TrainConfig(local_steps=2), cuda)
        assert eng.native == (trainer == "native") and eng.train_order == (order == "train")
        for _ in range(2):
            eng.run_round()
        res.append((eng.global_flat.clone().cpu(), eng.losses.clone().cpu(), eng.trainer.X.X.clone().cpu()))
    (ga, la, xa), (gb, lb, xb) = res
    assert torch.isfinite(ga).all()
    assert torch.equal(la, lb)
    assert torch.equal(xa, xb)
    assert torch.equal(ga, gb)


@pytest.mark.parametrize("defer,multi_k", [("1", 4), ("1", 1), ("2", 4), ("2", 1)])
def test_deferred_dead_taps_bit_identical(cuda, monkeypatch, defer, multi_k):
    """FLR_DEFER_DEAD=1 (opt-in): the training phase leaves X's dead-tap slabs
    to a side-stream fill beside the reference-exact Krum distances, which
    read those taps from the global vector meanwhile; =2: never written — the
    distances and the Multi-Krum mean (flr_rows_mean_dead; the selected row
    itself at multi_k = 1) read them from the round's global vector, and
    materialize() writes them for other readers.  Against the slabs written
    last in the training phase (FLR_DEFER_DEAD=0): the same distance matrix,
    selection, client matrix and global model bit for bit, over 2 rounds of
    HIP-graph replay with sign-flip attackers, on the full ResNet-18 + GRU
    model (dead taps in layers 3-4)."""
    from flr.models.multimodal import ModelSpec
    spec = ModelSpec()
    rc = RoundConfig(num_clients=8, batch=4, defense="krum", attack="sign_flip", num_attackers=1,
                     defense_cfg={"pairwise_method": "reference", "multi_k": multi_k})
    res = []
    for d in ("0", defer):
        monkeypatch.setenv("FLR_DEFER_DEAD", d)
        eng = RoundEngine(spec, rc, TrainConfig(local_steps=2), cuda)
        assert eng.train_order and (eng._fill is not None) == (d == "1") and (eng._lazy is not None) == (d == "2")
        for _ in range(2):
            eng.run_round()
        eng.defense.publish()
        eng.materialize()
        res.append((eng.global_flat.clone().cpu(), eng.defense.distances.clone().cpu(),
                    list(eng.defense.selected_clients), eng.trainer.X.X.clone().cpu()))
    (ga, da, sa, xa), (gb, db, sb, xb) = res
    assert torch.isfinite(ga).all() and torch.isfinite(da).all()
    assert torch.equal(da, db) and sa == sb
    assert torch.equal(xa, xb)
    assert torch.equal(ga, gb)


def test_dead_deferral_only_where_the_defense_reads_it(cuda, monkeypatch):
    """The dead-tap deferral (FLR_DEFER_DEAD=2, default) is on only for a
    defense that reads the unwritten ranges through the global vector (Krum /
    Multi-Krum, `supports_dead_rows`); Krum + trimmed mean reads the selected
    rows whole, so its rounds keep the slabs written — the same global model
    as with the deferral switched off."""
    from flr.models.multimodal import ModelSpec
    spec = ModelSpec()
    monkeypatch.delenv("FLR_DEFER_DEAD", raising=False)
    kw = dict(num_clients=8, batch=4, attack="sign_flip", num_attackers=1)
    eng = RoundEngine(spec, RoundConfig(defense="krum", defense_cfg={"multi_k": 4}, **kw),
                      TrainConfig(local_steps=1), cuda)
    assert eng._lazy is not None and eng.trainer.defer_dead
    outs = []
    for d in (None, "0"):
        if d is not None:
            monkeypatch.setenv("FLR_DEFER_DEAD", d)
        eng = RoundEngine(spec, RoundConfig(defense="krum_trimmed_mean", defense_cfg={"multi_k": 6,
                                                                                       "trim_ratio": 0.2}, **kw),
                          TrainConfig(local_steps=1), cuda)
        assert eng.train_order and eng._lazy is None and eng._fill is None and not eng.trainer.defer_dead
        outs.append(eng.run_round().clone().cpu())
    assert torch.isfinite(outs[0]).all() and torch.equal(outs[0], outs[1])
