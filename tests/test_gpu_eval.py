"""GPU parity: per-round evaluation of the global model
on the HIP kernels vs the oracle's restatement of src/utils/metrics.py:14-157
and the backdoor's triggered test set (src/attacks/backdoor.py:62-112).
Counts are exact, the loss within 1e-5.  The model is first trained one round
so that the weights, and the predictions, are not the init's."""
import pytest
import torch

from oracle import evaluation as oeval
from flr.attacks import Backdoor
from flr.metrics import GlobalEvaluator
from flr.models.multimodal import CUB, TINY, ModelSpec, model_class
from flr.round import RoundConfig, RoundEngine
from flr.train import TrainConfig, synthetic_batches

pytestmark = pytest.mark.gpu


def _test_set(spec, n, seed):
    """n samples as one 'client' stream (synthetic_batches with one step)."""
    im, tx, lb = synthetic_batches(spec, 1, [seed], n, "cpu")[0]
    return im[0], tx[0], lb[0]


@pytest.mark.parametrize("spec", [TINY, CUB, ModelSpec()], ids=["tiny", "cub-c1", "resnet18-gru"])
def test_evaluate_and_asr_match_reference(cuda, spec):
    eng = RoundEngine(spec, RoundConfig(num_clients=4, batch=8, defense="fedavg", attack="none", num_attackers=0),
                      TrainConfig(local_steps=2), cuda)
    glob = eng.run_round().clone()
    images, text, labels = _test_set(spec, 70, 5000)  # 2 full batches of 32 + a partial one of 6
    ev = GlobalEvaluator(spec, cuda, batch_size=32, chunk=64)
    ev.load(glob)
    got = ev.evaluate_model(images, text, labels)
    ref = oeval.evaluate_model(model_class(spec), spec, glob.cpu(), images, text, labels)
    assert got["total"] == ref["total"] == 70
    assert got["correct"] == ref["correct"], (got, ref)
    assert abs(got["loss"] - ref["loss"]) <= 1e-5 * max(1.0, abs(ref["loss"]))

    bd = Backdoor(target_class=0, image_size=(spec.image_size, spec.image_size))
    asr = ev.attack_success_rate(images, text, labels, bd)
    ti, tt, _ = oeval.triggered_testset(images, text, labels, bd)
    assert asr == oeval.attack_success_rate(model_class(spec), spec, glob.cpu(), ti, tt, 0)

    lf = ev.label_flip_asr(images, text, labels, source_class=3, target_class=0)
    assert lf == oeval.label_flip_asr(model_class(spec), spec, glob.cpu(), images, text, labels, 3, 0)


def test_classify_rows_tie_and_nan_rules(cuda):
    """torch.max(outputs, 1): first maximal index; NaN counts as the maximum."""
    from flr import _capi
    z = torch.tensor([[1.0, 3.0, 3.0, 0.0], [float("nan"), 5.0, float("nan"), 1.0], [2.0, 2.0, 2.0, 2.0],
                      [-float("inf")] * 4])
    pred = torch.empty(4, dtype=torch.int32, device=cuda)
    rows = torch.empty(4, device=cuda)
    counts = torch.zeros(5, dtype=torch.int64, device=cuda)
    lab = torch.tensor([1, 1, 3, 0], device=cuda)
    zc = z.to(cuda)
    _capi.call("flr_classify_rows", zc.data_ptr(), lab.data_ptr(), 4, 4, 2, -1, pred.data_ptr(), rows.data_ptr(),
               counts.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert pred.cpu().tolist() == torch.max(z, 1)[1].tolist()
    assert counts.cpu().tolist()[:2] == [int((torch.max(z, 1)[1] == lab.cpu()).sum()), 0]


def test_round_engine_evaluate(cuda):
    """RoundEngine.evaluate == the evaluator on the engine's global vector."""
    spec = TINY
    eng = RoundEngine(spec, RoundConfig(num_clients=4, batch=8, defense="krum", num_attackers=0), TrainConfig(
        local_steps=1), cuda)
    eng.run_round()
    images, text, labels = _test_set(spec, 40, 77)
    got = eng.evaluate(images, text, labels)
    ref = oeval.evaluate_model(model_class(spec), spec, eng.global_flat.cpu(), images, text, labels, batch_size=8)
    assert got["correct"] == ref["correct"] and abs(got["loss"] - ref["loss"]) <= 1e-5 * max(1.0, ref["loss"])
