"""GPU parity for FLTrust (§8f rank 4): the server update on the
client-batched trainer vs the oracle training loop (no clipping), and the
trust-weighted aggregate vs the oracle restatement of fltrust.py:158-270."""
import numpy as np
import pytest
import torch

from oracle import aggregation as orc
from oracle.training import local_update
from flr.defenses import get_defense
from flr.models.multimodal import TINY, MultimodalNet
from flr.round import initial_global

pytestmark = pytest.mark.gpu


def test_fltrust_vs_oracle(cuda):
    spec = TINY
    g = torch.Generator().manual_seed(11)
    N = 40
    images = torch.randn(N, spec.in_channels, spec.image_size, spec.image_size, generator=g)
    tokens = torch.randint(0, spec.vocab, (N, spec.seq_len), generator=g)
    labels = torch.randint(0, spec.num_classes, (N,), generator=g)
    glob = initial_global(spec, 42, "cpu")
    d = get_defense("fltrust", {"batch_size": 16, "local_epochs": 2, "shuffle": False, "learning_rate": 0.05})
    d.set_root_dataset(images, tokens, labels)
    d.set_model(spec)

    # oracle server update: same batches in order, 2 epochs, one optimizer, no clipping
    batches = [(images[s:s + 16], tokens[s:s + 16], labels[s:s + 16]) for s in range(0, N, 16)] * 2
    after, _ = local_update(MultimodalNet, spec, glob, batches, lr=0.05, max_norm=float("inf"))
    sg = [a - b for a, b in zip(after, _split(glob, spec))]

    K = 7
    ups = []
    for i in range(K):
        sgn = -1.0 if i < 2 else 1.0  # two clients opposed to the server direction -> trust 0
        ups.append([sgn * t + 0.3 * torch.randn(t.shape, generator=g) * t.abs().mean() for t in sg])
    want, wtrust = orc.fltrust(ups, sg)
    got = d.aggregate([[t.to(cuda) for t in u] for u in ups], [1] * K,
                      global_params=[t.to(cuda) for t in _split(glob, spec)])
    sgot = d.server_gradient.cpu()
    swant = torch.cat([t.reshape(-1) for t in sg])
    assert (sgot - swant).abs().max().item() <= 1e-5 * max(1.0, swant.abs().max().item())
    assert np.allclose(d.trust_scores, wtrust, rtol=1e-4, atol=1e-6)
    assert d.trust_scores[0] == 0.0 and d.trust_scores[1] == 0.0
    for a, b in zip(got, want):
        err = (a.cpu().double() - b.double()).abs().max().item()
        assert err <= 1e-5 * max(1.0, b.abs().max().item()), err
    assert d.detect_malicious(None, None) == [i for i, s in enumerate(wtrust) if s < 0.1]


def _split(flat, spec):
    m = MultimodalNet(spec)
    out, off = [], 0
    for p in m.parameters():
        out.append(flat[off:off + p.numel()].view(p.shape).clone())
        off += p.numel()
    return out
