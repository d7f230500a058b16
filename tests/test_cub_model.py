"""CPU: the C1 model family — the reference's CUB200MultimodalCNN structure
(src/models/cub200_cnn.py:57-118) as flr's CubMultimodalNet.

* parameter count / order: SURVEY App. B (874,056 at C = 200, 312 attributes;
  825,226 at C = 10), names in the reference's nn.Sequential numbering;
* the reference's own shape tests restated (tests/test_models.py:117-142:
  multimodal and image-only forward at 224x224, C = 200);
* the engine's client-batched forward (torch path, CPU) equals the per-client
  module on every client."""
import dataclasses

import torch

from flr.models.multimodal import CUB, CubMultimodalNet, batched_forward, conv_geometry, num_params, param_layout, \
    split_params
from flr.train import synthetic_batches


def test_parameter_count_and_order():
    assert num_params(dataclasses.replace(CUB, num_classes=200)) == 874_056
    assert num_params(CUB) == 825_226
    names = [n for n, _ in param_layout(CUB)]
    assert names[:4] == ["image_conv.0.weight", "image_conv.0.bias", "image_conv.1.weight", "image_conv.1.bias"]
    assert names[-2:] == ["fusion.3.weight", "fusion.3.bias"]
    assert set(conv_geometry(CUB)) == {n for n, s in param_layout(CUB) if len(s) == 4}


def test_reference_shape_tests():
    """tests/test_models.py:120-142 (multimodal and image-only forward)."""
    torch.manual_seed(0)
    model = CubMultimodalNet(dataclasses.replace(CUB, num_classes=200))
    images = torch.randn(2, 3, 224, 224)
    assert model(images, torch.randn(2, 312)).shape == (2, 200)
    assert model(images, attributes=None).shape == (2, 200)


def test_batched_forward_matches_per_client_module():
    spec = CUB
    K, B = 3, 4
    torch.manual_seed(1)
    rows = []
    for _ in range(K):
        m = CubMultimodalNet(spec)
        rows.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]))
    X = torch.stack(rows)
    images, attrs, _ = synthetic_batches(spec, 1, range(K), B, "cpu")[0]
    assert attrs.shape == (K, B, spec.vocab) and set(attrs.unique().tolist()) <= {0.0, 1.0}
    got = batched_forward(split_params(X, spec), images, attrs, spec)
    for k in range(K):
        m = CubMultimodalNet(spec)
        off = 0
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(X[k, off:off + p.numel()].view(p.shape))
                off += p.numel()
        m.train()  # batch statistics, as in training
        m.fusion[2] = torch.nn.Identity()  # the engine applies dropout through explicit masks
        ref = m(images[k], attrs[k])
        assert torch.allclose(got[k], ref, rtol=1e-5, atol=1e-5), (got[k] - ref).abs().max()
