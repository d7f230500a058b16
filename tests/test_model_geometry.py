"""CPU: the static conv geometry the trainer uses to find dead kernel taps
(flr.models.multimodal.conv_geometry / live_taps) matches the real network,
and a dead tap's gradient is exactly zero in the reference model."""
import torch
import torch.nn as nn

from flr.models.multimodal import ModelSpec, MultimodalNet, conv_geometry, live_taps, param_layout


def _observed(spec):
    m = MultimodalNet(spec)
    seen = {}
    names = {id(mod): n for n, mod in m.named_modules()}

    def hook(mod, inp, out):
        seen[names[id(mod)] + ".weight"] = (inp[0].shape[-1], mod.kernel_size[0], mod.stride[0], mod.padding[0],
                                            out.shape[-1])
    for mod in m.modules():
        if isinstance(mod, nn.Conv2d):
            mod.register_forward_hook(hook)
    m(torch.randn(2, 3, spec.image_size, spec.image_size), torch.randint(0, spec.vocab, (2, spec.seq_len)))
    return m, seen


def test_conv_geometry_matches_network():
    for spec in (ModelSpec(), ModelSpec(widths=(8, 16, 16, 32), blocks=(1, 1, 1, 1), vocab=50, embed=8, hidden=16,
                                        fusion=16)):
        _, seen = _observed(spec)
        geo = conv_geometry(spec)
        assert geo == seen
        assert set(geo) == {n for n, s in param_layout(spec) if len(s) == 4}


def test_dead_taps_have_zero_gradient():
    spec = ModelSpec()
    torch.manual_seed(0)
    m, _ = _observed(spec)
    loss = m(torch.randn(3, 3, 32, 32), torch.randint(0, spec.vocab, (3, spec.seq_len))).square().sum()
    loss.backward()
    geo = conv_geometry(spec)
    dead_total = 0
    for n, p in m.named_parameters():
        if n in geo:
            H, k, s, pd, _ = geo[n]
            live = set(live_taps(H, k, s, pd))
            g = p.grad.reshape(p.shape[0], p.shape[1], k * k)
            for t in range(k * k):
                if t not in live:
                    assert torch.count_nonzero(g[:, :, t]) == 0, (n, t)
                    dead_total += p.shape[0] * p.shape[1]
    assert dead_total > 6_000_000  # most of layer4's 3x3 weights
