"""CPU: the C4/C5 model family's client-batched form (torch ops, the layout the
HIP kernels run) against one ViTBertNet per client — logits and every
parameter gradient — plus its geometry (P of ViT-S/4 + BERT-mini)."""
import pytest
import torch

from flr.models.multimodal import VIT_BERT, VIT_BERT_TINY, batched_forward, model_class, num_params, split_params
from flr.models.transformer import patchify


def test_vit_bert_parameter_count():
    # ViT-S/4 at 32x32 (21.3M) + BERT-mini (11.2M) + the fusion head: ~3.3e7 (SURVEY §8 nominal)
    assert num_params(VIT_BERT) == 32_675_722


def test_patchify_matches_conv():
    g = torch.Generator().manual_seed(0)
    img = torch.randn(2, 3, 32, 32, generator=g)
    w = torch.randn(16, 3, 4, 4, generator=g)
    conv = torch.nn.functional.conv2d(img, w, stride=4).flatten(2).transpose(1, 2)  # [B, 64, 16]
    lin = patchify(img, 4) @ w.reshape(16, -1).T
    torch.testing.assert_close(lin, conv, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("K", [1, 3])
def test_batched_form_matches_per_client_module(K):
    spec = VIT_BERT_TINY
    B = 4
    g = torch.Generator().manual_seed(K)
    torch.manual_seed(7)
    base = torch.cat([p.detach().reshape(-1) for p in model_class(spec)(spec).parameters()])
    P = base.numel()
    X = (base + 0.01 * torch.randn(K, P, generator=g)).requires_grad_(True)
    images = torch.randn(K, B, 3, spec.image_size, spec.image_size, generator=g)
    tokens = torch.randint(0, spec.vocab, (K, B, spec.seq_len), generator=g)
    labels = torch.randint(0, spec.num_classes, (K, B), generator=g)
    logits = batched_forward(split_params(X, spec), images, tokens, spec)
    loss = torch.nn.functional.cross_entropy(logits.reshape(K * B, -1), labels.reshape(-1), reduction="sum")
    (gX,) = torch.autograd.grad(loss, X)
    for k in range(K):
        m = model_class(spec)(spec)
        off = 0
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(X[k, off:off + p.numel()].view(p.shape))
                off += p.numel()
        out = m(images[k], tokens[k])
        torch.testing.assert_close(logits[k].detach(), out.detach(), rtol=1e-5, atol=1e-5)
        lk = torch.nn.functional.cross_entropy(out, labels[k], reduction="sum")
        grads = torch.autograd.grad(lk, list(m.parameters()))
        ref = torch.cat([t.reshape(-1) for t in grads])
        torch.testing.assert_close(gX[k], ref, rtol=1e-4, atol=1e-6)
