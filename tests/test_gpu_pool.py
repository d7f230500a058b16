"""GPU parity: the native max-pool (flr_maxpool2d_fwd/_bwd) vs torch's CPU
F.max_pool2d forward and backward — bit-exact, including the exact-zero ties a
ReLU in front of the pool produces (the stem: relu(bn(conv)) -> 3x3/2 pad 1)."""
import pytest
import torch
import torch.nn.functional as F

from flr.nn import client_maxpool2d

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,k,s,p", [((4, 6, 16, 16), 3, 2, 1), ((2, 5, 7, 9), 3, 2, 1), ((3, 4, 8, 8), 2, 2, 0),
                                         ((2, 3, 5, 5), 3, 1, 1), ((1, 2, 1, 1), 3, 2, 1),
                                         ((1, 3, 64, 64), 3, 2, 1), ((2, 3, 33, 17), 3, 2, 1),
                                         ((2, 3, 10, 11), 3, 3, 1)])  # stride 3: the generic-stride kernel
@pytest.mark.parametrize("relu", [False, True])
def test_maxpool_matches_torch_cpu(cuda, shape, k, s, p, relu):
    g = torch.Generator().manual_seed(sum(shape) + k)
    x = torch.randn(*shape, generator=g)
    if relu:
        x = F.relu(x)
    xc = x.clone().requires_grad_(True)
    yc = F.max_pool2d(xc, k, s, p)
    dy = torch.randn(yc.shape, generator=g)
    yc.backward(dy)
    xg = x.to(cuda).requires_grad_(True)
    yg = client_maxpool2d(xg, k, s, p)
    yg.backward(dy.to(cuda))
    assert torch.equal(yg.detach().cpu(), yc.detach())
    assert torch.equal(xg.grad.cpu(), xc.grad)
