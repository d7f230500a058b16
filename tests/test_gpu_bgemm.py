"""GPU: the batched dense GEMM (flr_bgemm, the text branch and late-fusion MLP
products) and ClientLinear vs fp64 torch.  Covers every operand mode (RK, KR,
scalar gather), bias / addend epilogues, split-K and ragged shapes; and that a
client's result does not depend on how many clients share the launch."""
import pytest
import torch

from flr.nn import bgemm, client_linear, sum_rows

pytestmark = pytest.mark.gpu


def _ref(A, B, bias=None, add=None):
    y = torch.bmm(A.double(), B.double().transpose(1, 2))
    if bias is not None:
        y = y + bias.double().unsqueeze(1)
    if add is not None:
        y = y + add.double()
    return y


def _check(got, ref, tol=2e-6):
    err = (got.double().cpu() - ref.cpu()).abs().max().item()
    scale = max(ref.abs().max().item(), 1.0)
    assert err <= tol * scale, (err, scale)


@pytest.mark.parametrize("K,M,N,R", [(3, 32, 256, 768), (2, 32, 10, 256), (4, 512, 768, 128), (2, 32, 768, 256),
                                     (3, 7, 9, 5), (2, 64, 64, 2048), (1, 33, 65, 130)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_bgemm_modes_vs_fp64(cuda, K, M, N, R, ta, tb):
    g = torch.Generator().manual_seed(K * 1000 + M + N + R)
    A = torch.randn(K, R, M, generator=g).transpose(1, 2) if ta else torch.randn(K, M, R, generator=g)
    B = torch.randn(K, R, N, generator=g).transpose(1, 2) if tb else torch.randn(K, N, R, generator=g)
    C = bgemm(A.to(cuda), B.to(cuda))
    _check(C, _ref(A, B))


def test_bgemm_bias_and_addend(cuda):
    g = torch.Generator().manual_seed(3)
    K, M, N, R = 3, 32, 768, 256
    A, B = torch.randn(K, M, R, generator=g), torch.randn(K, N, R, generator=g)
    bias, add = torch.randn(K, N, generator=g), torch.randn(K, M, N, generator=g)
    _check(bgemm(A.to(cuda), B.to(cuda), bias=bias.to(cuda)), _ref(A, B, bias=bias))
    _check(bgemm(A.to(cuda), B.to(cuda), add=add.to(cuda)), _ref(A, B, add=add))


def test_bgemm_batch_invariant(cuda):
    """Client k's product is bit-identical whether 2 or 16 clients share the launch."""
    g = torch.Generator().manual_seed(4)
    A, B = torch.randn(16, 32, 768, generator=g).to(cuda), torch.randn(16, 256, 768, generator=g).to(cuda)
    assert torch.equal(bgemm(A, B)[:2], bgemm(A[:2], B[:2]))


def test_client_linear_fwd_bwd(cuda):
    g = torch.Generator().manual_seed(5)
    K, M, I, O = 3, 32, 768, 10
    x, W, b = torch.randn(K, M, I, generator=g), torch.randn(K, O, I, generator=g) * 0.05, torch.randn(K, O, generator=g)
    dy = torch.randn(K, M, O, generator=g)
    xs = [t.to(cuda).requires_grad_(True) for t in (x, W, b)]
    y = client_linear(*xs)
    y.backward(dy.to(cuda))
    rs = [t.double().requires_grad_(True) for t in (x, W, b)]
    yr = torch.baddbmm(rs[2].unsqueeze(1), rs[0], rs[1].transpose(1, 2))
    yr.backward(dy.double())
    _check(y.detach(), yr.detach())
    for a, r in zip(xs, rs):
        _check(a.grad, r.grad)


def test_sum_rows(cuda):
    X = torch.randn(3, 513, 70)
    _check(sum_rows(X.to(cuda)), X.double().sum(dim=1), tol=1e-6)
