"""GPU: the LDS-DMA form of the batched GEMM (dsgemm_kernel, 128 x 128 tiles with
RK / KR operands) is bit-identical to the split-at-stash form (FLR_BGEMM_DMA=0,
an A/B switch; tools build only) — same bf16 products in the same order per accumulator — on the
encoder shapes, ragged edges (rows, columns and a partial last K-tile), split-K
and the bias / addend epilogues; and within 2e-6 of fp64."""
import pytest
import torch

from flr.nn import bgemm

# the LDS-DMA and pre-split forms measured slower: tools build only (make ABLATION=1)
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("ablation_build")]


def _ops(K, M, N, R, ta, tb, seed):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(K, R, M, generator=g).transpose(1, 2) if ta else torch.randn(K, M, R, generator=g)
    B = torch.randn(K, R, N, generator=g).transpose(1, 2) if tb else torch.randn(K, N, R, generator=g)
    return A, B


@pytest.mark.parametrize("K,M,N,R", [(2, 2080, 1152, 384), (3, 130, 200, 260), (2, 257, 132, 1000),
                                     (1, 128, 128, 8192), (4, 512, 1024, 256), (2, 192, 384, 2080)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_bgemm_dma_equals_stash(cuda, knob, K, M, N, R, ta, tb):
    A, B = _ops(K, M, N, R, ta, tb, K * 7 + M + N + R)
    A, B = A.to(cuda), B.to(cuda)
    knob("FLR_BGEMM_PRESPLIT", "0")
    knob("FLR_BGEMM_DMA", "0")
    C0 = bgemm(A, B)
    knob("FLR_BGEMM_DMA", "1")
    C1 = bgemm(A, B)
    torch.cuda.synchronize()
    assert torch.equal(C0, C1), (C0 - C1).abs().max().item()
    ref = torch.bmm(A.double(), B.double().transpose(1, 2))
    err = (C1.double() - ref).abs().max().item()
    assert err <= 2e-6 * max(ref.abs().max().item(), 1.0), err


def test_bgemm_dma_epilogues_equal_stash(cuda, knob):
    A, B = _ops(3, 260, 300, 512, False, False, 11)
    g = torch.Generator().manual_seed(12)
    bias, add = torch.randn(3, 300, generator=g).to(cuda), torch.randn(3, 260, 300, generator=g).to(cuda)
    A, B = A.to(cuda), B.to(cuda)
    knob("FLR_BGEMM_PRESPLIT", "0")
    outs = []
    for flag in ("0", "1"):
        knob("FLR_BGEMM_DMA", flag)
        outs.append((bgemm(A, B, bias=bias), bgemm(A, B, add=add)))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("K,M,N,R", [(2, 2080, 1152, 384), (3, 130, 200, 260), (2, 257, 132, 1000),
                                     (1, 128, 128, 8192), (4, 512, 1024, 256), (2, 192, 384, 2080)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_bgemm_presplit_equals_stash(cuda, knob, K, M, N, R, ta, tb):
    """The pre-split form (FLR_BGEMM_PRESPLIT=1, opt-in: measured slower; bf16 planes
    split once per GEMM, a six-product bf16 loop staged by LDS-DMA) against the
    default split-at-stash form: bit-identical, incl. ragged edges and split-K; and a
    scalar-gather operand (strides neither row- nor k-contiguous)."""
    A, B = _ops(K, M, N, R, ta, tb, K * 5 + M + N + R)
    A, B = A.to(cuda), B.to(cuda)
    outs = []
    for flag in ("0", "1"):
        knob("FLR_BGEMM_PRESPLIT", flag)
        outs.append(bgemm(A, B).clone())
        outs.append(bgemm(A[:, :, ::2][:, :, :R // 2], B[:, :, ::2][:, :, :R // 2]).clone())  # gather mode
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[2]), (outs[0] - outs[2]).abs().max().item()
    assert torch.equal(outs[1], outs[3])


def test_bgemm_presplit_epilogues_equal_stash(cuda, knob):
    A, B = _ops(3, 260, 300, 512, False, False, 13)
    g = torch.Generator().manual_seed(14)
    bias, add = torch.randn(3, 300, generator=g).to(cuda), torch.randn(3, 260, 300, generator=g).to(cuda)
    A, B = A.to(cuda), B.to(cuda)
    outs = []
    for flag in ("0", "1"):
        knob("FLR_BGEMM_PRESPLIT", flag)
        outs.append((bgemm(A, B, bias=bias), bgemm(A, B, add=add)))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
