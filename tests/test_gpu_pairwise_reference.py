"""GPU: the reference-exact Krum distance mode (pairwise_method="reference",
flr_pairwise_l2_reference) against the reference's own per-pair fp32
``torch.norm(fi - fj).item()`` (krum.py:89-97) — BIT-identical D, hence
identical scores, selected and rejected lists (krum.py:101-131, 174-176).

Oracles: oracle.aggregation.distance_matrix (torch.norm per pair, the
reference's op), oracle.normref (its C restatement, pinned against torch.norm
in tests/test_oracle.py; used where the torch loop would take minutes), and the
C3-shaped golden fixtures (their `dist` field is the oracle's torch.norm D)."""
import hashlib

import numpy as np
import pytest
import torch

from conftest import golden_files, load_golden
from oracle import aggregation as orc
from oracle import normref
from flr import ops
from flr.defenses import KrumDefense
from flr.matrix import ClientMatrix, padded_ld
from flr.workload import update_matrix

pytestmark = pytest.mark.gpu


def _matrix(K, P, seed, device):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(K, P, generator=g) * 0.05
    X[: K // 5] = -X[: K // 5]
    X += 1e-3 * torch.randn(K, P, generator=g) * torch.exp(torch.randn(K, P, generator=g))
    data = torch.zeros((K, padded_ld(P)), dtype=torch.float32)
    data[:, :P] = X
    return X, data.to(device)


@pytest.mark.parametrize("K,P", [(2, 0), (2, 1), (3, 7), (5, 8), (7, 9), (9, 255), (12, 256), (13, 257), (5, 12), (6, 13), (7, 15), (4, 4), (4, 6),
                                 (16, 4099), (33, 2053), (40, 65537), (1, 100)])
def test_reference_mode_equals_torch_norm(cuda, K, P):
    X, data = _matrix(K, P, K * 1000 + P, cuda)
    D = ops.pairwise_l2(data[:, :P], "reference").cpu().numpy()
    want = orc.distance_matrix([[X[k]] for k in range(K)])
    assert np.array_equal(D, want), np.abs(D - want).max()


def test_reference_mode_unaligned_view(cuda):
    """A row view starting 4 B into the buffer (not 16-B aligned): the op
    re-pads it; D unchanged."""
    K, P = 10, 3001
    X, _ = _matrix(K, P, 77, cuda)
    buf = torch.zeros((K, P + 1), dtype=torch.float32, device=cuda)
    buf[:, 1:] = X.to(cuda)
    D = ops.pairwise_l2(buf[:, 1:], "reference").cpu().numpy()
    assert np.array_equal(D, orc.distance_matrix([[X[k]] for k in range(K)]))


@pytest.mark.parametrize("K,P", [(128, 1 << 20), (64, 3_000_017), (300, 20_011)])
def test_reference_mode_large_vs_c_oracle(cuda, K, P):
    """Longer chains and K > 128 (more tiles than CUs) against the C restatement."""
    X, data = _matrix(K, P, 5 + K, cuda)
    D = ops.pairwise_l2(data[:, :P], "reference").cpu().numpy()
    assert np.array_equal(D, normref.distance_matrix(X.numpy()))


@pytest.mark.parametrize("K,P,two", [(33, 4099, "1"), (64, 65_537, "1"), (100, 20_011, "1"), (127, 3001, "1"),
                                     (300, 20_011, "0"), (257, 1000, "1")])
def test_reference_mode_two_chain_tiles(cuda, knob, K, P, two):
    """The K >= 256 form (ref_chain2_kernel: two chains per lane on the
    off-diagonal tiles, the 1-I circulant diagonal tiles, a 4-stage ring at two
    waves per SIMD) forced on below 256 (FLR_REF_2I=1) and off above it (=0):
    D bit-identical to the C restatement either way, ragged super-blocks
    included."""
    knob("FLR_REF_2I", two)
    X, data = _matrix(K, P, 31 + K, cuda)
    D = ops.pairwise_l2(data[:, :P], "reference").cpu().numpy()
    assert np.array_equal(D, normref.distance_matrix(X.numpy()))


@pytest.mark.parametrize("K,P,on,form", [(65, 4099, "1", "wg"), (100, 20_011, "1", "wg"), (130, 65_537, "1", "wg"),
                                         (200, 8, "1", "wg"), (300, 20_011, "1", "wg"), (480, 3001, "", "wg"),
                                         (512, 20_011, "", "wg"), (520, 1007, "", "wg"), (512, 2053, "0", "wg"),
                                         (100, 20_011, "1", "sg"), (520, 1007, "", "sg"),
                                         (65, 4099, "1", "4"), (300, 20_011, "1", "4"), (520, 1007, "", "4"),
                                         (70, 4099, "1", "8"), (130, 20_011, "1", "8"), (520, 1007, "", "8")])
def test_reference_mode_sgpr_tiles(cuda, knob, K, P, on, form):
    """The throughput form (quad_transpose_kernel, then ref_chain_w_kernel: 4-wave
    workgroups of 8 I rows per wave x one 64-row J block, both staged through
    LDS; FLR_REF_SGPR_FORM=sgpr: x_i as SGPR operands instead; =wave: the
    one-wave ref_chain_s_kernel with 4 or FLR_REF_SGPR_ROWS=8 I rows), K >= 480, forced on below it
    (FLR_REF_SGPR=1) and off at K = 512 (=0): D bit-identical to the C
    restatement, ragged J blocks and workgroups (K not a multiple of 64) and a
    single step (P = 8) included."""
    if on:
        knob("FLR_REF_SGPR", on)
    if form == "sg":
        knob("FLR_REF_SGPR_FORM", "sgpr")
    elif form != "wg":
        knob("FLR_REF_SGPR_FORM", "wave")
        knob("FLR_REF_SGPR_ROWS", form)
    X, data = _matrix(K, P, 57 + K, cuda)
    D = ops.pairwise_l2(data[:, :P], "reference").cpu().numpy()
    assert np.array_equal(D, normref.distance_matrix(X.numpy()))


@pytest.mark.parametrize("K,form", [(96, "wg"), (520, "wg"), (96, "4"), (100, "8")])
def test_reference_mode_sgpr_segmented(cuda, knob, K, form):
    """The throughput form over a workspace of 1024 chain steps: several
    segments, each chain continued from A (first = 0), the last segment
    zero-filled to 512 steps; D bit-identical to the one-segment call."""
    import ctypes
    from flr import _capi
    knob("FLR_REF_SGPR", "1")
    if form == "sg":
        knob("FLR_REF_SGPR_FORM", "sgpr")
    elif form != "wg":
        knob("FLR_REF_SGPR_FORM", "wave")
        knob("FLR_REF_SGPR_ROWS", form)
    P = 8 * 2900 + 3
    X, data = _matrix(K, P, 23 + K, cuda)
    lib = _capi.lib()
    Kp = (K + 63) // 64 * 64
    a_bytes = (8 * K * K * 4 + 255) // 256 * 256
    nbytes = a_bytes + Kp * 32 * 1024 + 4096 + 12 * Kp * 16
    assert nbytes < int(lib.flr_pairwise_l2_reference_workspace(K, P))
    ws = torch.empty(nbytes + 256, dtype=torch.uint8, device=cuda)
    wp = (ws.data_ptr() + 255) // 256 * 256
    D = torch.empty((K, K), dtype=torch.float64, device=cuda)
    st = torch.cuda.current_stream().cuda_stream
    _capi.call("flr_pairwise_l2_reference", data.data_ptr(), K, P, data.stride(0), D.data_ptr(), wp, nbytes, 0, 1,
               st)
    torch.cuda.synchronize()
    want = ops.pairwise_l2(data[:, :P], "reference").cpu().numpy()
    assert np.array_equal(D.cpu().numpy(), want)
    if K < 128:
        assert np.array_equal(want, normref.distance_matrix(X.numpy()))


@pytest.mark.parametrize("path", golden_files("c3krum"), ids=lambda p: p.split("/")[-1])
def test_reference_mode_c3_fixtures(cuda, path):
    """The C3-shaped fixtures (K = 128, f = 25 sign-flipped, multi_k = 64):
    D equals the fixture's reference fp32 norms bit for bit, and the Krum
    outputs (selected, rejected, the Multi-Krum mean) are the fixture's."""
    fx = load_golden(path)
    K, P, f, mk = (int(fx[k]) for k in ("K", "P", "f", "multi_k"))
    X = update_matrix(K, P, f=f, seed=int(fx["seed"]), device="cpu")[:, :P]
    data = torch.zeros((K, padded_ld(P)), dtype=torch.float32, device=cuda)
    data[:, :P] = X.to(cuda)
    d = KrumDefense({"num_malicious": f, "multi_k": mk, "pairwise_method": "reference"})
    flat = d.aggregate_flat(ClientMatrix(data, P, [(P,)]), [1] * K)
    assert np.array_equal(d.distances.cpu().numpy(), fx["dist"])
    assert d.client_scores == fx["scores"].tolist()
    assert d.selected_clients == fx["selected"].tolist()
    assert d.rejected_clients == fx["rejected"].tolist()
    assert hashlib.sha256(flat.cpu().numpy().tobytes()).hexdigest() == str(fx["agg_sha256"])


def test_reference_mode_round_engine(cuda):
    """A round with Krum in the reference mode: the engine hands the defense
    whole rows in the trainer's coordinate order with
    the map of each reference coordinate's column, and D / selection /
    rejection equal the oracle's torch.norm loop on the rows in the
    reference's order."""
    from flr.models.multimodal import TINY
    from flr.round import RoundConfig, RoundEngine
    from flr.train import TrainConfig
    K, f = 12, 2
    rc = RoundConfig(num_clients=K, batch=4, defense="krum", num_attackers=f,
                     defense_cfg={"pairwise_method": "reference"})
    eng = RoundEngine(TINY, rc, TrainConfig(local_steps=2), cuda)
    assert eng.train_order  # one GPU: the one coordinate slice is the whole matrix
    eng.run_round()
    eng.defense.publish()
    P = eng.trainer.P
    rows = [eng.trainer.to_torch_order(eng.trainer.X.data[k, :P]).cpu() for k in range(K)]
    _, scores, sel, rej, dist = orc.krum([[r] for r in rows], f, K // 2)
    assert np.array_equal(eng.defense.distances.cpu().numpy(), dist)
    assert eng.defense.client_scores == [float(s) for s in scores]
    assert eng.defense.selected_clients == sel and eng.defense.rejected_clients == rej


@pytest.mark.parametrize("K,blocks", [
    (16, [(5, 64, 64, 9), (36_869 + 7, 64, 3, 9), (36_869 + 7 + 1728 + 3, 128, 64, 1)]),
    (33, [(0, 128, 64, 9), (73_728 + 1, 40, 24, 9)]),
    (128, [(100, 512, 256, 9), (100 + 1_179_648 + 13, 64, 64, 1)]),
    (16, [(0, 64, 64, 9), (36_864, 128, 64, 1), (45_056, 64, 128, 9), (118_784 + 32, 256, 128, 9)]),
    (24, [(32, 128, 128, 9), (32 + 147_456, 256, 128, 1)])])
def test_reference_mode_tap_major_blocks(cuda, K, blocks):
    """A training-order matrix (convolution weights stored tap-major, column
    off + (t * Cin + ci) * Cout + co for reference coordinate
    off + (co * Cin + ci) * KK + t) read through flr_pairwise_l2_reference_tap:
    D bit-identical to the reference-order matrix's.  Blocks at odd offsets
    (chain steps shared with the plain columns beside them), partial 32-channel
    tiles, KK 9 and 1, a block reaching the tail; blocks at multiples of 32
    coordinates (every one of C3's: the 16-B store form of the dense writes)."""
    P = max(o + co * ci * kk for o, co, ci, kk in blocks) + 5
    X, data = _matrix(K, P, 13 + K, cuda)
    train = data.clone()
    for o, co, ci, kk in blocks:
        w = data[:, o:o + co * ci * kk].reshape(K, co, ci, kk)
        train[:, o:o + co * ci * kk] = w.permute(0, 3, 2, 1).reshape(K, -1)
    D = ops.pairwise_l2(train[:, :P], "reference", tap_blocks=blocks).cpu().numpy()
    want = ops.pairwise_l2(data[:, :P], "reference").cpu().numpy()
    assert np.array_equal(D, want)
    if K <= 33:
        assert np.array_equal(D, normref.distance_matrix(X.numpy()))


def test_reference_mode_tap_blocks_reach_the_tail(cuda):
    """A tap-major block ending at P with P % 8 != 0: the tail coordinates'
    columns come from the block."""
    K, blocks = 9, [(3, 64, 8, 9)]
    P = 3 + 64 * 8 * 9
    X, data = _matrix(K, P, 99, cuda)
    train = data.clone()
    w = data[:, 3:P].reshape(K, 64, 8, 9)
    train[:, 3:P] = w.permute(0, 3, 2, 1).reshape(K, -1)
    D = ops.pairwise_l2(train[:, :P], "reference", tap_blocks=blocks).cpu().numpy()
    assert np.array_equal(D, normref.distance_matrix(X.numpy()))


def test_reference_mode_tap_blocks_segmented(cuda):
    """A workspace for 2048 chain steps: four segments (3 x 2048 and a last one
    of 356 steps zero-filled to 512), tap blocks crossing the segment
    boundaries (the clipped runs: the tap kernel's general write loop), one
    with Cin * KK not a multiple of 8 and a partial ci tile (the dense write
    form for its whole tiles): D bit-identical to the reference-order
    matrix's through the whole workspace."""
    import ctypes
    from flr import _capi
    K = 16
    blocks = [(5, 64, 64, 9), (36_869 + 3, 64, 3, 9), (36_869 + 3 + 1728 + 1, 32, 40, 9)]
    P = 8 * 6500 + 5
    assert max(o + co * ci * kk for o, co, ci, kk in blocks) <= P
    X, data = _matrix(K, P, 21, cuda)
    train = data.clone()
    for o, co, ci, kk in blocks:
        w = data[:, o:o + co * ci * kk].reshape(K, co, ci, kk)
        train[:, o:o + co * ci * kk] = w.permute(0, 3, 2, 1).reshape(K, -1)
    lib = _capi.lib()
    a_bytes = (8 * K * K * 4 + 255) // 256 * 256
    nbytes = a_bytes + K * 32 * 2048 + 4096
    assert nbytes < int(lib.flr_pairwise_l2_reference_workspace(K, P))
    ws = torch.empty(nbytes + 256, dtype=torch.uint8, device=cuda)
    wp = (ws.data_ptr() + 255) // 256 * 256
    taps = [v for b in blocks for v in b]
    tarr = (ctypes.c_int64 * len(taps))(*taps)
    D = torch.empty((K, K), dtype=torch.float64, device=cuda)
    st = torch.cuda.current_stream().cuda_stream
    _capi.call("flr_pairwise_l2_reference_tap", train.data_ptr(), K, P, train.stride(0), ctypes.addressof(tarr),
               len(blocks), D.data_ptr(), wp, nbytes, 0, 1, st)
    torch.cuda.synchronize()
    want = ops.pairwise_l2(data[:, :P], "reference").cpu().numpy()
    assert np.array_equal(D.cpu().numpy(), want)
    assert np.array_equal(want, normref.distance_matrix(X.numpy()))


@pytest.mark.parametrize("K,blocks,masks,nneg", [
    (16, [(5, 64, 64, 9), (36_869 + 7, 64, 3, 9), (36_869 + 7 + 1728 + 3, 128, 64, 1)],
     [0b110101011, 0b000010000, 0b1], 3),
    (33, [(0, 128, 64, 9), (73_728 + 1, 40, 24, 9)], [0b011111110, 0b000000011], 0),
    (9, [(3, 64, 8, 9)], [0b000011111], 9)])
def test_reference_mode_deferred_dead_taps(cuda, K, blocks, masks, nneg):
    """flr_pairwise_l2_reference_tap_dead (the round engine's FLR_TC_DEFER_DEAD
    rounds): the dead-tap slabs are NaN in X and read from the global vector
    instead, negated on rows < nneg — D bit-identical to the call on the matrix
    with those slabs filled as flr_resnet_gru_fill_dead fills them."""
    P = max(o + co * ci * kk for o, co, ci, kk in blocks) + (5 if K != 9 else 0)
    X, data = _matrix(K, P, 31 + K, cuda)
    train = data.clone()
    for o, co, ci, kk in blocks:
        w = data[:, o:o + co * ci * kk].reshape(K, co, ci, kk)
        train[:, o:o + co * ci * kk] = w.permute(0, 3, 2, 1).reshape(K, -1)
    g = torch.randn(P, generator=torch.Generator().manual_seed(5)).to(cuda)
    filled, holes = train.clone(), train.clone()
    for (o, co, ci, kk), m in zip(blocks, masks):
        for t in range(kk):
            if m >> t & 1:
                sl = slice(o + t * ci * co, o + (t + 1) * ci * co)
                filled[:, sl] = g[sl]
                filled[:nneg, sl] = -g[sl]
                holes[:, sl] = float("nan")
    D = ops.pairwise_l2(holes[:, :P], "reference", tap_blocks=blocks, dead=(masks, g, nneg)).cpu().numpy()
    want = ops.pairwise_l2(filled[:, :P], "reference", tap_blocks=blocks).cpu().numpy()
    assert np.isfinite(want).all() and np.array_equal(D, want)


def test_reference_mode_dead_tap_in_the_tail_rejected(cuda):
    """The finish kernel reads the last P mod 8 coordinates from X itself: a
    dead tap among them is refused (the engine then writes the slabs first)."""
    from flr._capi import FlrError
    K, blocks = 9, [(3, 64, 8, 9)]
    P = 3 + 64 * 8 * 9  # tail: block columns of taps 6, 7, 8
    _, data = _matrix(K, P, 3, cuda)
    g = torch.zeros(P, device=cuda)
    with pytest.raises((FlrError, ValueError)):
        ops.pairwise_l2(data[:, :P], "reference", tap_blocks=blocks, dead=([1 << 8], g, 0))
    with pytest.raises((FlrError, ValueError)):  # a bit past the block's taps
        ops.pairwise_l2(data[:, :P], "reference", tap_blocks=blocks, dead=([1 << 9], g, 0))
