"""GPU: the coordinate-sharded exchange (flr.shard).

Bars: Krum's distance matrix from the per-slice phases, composed over any
split of the canonical slices, is BIT-identical to flr_pairwise_l2 on the
whole matrix; the aggregates of a sharded round are bit-identical to the
one-GPU round (2 ranks on one GPU over gloo, CUDA tensors staged through the
host — the RCCL path runs the same code with device collectives)."""
import os
import socket

import numpy as np
import pytest
import torch

from flr import _capi, ops
from flr.defenses import get_defense
from flr.matrix import ClientMatrix
from flr.shard import PW_SLICES, Comm, CoordPlan, CoordSlice, slice_chunks
from flr.workload import update_matrix

pytestmark = pytest.mark.gpu


def _phases(X_full, K, P, world):
    """The five phases of include/flr.h with the collectives done by hand."""
    lib = _capi.lib()
    dev = X_full.device
    plan = CoordPlan(P, world)
    ld = plan.ld
    st = torch.cuda.current_stream().cuda_stream
    parts = []
    for r in range(world):  # what rank r would receive from the all-to-all
        b, e = plan.coords(r)
        part = torch.zeros((K, ld), dtype=torch.float32, device=dev)
        part[:, : e - b] = X_full[:, b:e]
        parts.append(part)
    S = int(lib.flr_pairwise_sample_len(P))
    Xs = torch.zeros((K, S), dtype=torch.float32, device=dev)
    for r in range(world):
        c0, c1 = plan.chunks(r)
        xs_r = torch.full((K, S), float("nan"), device=dev)
        _capi.call("flr_pairwise_sample", parts[r].data_ptr(), K, ld, P, c0, c1, xs_r.data_ptr(), st)
        Xs += xs_r
    nsl = PW_SLICES // world
    nbytes = int(lib.flr_pairwise_sliced_workspace(K, P, nsl))
    ws, wp = ops._ws(nbytes, dev)
    pivot = torch.empty(int(lib.flr_pairwise_pivot_len()), dtype=torch.int32, device=dev)
    _capi.call("flr_pairwise_pivot", Xs.data_ptr(), K, P, pivot.data_ptr(), wp, nbytes, st)
    glen = int(lib.flr_pairwise_gsum_len(K))
    gsum = torch.empty((PW_SLICES, glen), dtype=torch.float64, device=dev)
    tail = torch.zeros((K, K), dtype=torch.float64, device=dev)
    for r in range(world):
        q0, q1 = plan.slices(r)
        _capi.call("flr_pairwise_gram_slices", parts[r].data_ptr(), K, ld, P, q0, q1, pivot.data_ptr(),
                   gsum[q0].data_ptr(), wp, nbytes, st, None, None)
        b, e = plan.coords(r)
        t0 = min(max((P // 64) * 64 - b, 0), e - b)
        t = torch.empty((K, K), dtype=torch.float64, device=dev)
        _capi.call("flr_pairwise_tail", parts[r].data_ptr(), K, ld, t0, e - b, t.data_ptr(), st)
        tail += t
    D = torch.empty((K, K), dtype=torch.float64, device=dev)
    _capi.call("flr_pairwise_finish", gsum.data_ptr(), tail.data_ptr(), K, D.data_ptr(), st)
    return D


@pytest.mark.parametrize("K,P", [(16, 64 * 8 * 3 + 5), (40, 4099), (128, 100_000 + 37), (130, 20_000),
                                 (9, 70)])
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_sharded_distances_bit_identical(cuda, K, P, world):
    X = update_matrix(K, P, f=K // 5, seed=K * 7 + P, device=cuda)
    D_full = ops.pairwise_l2(X[:, :P], "gram")
    D = _phases(X, K, P, world)
    assert torch.equal(D, D_full)


def test_slice_chunks_match_library():
    lib = _capi.lib()
    import ctypes
    for P in (0, 63, 64, 511, 512, 4099, 11_800_394):
        for q in range(PW_SLICES):
            a, b = ctypes.c_int64(), ctypes.c_int64()
            assert lib.flr_pw_slice_chunks(P, q, ctypes.byref(a), ctypes.byref(b)) == 0
            assert (a.value, b.value) == slice_chunks(P, q)


@pytest.mark.parametrize("name,cfg", [("krum", {"num_malicious": 3, "multi_k": 8, "pairwise_method": "gram"}),
                                      ("krum", {"num_malicious": 3, "multi_k": 1, "pairwise_method": "gram"}),
                                      ("trimmed_mean", {"trim_ratio": 0.2}), ("median", {}), ("fedavg", {})])
def test_sharded_defense_world1_equals_flat(cuda, name, cfg):
    """World 1: the sharded entry point on the whole matrix == aggregate_flat."""
    K, P = 16, 5000
    X = update_matrix(K, P, f=3, seed=5, device=cuda)
    cm = ClientMatrix(X, P, [torch.Size([P])])
    ne = list(range(1, K + 1))
    d1 = get_defense(name, dict(cfg))
    ref = d1.aggregate_flat(cm, ne)
    d2 = get_defense(name, dict(cfg))
    cs = CoordSlice(X, CoordPlan(P, 1), 0, Comm())
    out = torch.empty(P, device=cuda)
    cs.gather_vector(d2.aggregate_sharded(cs, ne), out)
    assert torch.equal(out, ref[:P])
    if name == "krum":
        assert d1.selected_clients == d2.selected_clients


# ---------------- 2 ranks on one GPU (gloo) vs 1 rank ----------------

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _round_worker(rank, world, port, defense, q, exchange="alltoall", spec="TINY"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from flr.models.multimodal import TINY
    from flr.round import RoundConfig, RoundEngine
    from flr.train import TrainConfig
    cfg = {"trim_ratio": 0.2} if defense == "trimmed_mean" else {"pairwise_method": "gram"} if defense == "krum" else {}
    if defense == "krum_ref":  # the reference-exact distances: pair tiles split over the ranks
        defense, cfg = "krum", {"pairwise_method": "reference"}
    rc = RoundConfig(num_clients=8, batch=4, defense=defense, num_attackers=1, exchange=exchange, defense_cfg=cfg)
    eng = RoundEngine(TINY if spec == "TINY" else MID, rc, TrainConfig(local_steps=2), torch.device("cuda:0"),
                      rank, world)
    for _ in range(2):
        g = eng.run_round()
    torch.cuda.synchronize()
    sel = None
    if defense == "krum":
        eng.defense.publish()
        sel = (eng.defense.selected_clients, eng.defense.distances.cpu().numpy().tobytes())
    q.put((rank, g.cpu().numpy(), sel, eng.train_order,
           eng.xchg.plan.coords(rank) if eng.xchg is not None else None))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _run(world, defense, exchange="alltoall", spec="TINY"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_round_worker, args=(r, world, port, defense, q, exchange, spec)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("defense,exchange", [("krum", "alltoall"), ("trimmed_mean", "alltoall"),
                                              ("krum", "allgather"), ("norm_bounding", "allgather")])
def test_sharded_round_two_ranks_equals_one(cuda, defense, exchange):
    """Both exchanges; 'allgather' is the path of every defense without a
    coordinate-sharded form (norm_bounding here), gloo-staged through the host."""
    one = _run(1, defense, exchange)
    two = _run(2, defense, exchange)
    assert np.array_equal(one[0][1], two[0][1]) and np.array_equal(two[0][1], two[1][1])
    assert one[0][2] == two[0][2] == two[1][2]


@pytest.mark.parametrize("defense,exchange", [("krum", "alltoall"), ("krum", "allgather"),
                                              ("median", "alltoall")])
def test_sharded_round_four_ranks_equals_one(cuda, defense, exchange):
    """World 4 (the K/G = 2 clients per rank of the C4/C5 partition at this
    size): every rank's global model and Krum selection equal the one-rank
    round bit for bit, for both exchanges."""
    one = _run(1, defense, exchange)
    four = _run(4, defense, exchange)
    for r in range(4):
        assert np.array_equal(one[0][1], four[r][1]), r
        assert one[0][2] == four[r][2]


@pytest.mark.parametrize("defense,exchange", [("krum", "alltoall"), ("krum", "allgather"), ("median", "alltoall"),
                                              ("krum_ref", "allgather"), ("krum_ref", "alltoall")])
def test_sharded_round_eight_ranks_equals_one(cuda, defense, exchange):
    """World 8, the node's GPU count (one client per rank at K = 8): every
    rank's global model, Krum selection and distance matrix equal the one-rank
    round bit for bit, for both exchanges and for the reference-exact distances
    — whole rows with their pair tiles split over the ranks (one exact
    all-reduce of D), or coordinate slices whose chains run through the ranks
    in order (the default exchange of the benchmarked C3 path)."""
    one = _run(1, defense, exchange)
    eight = _run(8, defense, exchange)
    for r in range(8):
        assert np.array_equal(one[0][1], eight[r][1]), r
        assert one[0][2] == eight[r][2], r


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("exchange", ["allgather", "alltoall"])
def test_reference_distances_split_over_ranks(cuda, world, exchange):
    """The reference-exact Krum distances over 2 / 4 ranks: pair tiles split
    (allgather) or the chains handed from rank to rank over the coordinate
    slices (alltoall): bit-identical to one rank."""
    one = _run(1, "krum_ref", exchange)
    many = _run(world, "krum_ref", exchange)
    for r in range(world):
        assert np.array_equal(one[0][1], many[r][1]) and one[0][2] == many[r][2], r


def _mid_spec():
    from flr.models.multimodal import ModelSpec
    # 64-wide stages: tap-major blocks (up to 36,864 coordinates) longer than
    # the canonical boundaries' distance to them at every world size
    return ModelSpec(widths=(64, 64, 64, 64), blocks=(1, 1, 1, 1), vocab=50, embed=8, hidden=16, fusion=16,
                     dropout=0.0)


MID = _mid_spec()


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("spec", ["TINY", "MID"])
def test_reference_training_order_over_ranks(cuda, spec, world):
    """The reference-exact Krum distances of a TRAINING-ORDER round (tap-major
    convolution weights, no torch-order copy) over 2 / 4 / 8 ranks: the rank
    boundaries are moved off the tap-major blocks (shard.aligned_bounds; at
    MID they differ from the canonical slices'), every rank keeps
    train_order, and the global model, selection and distance matrix equal
    the one-rank round's bit for bit."""
    one = _run(1, "krum_ref", "alltoall", spec)
    assert one[0][3] is True
    many = _run(world, "krum_ref", "alltoall", spec)
    for r in range(world):
        assert many[r][3] is True, r
        assert np.array_equal(one[0][1], many[r][1]) and one[0][2] == many[r][2], r
    P = one[0][1].size
    moved = any(many[r][4] != CoordPlan(P, world).coords(r) for r in range(world))
    assert moved == (spec == "MID")
