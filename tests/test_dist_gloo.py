"""CPU (gloo, world_size 2): client sharding + the one all-gather of a round.

The gathered client matrix must equal what a single process holds (global
client order), and the replicated aggregation then sees identical input on
every rank — checked here with the oracle as the aggregator (the HIP kernels
need a GPU; tests/test_gpu_aggregation.py covers them)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flr import dist as fdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, K, P, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = fdist.shard(K, world, rank)
    full_ref = torch.arange(K * P, dtype=torch.float32).view(K, P)
    local = full_ref[lo:hi].clone()
    full = torch.zeros(K, P)
    fdist.allgather_rows(local, full)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import aggregation as orc
    ups = [[full[i]] for i in range(K)]
    agg, _, sel, _, _ = orc.krum(ups, 1, K // 2)
    t = fdist.max_over_ranks(float(rank), torch.device("cpu"))
    q.put((rank, torch.equal(full, full_ref), sel, agg[0].sum().item(), t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_allgather_and_replicated_aggregation(world):
    K, P = 8, 37
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, P, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] for r in res)
    assert len({tuple(r[2]) for r in res}) == 1 and len({r[3] for r in res}) == 1
    assert all(r[4] == world - 1 for r in res)


def test_shard_ranges():
    assert fdist.shard(128, 8, 3) == (48, 64)
    assert [fdist.shard(512, 8, r) for r in (0, 7)] == [(0, 64), (448, 512)]
    with pytest.raises(ValueError):
        fdist.shard(10, 3, 0)


# ---------------- coordinate-sharded exchange (flr.shard) ----------------

def _shard_worker(rank, world, port, K, P, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import aggregation as orc
    from flr.shard import Comm, CoordExchange
    g = torch.Generator().manual_seed(3)
    full_ref = torch.randn(K, P, generator=g)
    lo, hi = fdist.shard(K, world, rank)
    local = torch.zeros(hi - lo, P + 11)  # padded row stride, like the trainer's matrix
    local[:, :P] = full_ref[lo:hi]
    xchg = CoordExchange(K, hi - lo, P, torch.device("cpu"), Comm())
    cs = xchg.exchange(local)
    b, e = cs.begin, cs.end
    ok_slice = torch.equal(cs.X, full_ref[:, b:e])
    # coordinate-wise aggregation of the range (oracle as the aggregator), then the P-vector all-gather
    med = orc.median([[cs.X[i].clone()] for i in range(K)])[0]
    out = torch.empty(P)
    cs.gather_vector(med, out)
    ref = orc.median([[full_ref[i]] for i in range(K)])[0]
    q.put((rank, ok_slice, torch.equal(out, ref), (b, e)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_coordinate_exchange(world):
    """The exchange's row pieces (batched p2p, no pack copy) over gloo on CPU
    ranks: every rank's slice is all K clients' columns of its range."""
    K, P = 8, 64 * 8 * 5 + 29
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, K, P, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs])
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] and r[2] for r in res), res
    ranges = [r[3] for r in res]
    assert ranges[0][0] == 0 and ranges[-1][1] == P
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))


def test_coord_plan_covers_vector():
    from flr.shard import CoordPlan, slice_chunks
    for P in (1, 63, 64 * 8, 64 * 8 * 3 + 7, 11_800_394):
        for world in (1, 2, 4, 8):
            plan = CoordPlan(P, world)
            spans = [plan.coords(r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == P
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert all(e - b <= plan.ld for b, e in spans) and plan.ld % 64 == 0
            # rank ranges are unions of canonical slices (G-invariant records)
            for r in range(world):
                q0, q1 = plan.slices(r)
                assert plan.chunks(r) == (slice_chunks(P, q0)[0], slice_chunks(P, q1 - 1)[1])
    with pytest.raises(ValueError):
        CoordPlan(100, 3)
