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
