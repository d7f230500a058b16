"""Where do a 1-rank and a 2-rank sharded round (gloo, one GPU) diverge?
Per round: the trained client rows, Krum's selection and the global vector.
Writes gpurun_out/diag_shard.log."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, graph, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", FLR_GRAPH=graph)
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from flr.models.multimodal import TINY
    from flr.round import RoundConfig, RoundEngine
    from flr.train import TrainConfig
    rc = RoundConfig(num_clients=8, batch=4, defense="krum", num_attackers=1, exchange="alltoall")
    eng = RoundEngine(TINY, rc, TrainConfig(local_steps=2), torch.device("cuda:0"), rank, world)
    out = []
    for _ in range(2):
        g0 = eng.global_flat.clone()
        g = eng.run_round()
        torch.cuda.synchronize()
        eng.defense.publish()
        D = eng.defense.distances
        out.append((g0.cpu().numpy(), eng.trainer.X.X.cpu().numpy(), list(eng.defense.selected_clients),
                    g.cpu().numpy().copy(), None if D is None else D.cpu().numpy()))
    q.put((rank, out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run(world, graph):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, world, port, graph, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=200) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    return res


def main():
    import numpy as np
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    f = open(os.path.join(ROOT, "gpurun_out", "diag_shard.log"), "w")
    for graph in ("1", "0"):
        one = run(1, graph)[0][1]
        two = run(2, graph)
        for r in range(2):
            g0a, Xa, sa, ga, Da = one[r]
            X2 = np.concatenate([two[0][1][r][1], two[1][1][r][1]])
            sb, gb, Db = two[0][1][r][2], two[0][1][r][3], two[0][1][r][4]
            gin = np.abs(g0a - two[0][1][r][0]).max()
            xd = np.abs(Xa - X2).max(axis=1).tolist()
            dd = None if Da is None or Db is None else np.abs(Da - Db).max()
            print(f"graph={graph} round {r}: |g_in diff| {gin:.3e} |X diff| per client {xd} sel1 {sa} sel2 {sb} "
                  f"|D diff| {dd} |g diff| {np.abs(ga - gb).max():.3e} "
                  f"rank1 g == rank0 g {np.array_equal(gb, two[1][1][r][3])}", file=f, flush=True)
    print("done", file=f, flush=True)


if __name__ == "__main__":
    main()
