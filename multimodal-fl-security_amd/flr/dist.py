"""Client sharding over the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
GPU g owns the contiguous clients [g*K/G, (g+1)*K/G), so global client ids,
attacker ids (0..f-1) and the row order of the client matrix mean the same at
every G.  The round's data exchange after local training is one of two
(flr.round, RoundConfig.exchange):
* "alltoall" (the default for the coordinate-wise and Krum defenses,
  flr.shard): one all-to-all hands GPU g all K clients' values of its
  coordinate range; each GPU aggregates its range (Krum: plus small
  collectives of the pivot sample, the tail term and the per-slice Gram
  records) and one all-gather of the aggregated slices rebuilds the global
  model;
* "allgather" (defenses that need whole rows): one all-gather of the
  (K/G)×P row blocks (allgather_rows below) gives every GPU the full K×P
  matrix in global client order and the aggregation runs replicated.
Both use deterministic fixed-order kernels, so every GPU ends the round with
the bit-identical global model at every G.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def env_world() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init(backend: str = "nccl") -> Tuple[int, int, int]:
    rank, world, local = env_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard(num_clients: int, world: int, rank: int) -> Tuple[int, int]:
    if num_clients % world != 0:
        raise ValueError(f"{num_clients} clients do not split evenly over {world} GPUs")
    per = num_clients // world
    return rank * per, (rank + 1) * per


def allgather_rows(local: torch.Tensor, full: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> None:
    """full[K, ld] <- concatenation over ranks of local[K/G, ld] (rank order)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        if full.data_ptr() != local.data_ptr():
            full.copy_(local)
        return
    if dist.get_backend(group) == "gloo" and full.is_cuda:
        # gloo has no device collectives: stage through host memory (the
        # world_size > 1 rehearsal on one GPU); RCCL takes the device tensors
        hf = full.cpu()
        dist.all_gather_into_tensor(hf, local.contiguous().cpu(), group=group)
        full.copy_(hf)
        return
    dist.all_gather_into_tensor(full, local.contiguous(), group=group)


def barrier() -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def max_over_ranks(value: float, device) -> float:
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    # gloo reduces host tensors; RCCL device tensors
    t = torch.tensor([value], dtype=torch.float64,
                     device="cpu" if dist.get_backend() == "gloo" else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
