"""Batch sharding across GPUs.

Payloads are independent, so a batch shards by payload index with no data-path
collective: rank g of G owns bodies [g*n/G, (g+1)*n/G).  RCCL (torch.distributed
"nccl") is used only as the launch/complete barrier and to take the max time
over ranks.  Pure host logic; covered by world_size-2 gloo tests on CPU.
"""
from __future__ import annotations


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of n bodies for `rank` of `world`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return n * rank // world, n * (rank + 1) // world


def rank_seed(base_seed: int, rank: int) -> int:
    """Per-rank synthetic-data seed (config C3: seed 0x5EED0005 + rank)."""
    return (base_seed + rank) & (2**64 - 1)


def barrier(dist, device=None):
    """Launch/complete barrier: a 1-element all-reduce on the communicator's
    backend (RCCL over xGMI for "nccl"), then wait for it."""
    import torch

    t = torch.ones(1, dtype=torch.int32, device=device)
    dist.all_reduce(t)
    if device is not None and str(device).startswith("cuda"):
        torch.cuda.synchronize(device)
    return int(t.item())


def max_over_ranks(dist, value: float, device=None) -> float:
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, value: int, device=None) -> int:
    import torch

    t = torch.tensor([value], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
