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


def min_over_ranks(dist, value: float, device=None) -> float:
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def sum_over_ranks(dist, value: int, device=None) -> int:
    import torch

    t = torch.tensor([value], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


# ---- one large body across GPUs (optional for C4) -------------
# A body too large for one GPU's share of the work is cut into contiguous byte
# ranges, one per rank; each rank CRCs its range on its own GPU
# (rpc_crc32_device_large), and the ONE exchange step is an all-gather of the
# 4-B partials and their lengths, folded in body order with zlib crc32_combine
# semantics: crc(A || B) = crc32_combine(crc(A), crc(B), len(B)).

def large_body_range(length: int, rank: int, world: int, align: int = 4096) -> tuple[int, int]:
    """[lo, hi) bytes of one body for `rank`: balanced, cut at multiples of
    `align` (so every range but the last is a whole number of rows)."""
    if align <= 0:
        raise ValueError("align must be positive")
    units = (length + align - 1) // align
    lo, hi = shard_range(units, rank, world)
    return min(lo * align, length), min(hi * align, length)


def fold_partials(parts, combine) -> int:
    """CRC of the concatenation of ranges whose (crc, length) pairs are `parts`,
    in body order.  `combine` is zlib's crc32_combine (rpc_crc32_combine)."""
    crc = 0  # CRC of the empty prefix; combine(0, c, n) == c
    for c, n in parts:
        crc = combine(crc, int(c) & 0xFFFFFFFF, int(n))
    return crc


def sharded_large_crc(dist, local_crc: int, local_len: int, device=None, combine=None) -> int:
    """Every rank passes the CRC of its range of the body (ranges in rank
    order); returns the whole body's CRC on every rank.  One all_gather of
    (crc, len) per rank -- RCCL over xGMI with the "nccl" backend."""
    import torch

    if combine is None:
        import rpc_amd

        combine = rpc_amd.crc32_combine
    mine = torch.tensor([int(local_crc) & 0xFFFFFFFF, int(local_len)], dtype=torch.int64, device=device)
    parts = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, mine)
    return fold_partials([(int(p[0]), int(p[1])) for p in parts], combine)
