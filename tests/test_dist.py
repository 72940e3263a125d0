"""Multi-rank path on CPU: world_size-2 gloo processes exercise the payload-index
sharding, the barrier and the max/sum-over-ranks reductions bench.py uses.  The
per-shard CRCs come from the oracle here (test stand-in for the device kernel);
gathering the shards must reproduce the whole batch exactly."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from rpc_amd.shard import max_over_ranks, rank_seed, shard_range, sum_over_ranks, barrier


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        from oracle import oracle
        n, L = 1000, 300
        data = oracle.splitmix_bytes(n * L, 42)  # every rank sees the same logical batch
        lo, hi = shard_range(n, rank, world)
        mine = oracle.crc32_uniform(data[lo * L:hi * L], hi - lo, L)
        parts = [None] * world
        dist.all_gather_object(parts, (lo, hi, mine.tolist()))
        assert barrier(dist) == world
        t = max_over_ranks(dist, 1.0 + rank)
        tot = sum_over_ranks(dist, hi - lo)
        if rank == 0:
            full = np.concatenate([np.array(p[2], dtype=np.uint32) for p in sorted(parts)])
            q.put((full.tolist(), oracle.crc32_uniform(data, n, L).tolist(), t, tot,
                   [tuple(p[:2]) for p in sorted(parts)]))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    for n in [0, 1, 7, 1000, 1 << 20]:
        for world in [1, 2, 3, 4, 8]:
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_rank_seed():
    assert rank_seed(0x5EED0005, 3) == 0x5EED0008


def test_gloo_world2_shards_reassemble():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, want, tmax, tot, spans = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert full == want
    assert tmax == 2.0 and tot == 1000
    assert spans == [(0, 500), (500, 1000)]
