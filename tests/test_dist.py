"""Multi-rank path: world_size-2 gloo processes exercise the payload-index sharding,
the barrier and the max/sum-over-ranks reductions bench.py uses.  On the CPU the
per-shard CRCs come from the oracle (the shard arithmetic is what is under test);
the GPU test runs the HIP kernel per shard (two ranks on cuda:0) and checks the
gathered CRCs against the oracle."""
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


def _hip_worker(rank, world, port, q):
    """One rank: its payload-index shard of a batch through the HIP kernel on cuda:0
    (two gloo ranks share the box's one GPU), gathered to rank 0."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        import rpc_amd
        torch.cuda.set_device(0)
        n, L = 30011, 1500  # uneven shards, partial rows
        lo, hi = shard_range(n, rank, world)
        x = torch.empty((n * L + 7) // 8 * 8, dtype=torch.uint8, device="cuda:0")
        rpc_amd.fill_random(x, 0x5EED0005)  # every rank sees the same logical batch
        mine = rpc_amd.device_uniform(x[lo * L:hi * L], hi - lo, L).cpu().numpy().view(np.uint32)
        parts = [None] * world
        dist.all_gather_object(parts, (lo, hi, mine.tolist()))
        if rank == 0:
            from oracle import oracle
            full = np.concatenate([np.array(p[2], dtype=np.uint32) for p in sorted(parts)])
            want = oracle.crc32_uniform(x.cpu().numpy(), n, L)
            q.put((int(np.count_nonzero(full != want)), len(full), rpc_amd.device_info()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gloo_world2_hip_shards_match_oracle():
    """the multi-rank test must run the HIP path per shard, not the oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hip_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    bad, n, info = q.get(timeout=110)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert n == 30011 and bad == 0
    assert "gfx950" in info
