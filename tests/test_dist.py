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

from rpc_amd.shard import (barrier, fold_partials, large_body_range, max_over_ranks, rank_seed, shard_range,
                           sharded_large_crc, sum_over_ranks)


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


# ---- one large body across ranks (optional for C4) ---------------

def test_large_body_range_and_fold():
    import zlib

    import rpc_amd
    from oracle import oracle
    data = oracle.splitmix_bytes(100_003, 9)
    for world in [1, 2, 3, 8]:
        for align in [16, 4096, 65536]:
            rs = [large_body_range(len(data), r, world, align) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == len(data)
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert all(lo % align == 0 for lo, _ in rs)
            parts = [(oracle.crc32(data[a:b]), b - a) for a, b in rs]
            assert fold_partials(parts, rpc_amd.crc32_combine) == zlib.crc32(data)
    assert fold_partials([], rpc_amd.crc32_combine) == 0


def _large_worker(rank, world, port, q, on_gpu):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        import rpc_amd
        from oracle import oracle
        length = (24 << 20) + 12345  # not a multiple of the range alignment
        lo, hi = large_body_range(length, rank, world)
        if on_gpu:
            torch.cuda.set_device(0)
            x = torch.empty((length + 7) // 8 * 8, dtype=torch.uint8, device="cuda:0")
            rpc_amd.fill_random(x, 0x5EED0006)  # every rank sees the same logical body
            mine = int(rpc_amd.device_large(x, [lo], [hi - lo]).cpu().numpy().view(np.uint32)[0])
            body = x[:length].cpu().numpy()
        else:  # CPU: the oracle stands in for the device CRC of the rank's range
            body = oracle.splitmix_bytes(length, 0x5EED0006)
            mine = oracle.crc32(body[lo:hi])
        crc = sharded_large_crc(dist, mine, hi - lo)
        allc = [None] * world
        dist.all_gather_object(allc, crc)
        if rank == 0:
            q.put((allc, oracle.crc32(body)))
    finally:
        dist.destroy_process_group()


def _run_large(world, on_gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_large_worker, args=(r, world, port, q, on_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    allc, want = q.get(timeout=110)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert allc == [want] * world


def test_gloo_world2_sharded_large_body():
    """One 24 MiB body cut into two ranges: one all_gather of (crc, len), folded with
    rpc_crc32_combine on every rank, equals the whole body's CRC."""
    _run_large(2, on_gpu=False)


@pytest.mark.gpu
def test_gloo_world2_sharded_large_body_hip():
    """The same through rpc_crc32_device_large per rank (two ranks on cuda:0)."""
    _run_large(2, on_gpu=True)


# ---- the "nccl" (RCCL) backend on hardware -----------------------------------
# RCCL refuses two ranks on one GPU, and a gpurun box has one, so this runs one
# rank: the communicator is created on cuda:0 and every collective bench.py and
# sharded_large_crc issue runs through RCCL on device tensors.

def _rccl_worker(port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        import rpc_amd
        from oracle import oracle
        out = {"backend": dist.get_backend(), "barrier": barrier(dist, dev),
               "max": max_over_ranks(dist, 2.5, dev), "sum": sum_over_ranks(dist, 1 << 40, dev)}
        length = (5 << 20) + 333
        x = torch.empty((length + 7) // 8 * 8, dtype=torch.uint8, device=dev)
        rpc_amd.fill_random(x, 0x5EED0007)
        lo, hi = large_body_range(length, 0, 1)
        mine = int(rpc_amd.device_large(x, [lo], [hi - lo]).cpu().numpy().view(np.uint32)[0])
        out["large"] = sharded_large_crc(dist, mine, hi - lo, device=dev)
        out["want"] = oracle.crc32(x[:length].cpu().numpy())
        q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_world1_collectives():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=110)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert out["backend"] == "nccl"
    assert out["barrier"] == 1 and out["max"] == 2.5 and out["sum"] == 1 << 40
    assert out["large"] == out["want"]
