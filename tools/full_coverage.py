#!/usr/bin/env python3
"""tools/full_coverage.py -- DEBUG (GPU): every CRC of large uniform, ragged and
large-body batches against the oracle (the checker), n x 4 KiB bodies (argv[1],
default 2^18), for dealing changes whose errors a sampled test could miss (one
lost round of 32 bodies in 1M).  Note: the oracle follows zlib's 32-bit length,
so the single-body check is only meaningful below 4 GiB."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import rpc_amd  # noqa: E402
from oracle import oracle  # noqa: E402  (the checker)

dev = torch.device("cuda", 0)
n, L = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18, 4096
x = torch.empty(n * L, dtype=torch.uint8, device=dev)
rpc_amd.fill_random(x, 0x5EED0003)
host = x.cpu().numpy()
want = oracle.crc32_uniform(host, n, L)
for rep in range(3):
    got = rpc_amd.device_uniform(x, n, L).cpu().numpy().view(np.uint32)
    bad = np.flatnonzero(got != want)
    print("uniform rep", rep, "mismatches", bad.size, "first", bad[:8].tolist(), "rounds", sorted(set((bad // 32).tolist()))[:8])
lens = np.full(n, L, dtype=np.uint32)
offs = (np.arange(n, dtype=np.uint64) * L)
got = rpc_amd.device_batch(x, torch.from_numpy(offs.view(np.int64)).to(dev),
                           torch.from_numpy(lens.view(np.int32)).to(dev)).cpu().numpy().view(np.uint32)
bad = np.flatnonzero(got != want)
print("ragged mismatches", bad.size, bad[:8].tolist())
whole = int(rpc_amd.device_large(x, [0], [n * L]).cpu().numpy().view(np.uint32)[0])
print("large", hex(whole), hex(oracle.crc32(host)), whole == oracle.crc32(host))
for Lb in (16384, 8192, 12288):
    nb = n * L // Lb
    wantb = oracle.crc32_uniform(host, nb, Lb)
    lens = np.full(nb, Lb, dtype=np.uint32)
    offs = (np.arange(nb, dtype=np.uint64) * Lb)
    got = rpc_amd.device_batch(x, torch.from_numpy(offs.view(np.int64)).to(dev),
                               torch.from_numpy(lens.view(np.int32)).to(dev)).cpu().numpy().view(np.uint32)
    bad = np.flatnonzero(got != wantb)
    print("ragged", Lb, "mismatches", bad.size, bad[:8].tolist(), "rounds", sorted(set((bad // 32).tolist()))[:12])
    gotu = rpc_amd.device_uniform(x, nb, Lb).cpu().numpy().view(np.uint32)
    bad = np.flatnonzero(gotu != wantb)
    print("uniform", Lb, "mismatches", bad.size, bad[:8].tolist(), "rounds", sorted(set((bad // 32).tolist()))[:12])
