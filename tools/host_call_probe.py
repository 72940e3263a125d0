"""Host-side cost of back-to-back batched calls: the enqueue time of K calls
(host clock, no sync) against their GPU time (sync after).  A call that blocks
the host (a pool wait) shows an enqueue time close to the GPU time.
Usage: python tools/host_call_probe.py"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import rpc_amd  # noqa: E402

DEV = "cuda:0"
K = 40
x = torch.empty(1 << 32, dtype=torch.uint8, device=DEV)
rpc_amd.fill_random(x, 0x77)
L = 256 << 20
offs, lens = [i * L for i in range(16)], [L] * 16
out_u = torch.empty(1 << 20, dtype=torch.int32, device=DEV)
out_l = torch.empty(16, dtype=torch.int32, device=DEV)
cases = {
    "ns_uniform": lambda: rpc_amd.device_uniform(x, 1 << 20, 4096, out=out_u),
    "c4_large": lambda: rpc_amd.device_large(x, offs, lens, out=out_l),
}
res = {}
for name, fn in cases.items():
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    res[name] = {"enqueue_us_per_call": round((t1 - t0) / K * 1e6, 1), "total_us_per_call": round((t2 - t0) / K * 1e6, 1)}
print(json.dumps(res))
