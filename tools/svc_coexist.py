"""Drop-in service beside the rows kernel: median per-launch time of a
256K x 4 KiB uniform batch alone and while one thread keeps the drop-in service
busy with bodies of a given length (RPCCRC_LIB selects the library).
Usage: python tools/svc_coexist.py LEN [LEN ...]"""
import json
import os
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, ".")
import rpc_amd  # noqa: E402

DEV = "cuda:0"
n, L = 1 << 18, 4096
if os.environ.get("SVC_BATCH_LEN") == "1024":  # the QB = 4 rows kernel (the largest LDS): 1M x 1 KiB
    n, L = 1 << 20, 1024
if os.environ.get("SVC_MAXBLOCKS"):  # persistent-grid cap (a placement test)
    rpc_amd.set_options(True, int(os.environ["SVC_MAXBLOCKS"]))
x = torch.empty(n * L, dtype=torch.uint8, device=DEV)
rpc_amd.fill_random(x, 0x5E7)


def timed(reps=20):
    s = torch.cuda.current_stream()
    for _ in range(6):
        rpc_amd.device_uniform(x, n, L)
    ev = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        rpc_amd.device_uniform(x, n, L)
        e1.record(s)
        ev.append((e0, e1))
    ev[-1][1].synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3


res = {"lib": os.environ.get("RPCCRC_LIB", "") or "head", "max_blocks": os.environ.get("SVC_MAXBLOCKS", "default"), "alone_us": round(min(timed() for _ in range(3)), 1)}
for blen in [int(a) for a in sys.argv[1:]]:
    body = bytes(range(256)) * 4
    body = body[:blen]
    stop, calls = threading.Event(), [0]

    def hammer():
        while not stop.is_set():
            rpc_amd.rpc_crc32(body)
            calls[0] += 1

    th = threading.Thread(target=hammer)
    th.start()
    try:
        t = min(timed() for _ in range(3))
    finally:
        stop.set()
        th.join()
    res[f"busy_{blen}B_us"] = round(t, 1)
    res[f"calls_{blen}B"] = calls[0]
print(json.dumps(res))
