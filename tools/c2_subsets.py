#!/usr/bin/env python3
"""tools/c2_subsets.py -- what C2's small bodies cost inside the product launch.

The C2 batch (BASELINE configs[2]: 4M bodies, log-uniform 64 B - 64 KiB, back to
back) and two sub-batches over the SAME buffer: only the bodies whose end-padded
length exceeds 1 KiB (their rows as in the full batch), and only the small ones.
Times rpc_crc32_device_batch_bounded on each, interleaved, order rotated.  If the
full batch costs about the large bodies' time plus their bytes' share, the small
bodies' 1.6M one-row steps are hidden; if it costs the sum, they are not.

  python tools/c2_subsets.py [--rounds 3] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import rpc_amd  # noqa: E402
from bench import _loguniform_lengths  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = 1 << 22
    lens = _loguniform_lengths(n, 0x5EED0004)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(lens.sum(dtype=np.uint64))
    base = torch.empty((total + 15) // 8 * 8, dtype=torch.uint8, device=dev)
    rpc_amd.fill_random(base, 0x5EED0004)
    z = (-(offs + lens.astype(np.uint64))) & np.uint64(15)  # buffer base is 256-B aligned
    small = lens.astype(np.uint64) + z <= np.uint64(1024)
    sets = {"all": np.ones(n, dtype=bool), "large": ~small, "small": small}
    dv = {}
    for k, m in sets.items():
        o, l = offs[m], lens[m]
        dv[k] = (torch.from_numpy(o.view(np.int64)).to(dev), torch.from_numpy(l.view(np.int32)).to(dev),
                 torch.empty(int(m.sum()), dtype=torch.int32, device=dev), int(m.sum()),
                 int(l.sum(dtype=np.uint64)))
    s = torch.cuda.current_stream()

    def step(k):
        o, l, out, _, _ = dv[k]
        rpc_amd.device_batch(base, o, l, out=out, max_len=65536)

    res = {k: [] for k in sets}
    names = list(sets)
    for r in range(a.rounds):
        for k in names[r % 3:] + names[:r % 3]:
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                step(k)
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                step(k)
            e1.record(s)
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3 / a.reps)
            print(f"c2_subsets: {k} {res[k][-1]:.1f} us", file=sys.stderr, flush=True)
    print(json.dumps({k: {"bodies": dv[k][3], "bytes": dv[k][4], "us": [round(x, 1) for x in v],
                          "min_us": round(min(v), 1)} for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
