#!/usr/bin/env python3
"""tools/small_batch.py -- the split path on frames-like batches (SURVEY.md 8f
row 1): n rpc.h bodies of 1 B - 1 KiB (MAX_BODY_LEN, rpc.h:17) behind 16-byte
headers, back to back, CRC'd by rpc_crc32_device_batch through the split path
(lists, then the small-body kernel / the rows kernel's QB = 4 loop for bodies
whose end-padded length fits 1 KiB, QB = 1 for the rest).  Every CRC is checked
against the oracle on a sample.  RPCCRC_SMALL_KERNEL=0 selects the QB = 4 loop.

  python tools/small_batch.py [--n 1048576] [--reps 10] [--rounds 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0x5EED0010)
    lens = rng.integers(1, 1025, a.n).astype(np.uint32)
    offs = np.cumsum(np.concatenate([[16], (lens[:-1].astype(np.uint64) + 16)]), dtype=np.uint64)
    total = int(offs[-1] + lens[-1]) + 16
    base = torch.empty((total + 7) // 8 * 8, dtype=torch.uint8, device=dev)
    rpc_amd.fill_random(base, 0x5EED0010)
    d_o = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_l = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = torch.empty(a.n, dtype=torch.int32, device=dev)
    rpc_amd.set_ragged_path("split")
    s = torch.cuda.current_stream()
    res = []
    for r in range(a.rounds):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            rpc_amd.device_batch(base, d_o, d_l, out=out, max_len=1024)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            rpc_amd.device_batch(base, d_o, d_l, out=out, max_len=1024)
        e1.record(s)
        e1.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / a.reps)
        print(f"small_batch: {res[-1]:.1f} us", file=sys.stderr, flush=True)
    rpc_amd.set_ragged_path("auto")
    # oracle check on a sample (test infrastructure: the checker, not the measured path)
    from oracle import oracle  # noqa: E402
    host = base.cpu().numpy()
    got = out.cpu().numpy().view(np.uint32)
    idx = rng.choice(a.n, 4096, replace=False)
    bad = sum(int(got[i]) != oracle.crc32(host[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()) for i in idx)
    print(json.dumps({"n": a.n, "small_kernel": os.environ.get("RPCCRC_SMALL_KERNEL", "1"),
                      "us": [round(x, 1) for x in res], "min_us": round(min(res), 1),
                      "frames_per_s": round(a.n / (min(res) * 1e-6)), "sample_mismatches": bad}), flush=True)


if __name__ == "__main__":
    main()
