#!/usr/bin/env python3
"""tools/c2_align.py -- does C2 pay for 128-B lines shared by neighbouring rows?

C2's bodies lie back to back at byte granularity, and the rows kernel cuts a
body into 4 KiB rows aligned to the body's 16-B-rounded END, so row boundaries
inside a body split 128-B lines (read once by each row, a step apart).  This
probe lays C2's body lengths (BASELINE configs[2], seed 0x5EED0004) out with each body's end rounded up to A bytes (A = 1: the bench layout; 16,
64, 128: padding between bodies) and times rpc_crc32_device_batch_bounded on
each layout (random bytes), interleaved, order rotated per round.  Algorithmic bytes are the
same in every layout (sum of lengths + 16 B of metadata per body).

  python tools/c2_align.py [--aligns 1,16,64,128] [--rounds 3] [--reps 10] [--only A]
--only A runs one layout a few times (a rocprofv3 --pmc pass per layout).
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


def layout(lens, align, start_align=False):
    n = lens.shape[0]
    offs = np.empty(n, dtype=np.uint64)
    pos = 0
    L = lens.astype(np.int64)
    if align <= 1:
        offs[:] = np.concatenate([[0], np.cumsum(L[:-1])]).astype(np.uint64)
        return offs, int(L.sum())
    # vectorised: each body's end rounded up to `align`; body i starts where the
    # previous (padded) one ended
    if start_align:
        padded = (L + align - 1) // align * align
        offs[:] = np.concatenate([[0], np.cumsum(padded[:-1])]).astype(np.uint64)
        return offs, int(padded.sum())
    for i in range(n):  # end alignment depends on the running position
        e = (pos + int(L[i]) + align - 1) // align * align
        offs[i] = e - int(L[i])
        pos = e
    return offs, pos


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--aligns", default="1,16,64,128")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", type=int, default=0)
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--abl", type=int, default=-1,
                    help="time tools/libprobe.so's ragged rows kernel with these ablation bits instead of the "
                         "product (65536: the product's pipeline with an XOR fold -- memory + control only)")
    ap.add_argument("--uniform4k", action="store_true", help="also a layout of 4 KiB bodies (same bytes) as a ragged batch")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lens = _loguniform_lengths(a.n, 0x5EED0004)
    aligns = [a.only] if a.only else [int(x) for x in a.aligns.split(",")]
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    lays = {}
    algo = int(lens.sum(dtype=np.uint64)) + 16 * a.n
    for A in aligns:  # each layout filled with its own random bytes (timing only)
        offs, total = layout(lens, A)
        buf = torch.empty((total + 4096 + 15) // 8 * 8, dtype=torch.uint8, device=dev)
        rpc_amd.fill_random(buf, 0x5EED0004 + A)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        out = torch.empty(a.n, dtype=torch.int32, device=dev)
        lays[A] = (buf, d_offs, out, total)
        print(f"c2_align: layout {A}: {total} B", file=sys.stderr, flush=True)
    torch.cuda.synchronize()

    if a.uniform4k:  # the same byte count cut into 4 KiB bodies, 4 KiB-aligned, passed as a ragged batch
        n4 = int(lens.sum(dtype=np.uint64)) // 4096
        buf = torch.empty(n4 * 4096, dtype=torch.uint8, device=dev)
        rpc_amd.fill_random(buf, 0x5EED0404)
        o4 = torch.from_numpy((np.arange(n4, dtype=np.uint64) * np.uint64(4096)).view(np.int64)).to(dev)
        l4 = torch.full((n4,), 4096, dtype=torch.int32, device=dev)
        lays[4096] = (buf, o4, torch.empty(n4, dtype=torch.int32, device=dev), n4 * 4096, l4)
        aligns.append(4096)
    probe = None
    if a.abl >= 0:
        import ctypes
        probe = ctypes.CDLL(os.path.join(REPO, "tools", "libprobe.so"))
        probe.probe_rows_ragged.restype = ctypes.c_int
        probe.probe_rows_ragged.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

    def step(A):
        buf, d_offs, out, _ = lays[A][:4]
        dl = lays[A][4] if len(lays[A]) > 4 else d_lens
        if probe is not None:
            rc = probe.probe_rows_ragged(buf.data_ptr(), d_offs.data_ptr(), dl.data_ptr(), d_offs.numel(),
                                         out.data_ptr(), a.abl, 256, torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc
        else:
            rpc_amd.device_batch(buf, d_offs, dl, out=out, max_len=65536)

    if a.only:
        for _ in range(a.reps):
            step(a.only)
        torch.cuda.synchronize()
        print(json.dumps({"only": a.only, "reps": a.reps}), flush=True)
        return
    s = torch.cuda.current_stream()
    res = {A: [] for A in aligns}
    for r in range(a.rounds):
        order = aligns[r % len(aligns):] + aligns[: r % len(aligns)]
        for A in order:
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                step(A)
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                step(A)
            e1.record(s)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            res[A].append(us)
            print(f"c2_align: round {r} align {A}: {us:.1f} us frac {algo / us / 8e6:.4f}", file=sys.stderr, flush=True)
    summary = {str(A): {"us": [round(x, 1) for x in v], "min_us": round(min(v), 1),
                        "frac_best": round(algo / min(v) / 8e6, 4), "span_bytes": lays[A][3]}
               for A, v in res.items()}
    print(json.dumps({"algo_bytes": algo, "abl": a.abl, "layouts": summary}), flush=True)


if __name__ == "__main__":
    main()
