#!/usr/bin/env python3
"""tools/slow_mode.py -- where does the stealing kernels' slow mode live
(some processes ran every C3 launch ~4 % slower)?

One process, several fresh workloads in turn: each allocates and fills its own
buffer, is prewarmed like the bench (0.5 s), then times K launches with HIP
events around the block (no marker between launches), and the previous
workload is freed before the next.  If the slow mode follows the allocation
(the physical placement of the buffer), workloads of one process differ; if it
follows the process (or the box's first use), only the first process is slow
and all its workloads alike.

  python tools/slow_mode.py [--config c3] [--rounds 3] [--steps 20] [--tag NAME]
"""
import argparse
import json
import os
import sys
import time

import torch

T0 = time.perf_counter()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import Workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--tag", default="")
    ap.add_argument("--prewarm-s", type=float, default=0.5)
    ap.add_argument("--blocks", type=int, default=1, help="consecutive timed blocks per round (a ramp shows as a trend)")
    ap.add_argument("--stride-kib", type=int, default=0,
                    help="uniform configs: bodies this far apart (the same bytes over a wider address range)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    for r in range(a.rounds):
        t_alloc = time.perf_counter()
        w = Workload(a.config, 0, dev)
        if a.stride_kib and w.kind == "uniform":  # the same bodies, spread: base i * stride
            import rpc_amd
            stride = a.stride_kib * 1024
            big = torch.empty(w.n * stride, dtype=torch.uint8, device=dev)
            rpc_amd.fill_random(big, 0x51DE)
            w.base = big
            w.step = lambda w=w, stride=stride: rpc_amd.device_uniform(w.base, w.n, w.L, stride=stride, out=w.out)
        torch.cuda.synchronize()
        t_alloc = time.perf_counter() - t_alloc
        t0 = time.perf_counter()
        n_pw = 0
        while time.perf_counter() - t0 < a.prewarm_s:
            w.step()
            torch.cuda.synchronize()
            n_pw += 1
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.blocks + 1)]
        ev[0].record(s)
        for b in range(a.blocks):
            for _ in range(a.steps):
                w.step()
            ev[b + 1].record(s)
        ev[-1].synchronize()
        us = [ev[b].elapsed_time(ev[b + 1]) * 1e3 / a.steps for b in range(a.blocks)]
        ptr = w.base.data_ptr() if hasattr(w, "base") else 0
        print(json.dumps({"tag": a.tag, "pid": os.getpid(), "config": a.config, "stride_kib": a.stride_kib, "round": r,
                          "us_per_launch": [round(x, 1) for x in us],
                          "frac": [round(w.algo_bytes / (x * 1e-6) / 8e12, 4) for x in us], "prewarm_launches": n_pw,
                          "since_start_s": round(time.perf_counter() - T0, 2),
                          "alloc_fill_s": round(t_alloc, 2), "base_ptr": hex(ptr)}), flush=True)
        del w
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
