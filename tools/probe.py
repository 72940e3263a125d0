#!/usr/bin/env python3
"""tools/probe.py -- one-process A/B timing of kernel variants on one GPU
(interleaved rounds, median; cdna_hip_programming.md 5.4 rule 24).

  python tools/probe.py [--config ns] [--rounds 5] [--reps 10]
Prints one JSON line per variant: stream-read patterns and CRC kernel options.
"""
import argparse
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import rpc_amd  # noqa: E402
from bench import Workload  # noqa: E402


def timed(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ns")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--grids", default="0,512,1024")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    w = Workload(a.config, 0, torch.device("cuda", 0))
    nbytes = (w.total // 4096) * 4096
    variants = {}
    for pat in (0, 1):
        for nt in (0, 1):
            variants[f"stream_read_p{pat}_nt{nt}"] = (lambda pat=pat, nt=nt: rpc_amd.stream_read(
                w.base, pat, bool(nt), nbytes=nbytes), nbytes, None)
    for nt in (0, 1):
        for g in [int(x) for x in a.grids.split(",")]:
            variants[f"crc_nt{nt}_grid{g}"] = (w.step, w.algo_bytes, (nt, g))
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, (fn, nb, opt) in variants.items():
            if opt is not None:
                rpc_amd.set_options(nontemporal=bool(opt[0]), max_blocks=opt[1])
            res[k].append(timed(fn, a.reps))
            rpc_amd.set_options(False, 0)
    for k, ts in res.items():
        med = statistics.median(ts)
        nb = variants[k][1]
        print(json.dumps({"variant": k, "config": a.config, "median_us": round(med * 1e6, 2),
                          "min_us": round(min(ts) * 1e6, 2), "GBps": round(nb / med / 1e9, 1),
                          "frac_of_8TBps": round(nb / med / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
