#!/usr/bin/env python3
"""tools/launch_series.py -- per-launch durations of one config's product call,
an event after every launch (each adds a marker between launches), after a
clock prewarm: do some launches stall (a protocol wait that resolves late)
while the rest run at speed?

  python tools/launch_series.py [--config c3] [--steps 40]
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
from bench import Workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    w = Workload(a.config, 0, torch.device("cuda", 0))
    s = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        w.step()
        torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    ev[0].record(s)
    for i in range(a.steps):
        w.step()
        ev[i + 1].record(s)
    ev[-1].synchronize()
    us = np.array([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(a.steps)])
    print(json.dumps({"config": a.config, "lib": os.environ.get("RPCCRC_LIB", "") or "head",
                      "mean_us": round(float(us.mean()), 1), "median_us": round(float(np.median(us)), 1),
                      "min_us": round(float(us.min()), 1), "max_us": round(float(us.max()), 1),
                      "us": [round(float(x), 1) for x in us]}), flush=True)


if __name__ == "__main__":
    main()
