#!/usr/bin/env python3
"""tools/frames_lifted.py [rounds] -- bench.py's extra.frames_lifted probe alone
(1024 LIFT_CAP frames, bodies log-uniform 1 B - 64 MiB, stamp + verify on the
device), repeated; one JSON line per round (A/B of route settings, e.g.
RPCCRC_BIG_MIN)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

bench._load_gpu_modules()
import torch  # noqa: E402

dev = torch.device("cuda:0")
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    r = bench.frames_lifted_probe(dev)
    r["big_min"] = os.environ.get("RPCCRC_BIG_MIN", "default")
    r["big_aligned"] = os.environ.get("RPCCRC_BIG_ALIGNED", "default")
    r["big_chunk"] = os.environ.get("RPCCRC_BIG_CHUNK", "default")
    r["big_span"] = os.environ.get("RPCCRC_BIG_SPAN", "default")
    r["round_combine"] = os.environ.get("RPCCRC_ROUND_COMBINE", "default")
    print(json.dumps(r), flush=True)
