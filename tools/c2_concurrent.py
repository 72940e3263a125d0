#!/usr/bin/env python3
"""tools/c2_concurrent.py -- can C2's small bodies run beside the large ones?

The C2 batch (BASELINE configs[2]) split host-side into its large bodies (end-
padded length > 1 KiB) and its small ones, over the same buffer.  Times, on one
box, interleaved and order rotated:
  all        -- the product launch over the whole batch (256 workgroups)
  split      -- the whole batch through the split path (lists, small bodies
                four per row, the rest one body per row sequence), one stream
  large@G    -- the large bodies alone on G workgroups (G of the 256 CUs)
  small@G    -- the small bodies alone (split path: four per QB = 4 row) on G
  conc@G     -- large@(256 - G) on one stream and small@G on a second, both
                enqueued before either runs; time = first start to last end
The persistent rows kernels take one CU per workgroup (~160 KiB LDS), so the two
launches of conc occupy disjoint CUs.  If conc@G ~ large@(256 - G) < all, the
small bodies' ~400 us row steps can hide behind the large bodies' HBM stream.

  python tools/c2_concurrent.py [--rounds 3] [--reps 5] [--gs 8,16,32]
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
    ap.add_argument("--gs", default="8,16,32")
    a = ap.parse_args()
    gs = [int(x) for x in a.gs.split(",")]
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
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
                 torch.empty(int(m.sum()), dtype=torch.int32, device=dev))
    ref = {}
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream(dev)

    def launch(k, g, stream, path="auto"):
        o, l, out = dv[k]
        rpc_amd.set_options(max_blocks=g)
        # the small bodies through the split path: all of them four per row
        rpc_amd.set_ragged_path("split" if k == "small" else path)
        rpc_amd.device_batch(base, o, l, out=out, stream=stream, max_len=1024 if k == "small" else 65536)
        rpc_amd.set_ragged_path("auto")

    def step(case):
        kind, g = case
        if kind == "all":
            launch("all", cus, s1)
        elif kind == "split":  # the whole batch through the split path, one stream
            launch("all", cus, s1, "split")
        elif kind in ("large", "small"):
            launch(kind, g, s1)
        else:  # conc: small first on s2 (after s1's prior work), then large on s1
            s2.wait_stream(s1)
            launch("small", g, s2)
            launch("large", cus - g, s1)
            s1.wait_stream(s2)

    cases = [("all", cus), ("split", cus), ("small", cus)]
    for g in gs:
        cases += [("large", cus - g), ("small", g), ("conc", g)]
    res = {f"{k}@{g}": [] for k, g in cases}
    for r in range(a.rounds):
        order = cases[r % len(cases):] + cases[:r % len(cases)]
        for case in order:
            name = f"{case[0]}@{case[1]}"
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                step(case)
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s1)
            for _ in range(a.reps):
                step(case)
            e1.record(s1)
            e1.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / a.reps)
            print(f"c2_concurrent: {name} {res[name][-1]:.1f} us", file=sys.stderr, flush=True)
            if case[0] in ("all", "conc", "split"):  # every CRC the same as the whole-batch launch's
                got = torch.empty(n, dtype=torch.int32, device=dev)
                if case[0] in ("all", "split"):
                    got = dv["all"][2].clone()
                else:
                    got[torch.from_numpy(np.flatnonzero(small)).to(dev)] = dv["small"][2]
                    got[torch.from_numpy(np.flatnonzero(~small)).to(dev)] = dv["large"][2]
                if "all" in ref:
                    assert torch.equal(got, ref["all"]), f"{name}: CRCs differ from the whole-batch launch"
                else:
                    ref["all"] = got
    rpc_amd.set_options(max_blocks=0)
    print(json.dumps({k: {"us": [round(x, 1) for x in v], "min_us": round(min(v), 1)} for k, v in res.items()}),
          flush=True)


if __name__ == "__main__":
    main()
