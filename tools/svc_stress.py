#!/usr/bin/env python3
"""tools/svc_stress.py -- the drop-in service under a long multi-thread stress:
T threads x N back-to-back rpc_crc32 calls of 0..240 B (around the 116-B inline
bound), each body different from the slot's previous one, every CRC against the
oracle.  Prints one JSON line with the call count and the wrong CRCs.

  python tools/svc_stress.py [--threads 10] [--calls 30000]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import rpc_amd  # noqa: E402
from oracle import oracle  # noqa: E402  (the checker)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=10)
    ap.add_argument("--calls", type=int, default=30000)
    a = ap.parse_args()
    pool = np.random.default_rng(17).integers(0, 256, 1 << 16, dtype=np.uint8).tobytes()
    errors, counts = [], [0] * a.threads

    def worker(k):
        r = np.random.default_rng(1000 + k)
        for _ in range(a.calls):
            L = int(r.integers(0, 241))
            o = int(r.integers(0, len(pool) - L))
            b = pool[o:o + L]
            if rpc_amd.rpc_crc32(b) != oracle.crc32(np.frombuffer(b, dtype=np.uint8)):
                errors.append((k, L))
            counts[k] += 1

    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(k,)) for k in range(a.threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    print(json.dumps({"threads": a.threads, "calls": sum(counts), "wrong": len(errors), "first": errors[:10],
                      "seconds": round(time.perf_counter() - t0, 1)}), flush=True)
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main())
