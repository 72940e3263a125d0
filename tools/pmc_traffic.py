#!/usr/bin/env python3
"""tools/pmc_traffic.py -- HBM bytes per launch of the CRC kernel from rocprofv3
PMC passes (MI355X_MICROARCH.md "HBM [CDNA4]"):

  * FETCH_SIZE and WRITE_SIZE are collected in SEPARATE rocprofv3 passes
    (tools/gpu_round.sh step `pmc`), each with --kernel-trace-free --pmc runs.
  * Both are reported in KiB (x 1024 -> bytes).
  * gfx950: FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane)
    coalesced streaming read -> doubled here.  WRITE_SIZE is exact for the
    16 B/lane stores it was calibrated on; our output writes are 4 B/lane
    (uncalibrated, and < 0.1 % of the traffic), reported as measured.

Usage: python tools/pmc_traffic.py <pmc_fetch_dir> <pmc_write_dir> <config> [--out profiles/traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_dispatch(d, counter, kernel_sub="rows_kernel"):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or kernel_sub not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for *{kernel_sub}* in {d}")
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("config")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "profiles", "traffic.json"))
    ap.add_argument("--algo-bytes", type=float, default=None)
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch_dir, "FETCH_SIZE")
    write = per_dispatch(a.write_dir, "WRITE_SIZE")
    fetch_kib = statistics.median(fetch)
    write_kib = statistics.median(write)
    hbm = 2.0 * fetch_kib * 1024 + write_kib * 1024
    rec = {
        "hbm_bytes_per_launch": hbm,
        "fetch_size_kib_median": fetch_kib,
        "write_size_kib_median": write_kib,
        "dispatches": {"fetch": len(fetch), "write": len(write)},
        "correction": "hbm = 2 * FETCH_SIZE * 1024 (gfx950 halves wide streaming reads) + WRITE_SIZE * 1024",
    }
    if a.algo_bytes:
        rec["algo_bytes_per_launch"] = a.algo_bytes
        rec["traffic_over_algo"] = hbm / a.algo_bytes
    data = {}
    if os.path.exists(a.out):
        data = json.load(open(a.out))
    data[a.config] = rec
    json.dump(data, open(a.out, "w"), indent=1)
    print(json.dumps({a.config: rec}))


if __name__ == "__main__":
    main()
