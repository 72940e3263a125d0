#!/usr/bin/env python3
"""tools/pmc_mix.py -- per-launch PMC counters of the rows kernel (median over
dispatches) from rocprofv3 --pmc CSV directories; divides by a row count.
Usage: python tools/pmc_mix.py <rows_per_launch> <dir> [<dir> ...]
(PMC_KERNEL=<name substring> selects another kernel.)"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    rows = float(sys.argv[1])
    out = {}
    for d in sys.argv[2:]:
        per = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if os.environ.get("PMC_KERNEL", "crc32_rows_kernel") not in r["Kernel_Name"]:
                    continue
                per.setdefault(r["Counter_Name"], {}).setdefault((f, r["Dispatch_Id"]), 0.0)
                per[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
        for k, v in per.items():
            # the same kernel also runs tiny launches (e.g. the big-body route's
            # chunk pass with no chunks): keep the dispatches of the main launch
            vals = sorted(v.values())
            big = [x for x in vals if x >= 0.5 * vals[-1]] or vals
            med = statistics.median(big)
            out[k] = {"per_launch": med, "per_row": round(med / rows, 2), "dispatches": len(v)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
