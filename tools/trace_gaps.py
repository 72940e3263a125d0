#!/usr/bin/env python3
"""tools/trace_gaps.py <kernel_trace.csv> [last_n] -- per-dispatch durations and the
idle gaps between consecutive dispatches (previous end -> next start) over the last
`last_n` dispatches of a rocprofv3 --kernel-trace run (e.g. tools/gpu_round.sh
prof_cfgs), grouped by kernel name: where a step's time goes besides the kernels."""
import csv
import json
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = rows[-last:]
dur, gaps = {}, []
for i, r in enumerate(rows):
    name = r["Kernel_Name"].split("(")[0][:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    dur.setdefault(name, []).append(d)
    if i:
        gaps.append((int(r["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(json.dumps({
    "dispatches": len(rows),
    "span_us": round(span, 1),
    "kernels": {k: {"n": len(v), "avg_us": round(statistics.mean(v), 2), "median_us": round(statistics.median(v), 2)}
                for k, v in dur.items()},
    "gap_us": {"avg": round(statistics.mean(gaps), 2), "median": round(statistics.median(gaps), 2),
               "min": round(min(gaps), 2), "max": round(max(gaps), 2)} if gaps else None,
}, indent=1))
