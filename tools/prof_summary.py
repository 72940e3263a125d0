#!/usr/bin/env python3
"""tools/prof_summary.py <run_dir> <out.json> -- condense a `rocprofv3 --kernel-trace
--stats` run of bench.py (tools/gpu_round.sh step `prof`) into the record
committed under profiles/: per-kernel stats, the average duration of the timed
launches (the last `steps` dispatches of the CRC kernel) and the bench line's own
HIP-event average, which must agree."""
import csv
import glob
import json
import os
import sys

run, out = sys.argv[1], sys.argv[2]
stats = list(csv.DictReader(open(glob.glob(os.path.join(run, "prof", "*kernel_stats.csv"))[0])))
trace = list(csv.DictReader(open(glob.glob(os.path.join(run, "prof", "*kernel_trace.csv"))[0])))
bench = [l for l in open(os.path.join(run, "prof.log")) if l.startswith('{"metric"')]
line = json.loads(bench[-1]) if bench else None
steps = line["steps"] if line else 20
crc = [r for r in trace if "rows_kernel" in r["Kernel_Name"]]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in crc]
rec = {
    "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 20 --warmup 3 "
               "--no-cpu-baseline --no-host-inclusive",
    "kernel_stats": [{k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
                     for r in stats],
    "crc_kernel": crc[0]["Kernel_Name"] if crc else None,
    "crc_dispatches": len(dur),
    "timed_launches_avg_us": round(sum(dur[-steps:]) / steps, 2) if dur else None,
    "bench_avg_launch_us": line["roofline"]["avg_launch_us"] if line else None,
    "bench_line": line,
    "resources": {k: crc[0].get(k) for k in ("VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Scratch_Size",
                                               "Workgroup_Size_X", "Grid_Size_X")} if crc else None,
}
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps({k: rec[k] for k in ("crc_kernel", "crc_dispatches", "timed_launches_avg_us",
                                      "bench_avg_launch_us")}))
