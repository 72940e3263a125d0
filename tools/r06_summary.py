"""Summarise a round-6 GPU pass (gpurun_out/<tag>): bench lines and kernel stats."""
import csv, glob, json, os, sys
t = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{t}/bench_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); r = d["roofline"]
            print(os.path.basename(f), d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"], r.get("frac_of_stream_read"), d.get("ranks_crc_ok"))
p = f"gpurun_out/{t}/prof_c2/run_kernel_stats.csv"
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["MinNs"]) / 1e3, 1))
