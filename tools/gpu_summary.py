#!/usr/bin/env python3
"""tools/gpu_summary.py <tag> -- one-screen summary of a tools/gpu_round.sh run
merged back under gpurun_out/<tag>/ (steps, test tail, bench lines, probes)."""
import glob
import json
import os
import sys

tag = sys.argv[1]
d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", tag)
if not os.path.isdir(d):
    sys.exit(f"no {d}")


def lines(name):
    p = os.path.join(d, name)
    return open(p).read().splitlines() if os.path.exists(p) else []


for l in lines("steps.log"):
    if "rc=" in l:
        print(l)
for l in lines("tests.log")[-2:]:
    print("tests:", l)
for f in sorted(glob.glob(os.path.join(d, "bench*.log"))):
    ls = [l for l in lines(os.path.basename(f)) if l.startswith("{")]
    if not ls:
        print(os.path.basename(f), "(no JSON line)")
        continue
    j = json.loads(ls[-1])
    r = j["roofline"]
    cpu = j.get("cpu_baseline") or {}
    print(f"{os.path.basename(f):14s} value={j['value']:8.1f} {j['unit']} us/launch={r['avg_launch_us']:9.1f} "
          f"frac={r['frac']:.4f} traffic={r.get('traffic')} cpu={cpu.get('value')} extra={j.get('extra')}")
for name in ("probe.log", "ablate.log", "ablate_nat.log", "ablate_c1.log", "ablate_mem.log", "ablate_g.log",
             "ablate_g_c1.log", "ablate_dyn.log"):
    for l in lines(name):
        if l.startswith("{"):
            j = json.loads(l)
            print(f"{name:14s} {j['variant']:28s} {j['config']:4s} {j['median_us']:9.2f} us  {j['GBps']:8.1f} GB/s")
for name in ("timeline.log", "timeline_c1.log", "timeline_g5.log", "timeline_save.log", "timeline_dyn.log"):
    for l in lines(name):
        if l.startswith("{"):
            print(name, l)
for l in lines("packed.log"):
    if l.startswith("{"):
        print("packed", l)
for l in lines("sustain.log"):
    if l.startswith('{"variant"'):
        j = json.loads(l)
        print(f"sustain {j['variant']:28s} first10={j['first10_us']:8.1f} last_q={j['last_quarter_us']:8.1f} "
              f"min={j['min_us']:8.1f} GB/s={j['mean_GBps']}")
smi = [json.loads(l) for l in lines("sustain.log") if l.startswith('{"smi_t_s"')]
if smi:
    print("smi (t, mean gfx MHz, W):", [(s["smi_t_s"], round(sum(s["gfx_mhz"]) / max(1, len(s["gfx_mhz"]))),
                                        s["power_w"][:1]) for s in smi[::3]])
