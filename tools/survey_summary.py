#!/usr/bin/env python3
"""tools/survey_summary.py -- one line per box from `gpu_round.sh <tag> survey`
passes: every config's launch time and frac, and the north star's steady-state
shader clock (median over the timed launches after the first).

  python tools/survey_summary.py gpurun_out/r06s1 [gpurun_out/r06s2 ...]
"""
import json
import os
import statistics
import sys

for d in sys.argv[1:]:
    cells = []
    for c in ("ns", "c1", "c2", "c3", "c4"):
        p = os.path.join(d, f"survey_{c}.log")
        line = [ln for ln in open(p) if ln.startswith('{"metric"')][-1] if os.path.exists(p) else None
        if line:
            r = json.loads(line)["roofline"]
            cells.append(f"{c} {r['avg_launch_us']:.1f} us {r['frac']:.3f}")
    p = os.path.join(d, "survey_tl_ns.log")
    if os.path.exists(p):
        tl = [json.loads(ln) for ln in open(p) if ln.startswith('{"mode"')][1:]
        if tl:
            cells.append("ns steady %.0f us @ %.0f MHz" % (statistics.median(t["exit_us"][1] for t in tl),
                                                          statistics.median(t["shader_clock_mhz_p0_50_100"][1] for t in tl)))
    print(os.path.basename(d.rstrip("/")), "; ".join(cells))
