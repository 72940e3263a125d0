#!/usr/bin/env python3
"""tools/c2_step_profile.py -- the C2 product step from a rocprofv3 kernel trace
(a C2 summary whose rows are the product's kernels alone).

A dense-mode C2 step is five dispatches in stream order:
dense_plan_kernel, dense_decide_kernel, the ragged rows pass (exits at once:
the batch is dense), the span pass (crc32_rows_kernel<..., 131072, ...>) and
dense_fold_kernel.  Every such sequence in the trace is one step; the bench's
other launches (stream-read probe, per-rank CRC check, unbounded calls) are
not.  Writes <out>.csv (per kernel: steps, mean / median / min us) and prints
the step's wall time (plan start -> fold end) beside the sum of its kernels.

  python tools/c2_step_profile.py gpurun_out/<tag>/prof_c2/run_kernel_trace.csv profiles/<tag>/c2_step
"""
import csv
import statistics
import sys

SEQ = ["dense_plan_kernel", "dense_decide_kernel", "crc32_rows_kernel<1, true, true, 0,",
       "crc32_rows_kernel<1, true, false, 131072,", "dense_fold_kernel"]
LABEL = ["plan", "decide", "rows pass (skipped)", "span pass", "fold"]


def main():
    src, out = sys.argv[1], sys.argv[2]
    rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
    steps = []
    i = 0
    while i + len(SEQ) <= len(rows):
        if all(SEQ[k] in rows[i + k]["Kernel_Name"] for k in range(len(SEQ))):
            steps.append(rows[i:i + len(SEQ)])
            i += len(SEQ)
        else:
            i += 1
    if not steps:
        sys.exit("no dense C2 step in the trace")
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per = [[dur(s[k]) for s in steps] for k in range(len(SEQ))]
    wall = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3 for s in steps]
    with open(out + ".csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "role", "steps", "mean_us", "median_us", "min_us"])
        for k in range(len(SEQ)):
            w.writerow([SEQ[k].rstrip(","), LABEL[k], len(steps), round(statistics.mean(per[k]), 2),
                        round(statistics.median(per[k]), 2), round(min(per[k]), 2)])
        w.writerow(["(step wall time: plan start -> fold end)", "step", len(steps), round(statistics.mean(wall), 2),
                    round(statistics.median(wall), 2), round(min(wall), 2)])
    ksum = sum(statistics.median(p) for p in per)
    print(f"{len(steps)} steps; median per kernel: " +
          ", ".join(f"{LABEL[k]} {statistics.median(per[k]):.1f}" for k in range(len(SEQ))) +
          f"; sum {ksum:.1f} us; step wall {statistics.median(wall):.1f} us (gaps {statistics.median(wall) - ksum:.1f})")


if __name__ == "__main__":
    main()
