#!/bin/bash
# C4 round-value combine A/B (RPCCRC_ROUND_COMBINE 1 / 0), run order rotated.
# Prints config, knob, average launch (us, rows kernel + combine per call) and roofline fraction.
mkdir -p gpurun_out
for r in 1 2 3; do
  if [ $((r % 2)) = 1 ]; then order="1 0"; else order="0 1"; fi
  for v in $order; do
    RPCCRC_ROUND_COMBINE=$v timeout -k 10 150 python bench.py --config c4 --steps 30 --no-cpu-baseline --no-host-inclusive --no-live-traffic > gpurun_out/c4ab_tmp.log 2>&1 || exit 1
    grep '^{' gpurun_out/c4ab_tmp.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c4 round', '$v', d['ms_per_step'], r['avg_launch_us'], r['frac'])"
  done
done
