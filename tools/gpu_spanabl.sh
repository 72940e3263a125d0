#!/bin/bash
# Span-pass ablations under rocprof (kernel medians of the dense C2 step),
# libraries rotated: SPAN_LIBS (abtest/<name>.so; head = in-tree).  The
# ablations give wrong CRCs by design (timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${T:-r06sa}; OUT=gpurun_out/$T; mkdir -p $OUT
read -r -a L <<< "${SPAN_LIBS:-head spanabl1 spanabl2}"
for i in 1 2; do
  for j in $(seq 0 $((${#L[@]} - 1))); do
    l=${L[$(( (j + i - 1) % ${#L[@]} ))]}
    if [ "$l" = head ]; then unset RPCCRC_LIB; else export RPCCRC_LIB=$PWD/abtest/$l.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_${l}_$i -o run --output-format csv -- \
      python3 bench.py --config ${SPAN_CFG:-c2} --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-live-traffic > $OUT/prof_${l}_$i.log 2>&1
    python3 tools/c2_step_profile.py $OUT/prof_${l}_$i/run_kernel_trace.csv $OUT/c2_step_${l}_$i | sed "s/^/$l $i: /"
  done
done
unset RPCCRC_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run --output-format csv -- \
  python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-live-traffic > $OUT/prof_c3.log 2>&1
python3 - $OUT/prof_c3/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "crc32_rows_kernel<1, true, false, 0," in r["Name"]:
        print("c3 rows kernel avg", round(float(r["AverageNs"]) / 1e3, 1), "min", round(float(r["MinNs"]) / 1e3, 1), "calls", r["Calls"])
PY
