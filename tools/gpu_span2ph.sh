#!/bin/bash
# Dense span pass in two phases (abtest/span2ph.so, RPCCRC_SPAN_TWO_PHASE=1) vs
# the in-tree one-loop build: dense / C2 parity tests on the variant, then C2
# rotated (bench, 3 rounds), then rocprof of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${T:-r06sp}; OUT=gpurun_out/$T; mkdir -p $OUT
RPCCRC_LIB=$PWD/abtest/span2ph.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dense or c2_full" \
  --timeout 120 --timeout-method thread > $OUT/tests_span2ph.log 2>&1 || { tail -8 $OUT/tests_span2ph.log; exit 1; }
tail -1 $OUT/tests_span2ph.log
timeout -k 10 900 bash tools/ab_lib.sh $T/ab "head span2ph" "c2" 3 || exit 1
for l in head span2ph; do
  if [ "$l" = head ]; then unset RPCCRC_LIB; else export RPCCRC_LIB=$PWD/abtest/$l.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$l -o run --output-format csv -- \
    python3 bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-live-traffic > $OUT/prof_$l.log 2>&1 || exit 1
  python3 tools/c2_step_profile.py $OUT/prof_$l/run_kernel_trace.csv $OUT/c2_step_$l | sed "s/^/$l: /"
done
