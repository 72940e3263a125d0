#!/bin/bash
# Fold A/B under rocprof (per-kernel durations of the dense C2 step), libraries
# rotated: FOLD_LIBS="head foldold" (abtest/<name>.so; head = in-tree).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${T:-r06w}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dense or c2_full" --timeout 120 --timeout-method thread > $OUT/tests_dense.log 2>&1 || { tail -5 $OUT/tests_dense.log; exit 1; }
tail -1 $OUT/tests_dense.log
read -r -a L <<< "${FOLD_LIBS:-head foldold}"
for i in 1 2; do
  for j in $(seq 0 $((${#L[@]} - 1))); do
    l=${L[$(( (j + i - 1) % ${#L[@]} ))]}
    if [ "$l" = head ]; then unset RPCCRC_LIB; else export RPCCRC_LIB=$PWD/abtest/$l.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_${l}_$i -o run --output-format csv -- \
      python3 bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-live-traffic > $OUT/prof_${l}_$i.log 2>&1 || exit 1
    python3 tools/c2_step_profile.py $OUT/prof_${l}_$i/run_kernel_trace.csv $OUT/c2_step_${l}_$i | sed "s/^/$l $i: /"
  done
done
