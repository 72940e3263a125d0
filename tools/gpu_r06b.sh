set -o pipefail
T=${T:-r06g}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rfE --timeout 180 --timeout-method thread -k "${TESTK:-dense or c2_full}" > gpurun_out/$T/tests_dense.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/$T/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 bash tools/ab_lib.sh $T/ab "head head:RPCCRC_DENSE=0" "c2" ${ROUNDS:-2} > gpurun_out/$T/ab_stdout.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive --no-live-traffic > gpurun_out/$T/prof_c2.log 2>&1 || exit 1
exit $rc
