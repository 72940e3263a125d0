set -o pipefail
mkdir -p gpurun_out/r06f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rfE --timeout 180 --timeout-method thread -k "dense or c2_full" > gpurun_out/r06f/tests_dense.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/r06f/steps.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config c2 --steps 20 --no-cpu-baseline --no-host-inclusive --no-live-traffic > gpurun_out/r06f/bench_c2_dense.log 2>&1 || exit 1
true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06f/prof_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-host-inclusive --no-live-traffic > gpurun_out/r06f/prof_c2.log 2>&1 || exit 1
exit $rc
