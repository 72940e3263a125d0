set -o pipefail
T=${T:-r06k}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
# the box's first processes first (the slow mode hit first processes)
for p in 1 2; do
  timeout -k 10 300 python tools/slow_mode.py --config c3 --rounds 3 --steps 20 --tag proc$p >> gpurun_out/$T/slow_mode.jsonl 2> gpurun_out/$T/slow_mode_$p.err || exit 1
done
bash tools/gpu_r06b.sh
