set -o pipefail
T=${T:-r06o}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
# a fresh box's first process: one allocation, 12 consecutive timed blocks of 20
# C3 launches (~1.2 s), after a 0.5 s prewarm; then a second process likewise
for p in 1 2; do
  timeout -k 10 300 python tools/slow_mode.py --config c3 --rounds 1 --steps 20 --blocks 12 --tag proc$p >> gpurun_out/$T/slow_mode.jsonl 2> gpurun_out/$T/slow_mode_$p.err || exit 1
done
timeout -k 10 300 python tools/slow_mode.py --config ns --rounds 1 --steps 100 --blocks 12 --tag ns >> gpurun_out/$T/slow_mode.jsonl 2> gpurun_out/$T/slow_mode_ns.err || exit 1
