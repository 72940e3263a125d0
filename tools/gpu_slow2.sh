set -o pipefail
T=${T:-r06q}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
S="timeout -k 10 300 python tools/slow_mode.py --rounds 1 --blocks 6"
$S --config ns --steps 100 --tag ns4k >> gpurun_out/$T/slow_mode.jsonl 2>> gpurun_out/$T/slow.err || exit 1
$S --config ns --steps 100 --stride-kib 32 --tag ns32k >> gpurun_out/$T/slow_mode.jsonl 2>> gpurun_out/$T/slow.err || exit 1
$S --config c3 --steps 20 --tag c3 >> gpurun_out/$T/slow_mode.jsonl 2>> gpurun_out/$T/slow.err || exit 1
$S --config ns --steps 100 --tag ns4k_again >> gpurun_out/$T/slow_mode.jsonl 2>> gpurun_out/$T/slow.err || exit 1
