set -o pipefail
T=${T:-r06p}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/$T/pmc_fold -o run --output-format csv -- python3 bench.py --config c2 --steps 3 --warmup 1 --prewarm-s 0.3 --no-cpu-baseline --no-host-inclusive --no-live-traffic > gpurun_out/$T/pmc_fold.log 2>&1
