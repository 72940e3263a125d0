#!/bin/bash
# tools/gpu_round.sh -- the GPU-box sequence: smoke, GPU tests, bench, probe,
# rocprofv3 kernel-trace.  Each GPU step has its own time limit; after a fault,
# abort or timeout (exit >= 124 or signal) nothing further touches the GPU.
# Usage: bash tools/gpu_round.sh [tag] [steps...]   (steps: smoke tests bench probe prof pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}; shift || true
STEPS=${*:-"smoke tests bench probe prof"}
SUSTAIN=${SUSTAIN:-product,stream_nt1,qb1_pair1_nt1_abl3_d1,qb1_pair1_nt1_abl4_d1}
ABLATE=${ABLATE:-qb1_pair1_nt1_abl0_d1,qb1_pair1_nt1_abl3_d1,qb1_pair1_nt1_abl4_d1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "FATAL step $name rc=$rc; stopping"; exit $rc; fi
  if [ "${STRICT:-0}" = 1 ] && [ $rc -ne 0 ]; then echo "STRICT: step $name failed rc=$rc; stopping"; exit $rc; fi
  return $rc
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    tests_all) run tests_all 900 python -u -m pytest tests -m gpu -q -rfE --timeout 120 --timeout-method thread ;;
    tests_sel) run tests_sel 600 python -u -m pytest ${TESTS_SEL:-tests} -m gpu -q -rfE --timeout 120 --timeout-method thread ;;
    prof_cfgs)
           for c in ${PROF_CFGS:-c2}; do
             run prof_$c 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv -- \
                 python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-live-traffic || exit 1
           done ;;
    power_sweep)
           run ps_ns20 300 python bench.py --steps 20 --no-cpu-baseline --no-host-inclusive --no-live-traffic &&
           run ps_ns160 300 python bench.py --steps 160 --no-cpu-baseline --no-host-inclusive --no-live-traffic &&
           run ps_ns800 300 python bench.py --steps 800 --no-cpu-baseline --no-host-inclusive --no-live-traffic &&
           run ps_c3_3 300 python bench.py --config c3 --steps 3 --no-cpu-baseline --no-host-inclusive --no-live-traffic &&
           run ps_c3_20 300 python bench.py --config c3 --steps 20 --no-cpu-baseline --no-host-inclusive --no-live-traffic ;;
    ablate_r02)
           V=qb1_pair1_nt1_abl1024_d1,qb1_pair1_nt1_abl1028_d1,qb1_pair1_nt1_abl1027_d1,qb1_pair1_nt1_abl1025_d1,qb1_pair1_nt1_abl1026_d1,qb1_pair1_nt1_abl1056_d1,qb1_pair1_nt1_abl1059_d1
           for c in ${ABL_CFGS:-ns u3k u2k}; do run ablate_r02_$c 600 python tools/probe.py --mode ablate --rounds 3 --config $c --only $V || exit 1; done
           run lib_r02 300 python tools/probe.py --mode lib --rounds 3 ;;
    pmc_mix)
           for c in ${PMC_CFGS:-ns c2}; do
             run pmcmix1_$c 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
                 -d "$OUT/pmcmix1_$c" -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --prewarm-s 0.3 --no-cpu-baseline --no-host-inclusive --no-live-traffic || exit 1
             run pmcmix2_$c 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
                 -d "$OUT/pmcmix2_$c" -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --prewarm-s 0.3 --no-cpu-baseline --no-host-inclusive --no-live-traffic || exit 1
           done ;;
    bench_c3) run bench_c3 600 python bench.py --config c3 --no-cpu-baseline --no-host-inclusive ;;
    tests_variant) # GPU parity of an A/B build: VARIANT=<abtest name>
           RPCCRC_LIB=$PWD/abtest/${VARIANT}.so run tests_variant_$VARIANT 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rfE \
               --timeout 120 --timeout-method thread -k "dynamic or stealing or c1_ or north_star or uniform or c2_ or c4_" ;;
    ab) run ab 1200 bash tools/ab_lib.sh "$TAG/ab" "${AB_LIBS:-head}" "${AB_CFGS:-ns}" "${AB_ROUNDS:-2}" ;;
    ablate_half) run ablate_half 600 python tools/probe.py --mode ablate --rounds 3 --config u2k \
                   --only qb1_pair1_nt1_abl1024_d1,qb1_pair1_nt1_abl9216_d1,qb1_pair1_nt1_abl1027_d1 ;;
    frames_chunks)
           for k in ${FRAMES_CHUNKS:-4080 8176 16368}; do
             RPCCRC_BIG_CHUNK=$k run frames_chunk$k 300 python tools/frames_lifted.py 3 || exit 1
           done ;;
    frames_ab) # interleaved: route-all span mode on (1) / off (0, aligned 8 KiB chunks)
           for i in 1 2; do
             for v in 1 0; do
               RPCCRC_BIG_SPAN=$v run frames_span${v}_$i 300 python tools/frames_lifted.py 2 || exit 1
             done
           done ;;
    frames_round_ab) # interleaved, order rotated: span-pass round values on (1) / off (0)
           for i in 1 2 3; do
             if [ $((i % 2)) = 1 ]; then order="1 0"; else order="0 1"; fi
             for v in $order; do
               RPCCRC_ROUND_COMBINE=$v run frames_round${v}_$i 300 python tools/frames_lifted.py 2 || exit 1
             done
           done ;;
    frames_libs) # lifted-cap frames probe per library (A/B, order rotated): FRAMES_LIBS="head name ..."
           read -r -a FL <<< "${FRAMES_LIBS:-head}"
           for i in 1 2 3; do
             for j in $(seq 0 $((${#FL[@]} - 1))); do
               l=${FL[$(( (j + i - 1) % ${#FL[@]} ))]}
               if [ "$l" = head ]; then lib=""; else lib=$PWD/abtest/$l.so; fi
               RPCCRC_LIB=$lib run frames_${l}_$i 300 python tools/frames_lifted.py 2 || exit 1
             done
           done ;;
    prof_frames) run prof_frames 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_frames" -o run --output-format csv -- \
                   python3 tools/frames_lifted.py 3 ;;
    ragged) run ragged_${RAGGED_CFG:-c2} 300 python tools/probe.py --mode ragged --config ${RAGGED_CFG:-c2} --rounds ${RAGGED_ROUNDS:-3} --reps 5 ;;
    bench_scalar) run bench_scalar 300 tools/scalar_bench oracle/_ref/libref_crc.so ;;
    bench) run bench 600 python bench.py ;;
    probe) run probe 600 python tools/probe.py ;;
    ablate) run ablate 600 python tools/probe.py --mode ablate --rounds 3 ;;
    ablate_nat) run ablate_nat 600 python tools/probe.py --mode ablate --rounds 3 --only $ABLATE ;;
    sustain) run sustain 600 python tools/probe.py --mode sustain --launches 1500 --smi-out $OUT/smi.jsonl --only $SUSTAIN ;;
    ablate_c1) run ablate_c1 600 python tools/probe.py --mode ablate --rounds 3 --config c1 --only qb4_pair1_nt1_abl0_d1,qb4_pair1_nt1_abl3_d1,qb4_pair1_nt1_abl4_d1,qb4_pair1_nt1_abl0_d2 ;;
    bench_c1) run bench_c1 600 python bench.py --config c1 --no-cpu-baseline --no-host-inclusive ;;
    bench_c2) run bench_c2 600 python bench.py --config c2 --no-cpu-baseline --no-host-inclusive ;;
    bench_c2_rows) run bench_c2_rows 600 python bench.py --config c2 --ragged-path rows --no-cpu-baseline --no-host-inclusive --no-live-traffic ;;
    timeline) run timeline 300 python tools/probe.py --mode timeline --reps 3 ;;
    slowcap) # the slow mode: the lease's first processes, clocks read before and after
           rocm-smi --showclocks --showtemp --showpower > "$OUT/smi_before.txt" 2>&1
           run tl_c3_first 300 python tools/probe.py --mode timeline --reps 3 --config c3 --steal || exit 1
           run tl_c3_second 300 python tools/probe.py --mode timeline --reps 3 --config c3 --steal || exit 1
           run slow_c3_ns 300 python tools/slow_mode.py --config c3 --rounds 2 --blocks 3 --steps 20 --tag c3 || exit 1
           rocm-smi --showclocks --showtemp --showpower > "$OUT/smi_after.txt" 2>&1 ;;
    slowwrap) # the same 32 GiB read per launch over a 32 GiB vs a 4 GiB buffer (ragged rows kernel), rotated
           for wv in 32 4 4 32; do
             run tl_wrap${wv}_$RANDOM 300 python tools/probe.py --mode timeline --reps 6 --config c3 --steal --wrap-gib $wv || exit 1
           done ;;
    firstproc) # the lease's first processes: the same north-star line three times, then C3 twice
           for k in 1 2 3; do
             run fp_ns_$k 300 python bench.py --no-cpu-baseline --no-host-inclusive --no-live-traffic --no-scalar-latency || exit 1
           done
           for k in 1 2; do
             run fp_c3_$k 300 python bench.py --config c3 --no-cpu-baseline --no-host-inclusive --no-live-traffic --no-scalar-latency || exit 1
           done ;;
    survey) # one box: every config's bench line (no PMC / CPU legs) and the steady-state NS clock
           for c in ns c1 c2 c3 c4; do
             run survey_$c 300 python bench.py --config $c --no-cpu-baseline --no-host-inclusive --no-live-traffic --no-scalar-latency || exit 1
           done
           run survey_tl_ns 300 python tools/probe.py --mode timeline --reps 4 --config ns --steal --surround-ms 60 || exit 1 ;;
    slowss) # the shader clock in steady state: each timed launch inside 60 ms of back-to-back steps
           run tl_ns_ss 300 python tools/probe.py --mode timeline --reps 5 --config ns --steal --surround-ms 60 || exit 1
           run tl_c3_ss 300 python tools/probe.py --mode timeline --reps 5 --config c3 --steal --surround-ms 60 || exit 1
           run tl_c1_ss 300 python tools/probe.py --mode timeline --reps 5 --config c1 --steal --surround-ms 60 || exit 1
           run tl_ns_ss2 300 python tools/probe.py --mode timeline --reps 5 --config ns --steal --surround-ms 60 || exit 1 ;;
    slowclk) # per-wave shader clock beside the launch times (s_memtime / s_memrealtime)
           run tl_c3_clk 300 python tools/probe.py --mode timeline --reps 8 --config c3 --steal || exit 1
           run tl_ns_clk 300 python tools/probe.py --mode timeline --reps 8 --config ns --steal || exit 1
           run tl_c3_clk2 300 python tools/probe.py --mode timeline --reps 8 --config c3 --steal || exit 1 ;;
    timeline_c1) run timeline_c1 300 python tools/probe.py --mode timeline --reps 3 --config c1 ;;
    timeline_steal) run timeline_steal_ns 300 python tools/probe.py --mode timeline --reps 3 --steal &&
                    run timeline_steal_c1 300 python tools/probe.py --mode timeline --reps 3 --config c1 --steal ;;
    ablate_mem) run ablate_mem 600 python tools/probe.py --mode ablate --rounds 3 --only qb1_pair1_nt1_abl0_d1,qb1_pair1_nt1_abl3_d1,qb1_pair1_nt1_abl19_d1,qb1_pair1_nt1_abl259_d1,qb1_pair1_nt1_abl275_d1 ;;
    ablate_g) run ablate_g 600 python tools/probe.py --mode ablate --rounds 3 --only qb1_pair1_nt1_abl0_d1,qb1_pair1_nt1_abl0_d1_g1,qb1_pair1_nt1_abl0_d1_g2,qb1_pair1_nt1_abl0_d1_g3,qb1_pair1_nt1_abl0_d1_g4,qb1_pair1_nt1_abl0_d1_g5,qb1_pair1_nt1_abl3_d1,qb1_pair1_nt1_abl3_d1_g5,qb1_pair1_nt1_abl19_d1_g5 ;;
    ablate_g_c1) run ablate_g_c1 600 python tools/probe.py --mode ablate --rounds 3 --config c1 --only qb4_pair1_nt1_abl0_d1,qb4_pair1_nt1_abl0_d1_g1,qb4_pair1_nt1_abl0_d1_g2,qb4_pair1_nt1_abl0_d1_g3,qb4_pair1_nt1_abl0_d1_g4,qb4_pair1_nt1_abl0_d1_g5 ;;
    timeline_g5) run timeline_g5 300 python tools/probe.py --mode timeline --reps 2 --gshift 5 --save $OUT/tl_g5 ;;
    timeline_save) run timeline_save 300 python tools/probe.py --mode timeline --reps 2 --save $OUT/tl_g0 ;;
    ablate_dyn) run ablate_dyn 600 python tools/probe.py --mode ablate --rounds 3 --only qb1_pair1_nt1_abl0_d1,qb1_pair1_nt1_abl0_d1_g3,qb1_pair1_nt1_abl1024_d1,qb1_pair1_nt1_abl3_d1,qb1_pair1_nt1_abl1027_d1,qb1_pair1_nt1_abl19_d1,qb1_pair1_nt1_abl1043_d1 ;;
    timeline_dyn) run timeline_dyn 300 python tools/probe.py --mode timeline --reps 2 --dyn --save $OUT/tl_dyn ;;
    packed_slice)
           for m in 32 128 512; do
             RPCCRC_PACKED_MIN_SLICE=$m run packed_s$m 300 python tools/probe.py --mode packed --rounds 3 --reps 5 --shapes 4096x1M,1024x1M,c2 --paths packed || exit 1
           done ;;
    packed_slice_small)
           for m in 8 16; do
             RPCCRC_PACKED_MIN_SLICE=$m run packed_s$m 300 python tools/probe.py --mode packed --rounds 3 --reps 5 --shapes 4096x1M,1024x1M,c2 --paths rows,packed || exit 1
           done ;;
    pmcpacked)
           run pmcpacked 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
               -d "$OUT/pmcpacked" -o run --output-format csv -- python3 tools/probe.py --mode packed --rounds 1 --reps 2 --shapes 4096x1M,1024x1M ;;
    c4_chunks)
           for k in ${C4_CHUNKS:-0 1024 256 64 32}; do
             run c4_chunk$k 300 python bench.py --config c4 --chunk-kib $k --no-cpu-baseline --no-host-inclusive --no-live-traffic --steps 10 || exit 1
           done ;;
    prof_c4)
           for k in ${C4_PROF_CHUNKS:-1024 64}; do
             run prof_c4_$k 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof_c4_$k" -o run --output-format csv -- \
               python3 bench.py --config c4 --chunk-kib $k --steps 10 --warmup 3 --prewarm-s 0.2 --no-cpu-baseline --no-host-inclusive --no-live-traffic || exit 1
           done ;;
    packed) run packed 600 python tools/probe.py --mode packed --rounds 3 --reps 5 ;;
    bench_c4) run bench_c4 600 python bench.py --config c4 --no-cpu-baseline --no-host-inclusive ;;
    counters) run counters 120 rocprofv3 -L ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
               python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-live-traffic ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
               python3 bench.py --steps 3 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-host-inclusive --no-live-traffic &&
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
               python3 bench.py --steps 3 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-host-inclusive --no-live-traffic ;;
    pmc_cfgs)
           for c in ${PMC_CFGS:-c1 c2 c4}; do
             run pmc_fetch_$c 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$c" -o run --output-format csv -- \
                 python3 bench.py --config $c --steps 3 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-host-inclusive --no-live-traffic || exit 1
             run pmc_write_$c 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$c" -o run --output-format csv -- \
                 python3 bench.py --config $c --steps 3 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-host-inclusive --no-live-traffic || exit 1
           done ;;
    pmcprobe)
           V=qb1_pair1_nt1_abl0_d1,qb1_pair1_nt1_abl6_d1,qb1_pair1_nt1_abl4_d1,qb1_pair1_nt1_abl0_d2
           run pmcprobe1 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
               -d "$OUT/pmcprobe1" -o run --output-format csv -- python3 tools/probe.py --mode ablate --rounds 1 --reps 2 --only $V &&
           run pmcprobe2 600 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
               -d "$OUT/pmcprobe2" -o run --output-format csv -- python3 tools/probe.py --mode ablate --rounds 1 --reps 2 --only $V ;;
    *) python3 -c "print('unknown step $s')";;
  esac
done
echo done
