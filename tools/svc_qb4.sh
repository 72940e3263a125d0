#!/bin/bash
# The QB = 4 rows kernel (C1-shaped batch) beside a busy drop-in service, per library
# (head / abtest/<name>.so), then C1 A/B of the same libraries, rotated.
mkdir -p gpurun_out/r04za
for v in ${SVC_LIBS:-head s6}; do
  if [ $v = head ]; then lib=""; else lib=$PWD/abtest/$v.so; fi
  SVC_BATCH_LEN=1024 RPCCRC_LIB=$lib timeout -k 10 200 python tools/svc_coexist.py 12 116 1024 116 > gpurun_out/r04za/svc_coexist_1024_$v.log 2>&1 || exit 1
  echo "batch 1024 $v: $(grep '^{' gpurun_out/r04za/svc_coexist_1024_$v.log | tail -1)"
done
timeout -k 10 900 bash tools/ab_lib.sh r04za/ab "${SVC_LIBS:-head s6}" "c1" 3
