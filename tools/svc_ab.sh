#!/bin/bash
# Drop-in service A/B (in-tree library vs abtest/scalar_bench_$SVC_VARIANT linked to abtest/${SVC_VARIANT}lib, default base),
# rotated, then the service beside rows launches (NS-shaped and C1-shaped batches).
# The base side is built in this container first:
#   mkdir -p abtest/baselib && cp abtest/base.so abtest/baselib/librpccrc.so &&
#   gcc -O2 -std=c11 -D_POSIX_C_SOURCE=200809L -Iinclude -o abtest/scalar_bench_base \
#       tools/scalar_bench.c -Labtest/baselib -lrpccrc -Wl,-rpath,'$ORIGIN/baselib' -ldl -lpthread
mkdir -p gpurun_out/r04z
for r in 1 2 3; do
  V=${SVC_VARIANT:-base}
  if [ $((r % 2)) = 1 ]; then order="head $V"; else order="$V head"; fi
  for v in $order; do
    if [ $v = head ]; then b=tools/scalar_bench; else b=abtest/scalar_bench_$v; fi
    timeout -k 10 120 $b oracle/_ref/libref_crc.so > gpurun_out/r04z/scalar_${v}_$r.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r04z/scalar_${v}_$r.log') if l.startswith('{')][-1])
print('$v', ' '.join(f\"{x['bytes']}B/{x['threads']}t:{x['gpu_us']}\" for x in d['rows']))"
  done
done
for bl in 4096 1024; do
  for v in head ${SVC_VARIANT:-base}; do
    if [ $v = head ]; then lib=""; else lib=$PWD/abtest/$v.so; fi
    SVC_BATCH_LEN=$bl RPCCRC_LIB=$lib timeout -k 10 200 python tools/svc_coexist.py 12 116 1024 > gpurun_out/r04z/svc_coexist_${bl}_$v.log 2>&1 || exit 1
    echo "batch $bl $v: $(grep '^{' gpurun_out/r04z/svc_coexist_${bl}_$v.log | tail -1)"
  done
done
