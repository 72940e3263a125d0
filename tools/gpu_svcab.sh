#!/bin/bash
# Drop-in service A/B on one box, rotated: the in-tree library (round-6 request
# check) vs abtest/scalar_bench_svc5 linked to abtest/svc5lib (round-5 check).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${T:-r06x}; OUT=gpurun_out/$T; mkdir -p $OUT
for r in 1 2 3; do
  if [ $((r % 2)) = 1 ]; then order="head svc5"; else order="svc5 head"; fi
  for v in $order; do
    if [ $v = head ]; then b=tools/scalar_bench; else b=abtest/scalar_bench_$v; fi
    timeout -k 10 120 $b oracle/_ref/libref_crc.so > $OUT/scalar_${v}_$r.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$OUT/scalar_${v}_$r.log') if l.startswith('{')][-1])
print('$v', ' '.join(f\"{x['bytes']}B/{x['threads']}t:{x['gpu_us']}\" for x in d['rows']))"
  done
done
