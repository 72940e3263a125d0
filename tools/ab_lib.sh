#!/bin/bash
# tools/ab_lib.sh -- interleaved A/B of librpccrc builds on one box.
# Usage: bash tools/ab_lib.sh TAG "libA libB ..." "cfg1 cfg2 ..." [rounds]
# lib "head" = the in-tree library; other names = abtest/<name>.so; a lib may
# carry environment settings after a colon, commas for spaces: head:RPCCRC_X=0
# cfg may carry bench flags after a colon, commas for spaces: c4:--chunk-kib,4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; LIBS=$2; CFGS=$3; ROUNDS=${4:-2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
# the library order rotates by one each round (a run's position in a round
# shifts its result: the first run after a config switch ran slowest, r04k)
read -r -a LIBARR <<< "$LIBS"
NL=${#LIBARR[@]}
for i in $(seq 1 "$ROUNDS"); do
  for c in $CFGS; do
    for j in $(seq 0 $((NL - 1))); do
      l=${LIBARR[$(( (j + i - 1) % NL ))]}
      lib=${l%%:*}; envs=""; [ "$lib" != "$l" ] && envs=$(echo "${l#*:}" | tr ',' ' ')
      if [ "$lib" = head ]; then unset RPCCRC_LIB; else export RPCCRC_LIB=$PWD/abtest/$lib.so; fi
      cfg=${c%%:*}; extra=""; [ "$cfg" != "$c" ] && extra=$(echo "${c#*:}" | tr ',' ' ')
      tag=$(echo "$c" | tr -c 'a-zA-Z0-9_\n' '_'); ltag=$(echo "$l" | tr -c 'a-zA-Z0-9_\n' '_')
      timeout -k 10 300 env $envs python bench.py --config "$cfg" $extra --no-cpu-baseline --no-host-inclusive --no-live-traffic > "$OUT/${tag}_${ltag}_$i.log" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "FAIL $c $l rc=$rc"; tail -3 "$OUT/${tag}_${ltag}_$i.log"; [ $rc -ge 124 ] && exit $rc; continue; fi
      python3 - "$OUT/${tag}_${ltag}_$i.log" "$c" "$l" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[2], sys.argv[3], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
PY
    done
  done
done | tee "$OUT/ab.txt"
