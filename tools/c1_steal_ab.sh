for r in 1 2 3; do
  for v in "0.15 head" "0.08 head" "0.25 head" "0.15 early"; do set -- $v
    if [ $2 = head ]; then l=""; else l=$PWD/abtest/$2.so; fi
    RPCCRC_LIB=$l RPCCRC_STEAL_FRAC=$1 timeout -k 10 120 python bench.py --config c1 --steps 50 --no-cpu-baseline --no-host-inclusive --no-live-traffic > gpurun_out/c1ab_tmp.log 2>&1 || exit 1
    grep '^{' gpurun_out/c1ab_tmp.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c1', '$1', '$2', r['avg_launch_us'], r['frac'])"
  done
done
