#!/bin/bash
# Round 4: cost of the main stream's wait on the background spawn kernel
# (diagnostic SNAKE_BG_NOWAIT build of that time: the wait dropped, timing only;
# the product has since dropped the wait for a device-side gate).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04t}
mkdir -p $OUT
i=0
for c in cfg5 cfg2; do
  bg=0; [ $c = cfg2 ] && bg=1
  for l in base nowait base nowait; do
    i=$((i+1))
    SNAKE_LIB=marl-snake_amd/build/var/libsnake_$l.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 2000 --warmup 200 --spawn-background $bg > $OUT/$i.log 2>&1 || { echo "fail $c $l"; tail -5 $OUT/$i.log; exit 3; }
    echo "$c $l bg=$bg $(tail -1 $OUT/$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead',{}).get('hit_rate'))")"
  done
done
echo all-ok
