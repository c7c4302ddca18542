#!/bin/bash
# Round-4: background spawn-ahead (k_spawn) at 20x20 with the table encode, on/off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04f}
mkdir -p $OUT
i=0
for c in cfg3 cfg4 cfg2; do
  for bg in 0 1 0 1; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 1000 --warmup 200 --spawn-background $bg > $OUT/$i.log 2>&1 || { echo "fail $c $bg"; tail -5 $OUT/$i.log; exit 3; }
    echo "$c bg=$bg $(tail -1 $OUT/$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead'))")"
  done
done
echo all-ok
