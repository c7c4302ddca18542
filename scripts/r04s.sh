#!/bin/bash
# Round 4: background spawn-ahead (k_spawn on the state's side stream) against
# the in-step attempts on the small and mid-size 20x20 configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r04s}
mkdir -p $OUT
i=0
for c in ${CONFIGS:-cfg2 cfg4 cfg3}; do
  for bg in ${BGS:--1 1 -1 1}; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 2000 --warmup 200 --spawn-background $bg > $OUT/$i.log 2>&1 || { echo "fail $c $bg"; tail -5 $OUT/$i.log; exit 3; }
    echo "$c bg=$bg $(tail -1 $OUT/$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels'], d.get('spawn_ahead'))")"
  done
done
echo all-ok
